// Training-step kernels around the GEMMs (gemm_f16x3.hip): the loss of LitNeRF.training_step
// (model.py:256-282, helper.py:17-18), the backward of volumetric_rendering (helper.py:157-195)
// with the rgb / sigma activations (model.py:186-187), bias-gradient column sums and the Adam
// update of configure_optimizers / optimizer_step (model.py:386-419).
#include "aon_common.hpp"

#include <cmath>

namespace aon {

constexpr int kBwdWaves = 4;

__device__ __forceinline__ void wave_sync_t() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// d act(x) / dx from the raw value (reference activations, model.py:186-187 and
// model_autodecoder.py:321-323)
__device__ __forceinline__ float dact_rgb(float x, int act) {
  if (act == AON_ACT_NONE) return 1.0f;
  const float s = __fdiv_rn(1.0f, __fadd_rn(1.0f, exp_sleef(-x)));
  const float d = __fmul_rn(s, __fsub_rn(1.0f, s));
  return act == AON_ACT_ARTIC ? __fmul_rn(d, 1.002f) : d;
}

__device__ __forceinline__ float dact_sigma(float x, int act) {
  if (act == AON_ACT_NONE) return 1.0f;
  if (act == AON_ACT_VANILLA) return x > 0.0f ? 1.0f : 0.0f;
  // softplus(z)' with threshold 20, as torch's CPU softplus_backward forms it: e/(e + 1)
  // with e = exp(z) (SLEEF)
  const float z = __fsub_rn(x, 1.0f);
  if (z > 20.0f) return 1.0f;
  const float e = exp_sleef(z);
  return __fdiv_rn(e, __fadd_rn(e, 1.0f));
}

// Backward of volumetric_rendering for one ray per wave.  With f_j = 1 - alpha_j + 1e-10,
// T_i = prod_{j<i} f_j, w_i = alpha_i T_i and q_i = dL/dw_i = g.(c_i - white) + g_acc + g_depth t_i:
//   dL/dc_i     = g w_i
//   dL/dalpha_i = T_i (q_i - R_{i+1}),  R_i = alpha_i q_i + f_i R_{i+1},  R_S = 0
// (the suffix recurrence replaces the division by f_i of a cumprod backward), then
// dalpha/dsigma = exp(-sigma D) D with D = dist * |d| (dist_last = 1e10).  R is an affine
// suffix scan per 64-sample block (6 shuffle steps, fp64) carried from the last block down.
template <int NB>
__global__ __launch_bounds__(64 * kBwdWaves) void k_composite_bwd(
    const float* __restrict__ rgb, int64_t rgb_stride, const float* __restrict__ sig,
    int64_t sig_stride, const float* __restrict__ tv, const float* __restrict__ dirs, int64_t B,
    int S, int white, int act, const float* __restrict__ g_rgb, const float* __restrict__ g_acc,
    const float* __restrict__ g_depth, float* __restrict__ d_rgb, float* __restrict__ d_sig,
    int64_t d_stride) {
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = (int64_t)gridDim.x * kBwdWaves;
  for (int64_t ray = (int64_t)blockIdx.x * kBwdWaves + (threadIdx.x >> 6); ray < B;
       ray += nwaves) {
    const int64_t row0 = ray * S;
    const float dx = dirs[3 * ray], dy = dirs[3 * ray + 1], dz = dirs[3 * ray + 2];
    const float dnorm = sqrtf(fmaf(dz, dz, fmaf(dy, dy, __fmul_rn(dx, dx))));
    const float g0 = g_rgb[3 * ray], g1 = g_rgb[3 * ray + 1], g2 = g_rgb[3 * ray + 2];
    const float ga = g_acc ? g_acc[ray] : 0.0f, gd = g_depth ? g_depth[ray] : 0.0f;
    const float wb = white ? 1.0f : 0.0f;
    float alpha[NB], f[NB], T[NB], q[NB], dsd[NB];
    double carry = 1.0;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int i = 64 * b + lane;
      const bool valid = i < S;
      alpha[b] = 0.f;
      f[b] = 1.f;
      q[b] = 0.f;
      dsd[b] = 0.f;
      double fi = 1.0;
      if (valid) {
        const int64_t r = row0 + i;
        const float ti = tv[r];
        const float dist = (i + 1 < S) ? __fsub_rn(tv[r + 1], ti) : 1e10f;
        const float D = __fmul_rn(dist, dnorm);
        const float sraw = sig[r * sig_stride];
        const float sgm = act_sigma(sraw, act);
        const float e = exp_cr(__fmul_rn(-sgm, D));
        const float a = __fsub_rn(1.0f, e);
        alpha[b] = a;
        if (i + 1 < S) {
          f[b] = __fadd_rn(__fsub_rn(1.0f, a), 1e-10f);
          fi = (double)f[b];
        } else {
          f[b] = 0.f;  // R of the last sample has no successor term
        }
        const float* c = rgb + r * rgb_stride;
        const float c0 = act_rgb(c[0], act), c1 = act_rgb(c[1], act), c2 = act_rgb(c[2], act);
        q[b] = __fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(g0, __fsub_rn(c0, wb)),
                                             __fmul_rn(g1, __fsub_rn(c1, wb))),
                                   __fadd_rn(__fmul_rn(g2, __fsub_rn(c2, wb)), ga)),
                         __fmul_rn(gd, ti));
        dsd[b] = __fmul_rn(__fmul_rn(e, D), dact_sigma(sraw, act));
      }
      // exclusive prefix product (forward scan of the compositor)
      double incl = fi;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const double v = __shfl_up(incl, o);
        if (lane >= o) incl *= v;
      }
      double excl = __shfl_up(incl, 1);
      if (lane == 0) excl = 1.0;
      T[b] = (float)(carry * excl);
      carry *= __shfl(incl, 63);
    }
    double Rc = 0.0;  // R at the first sample of the block after the current one
#pragma unroll
    for (int b = NB - 1; b >= 0; --b) {
      const int i = 64 * b + lane;
      const bool valid = i < S;
      // (A, Bv): R_i = Bv + A * R_{end of block}
      double A = valid ? (double)f[b] : 1.0;
      double Bv = valid ? (double)alpha[b] * (double)q[b] : 0.0;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const double Ao = __shfl_down(A, o), Bo = __shfl_down(Bv, o);
        if (lane + o < 64) {
          Bv = Bv + A * Bo;
          A = A * Ao;
        }
      }
      const double R = Bv + A * Rc;       // R_i
      double Rn = __shfl_down(R, 1);      // R_{i+1}
      if (lane == 63) Rn = Rc;
      Rc = __shfl(R, 0);
      if (valid) {
        const int64_t r = row0 + i;
        const float w = __fmul_rn(alpha[b], T[b]);
        const float da = __fmul_rn(T[b], (float)((double)q[b] - Rn));
        const float* c = rgb + r * rgb_stride;
        float* o = d_rgb + r * d_stride;
        o[0] = __fmul_rn(__fmul_rn(g0, w), dact_rgb(c[0], act));
        o[1] = __fmul_rn(__fmul_rn(g1, w), dact_rgb(c[1], act));
        o[2] = __fmul_rn(__fmul_rn(g2, w), dact_rgb(c[2], act));
        d_sig[r * d_stride] = __fmul_rn(da, dsd[b]);
      }
    }
  }
}

// loss = mean((pred - target)^2) over n values, grad = scale * 2 (pred - target) / n
// (helper.py:17-18; `scale` folds dL/dloss).  One workgroup; loss accumulated in fp64.
__global__ __launch_bounds__(256) void k_mse(const float* __restrict__ pred,
                                             const float* __restrict__ target, int64_t n,
                                             float scale, float* __restrict__ loss,
                                             float* __restrict__ grad) {
  __shared__ double part[256];
  double s = 0.0;
  const float gscale = __fdiv_rn(2.0f * scale, (float)n);
  // 8 strided elements' loads in flight per thread before the in-order fp64 accumulation (a
  // single workgroup: the loop was one dependent load round trip per element, ~20 us per call)
  constexpr int kU = 8;
  for (int64_t i0 = threadIdx.x; i0 < n; i0 += 256 * kU) {
    float p[kU], q[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t i = i0 + 256 * u;
      p[u] = i < n ? pred[i] : 0.f;
      q[u] = i < n ? target[i] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t i = i0 + 256 * u;
      if (i < n) {
        const float d = __fsub_rn(p[u], q[u]);
        s += (double)d * (double)d;
        if (grad) grad[i] = __fmul_rn(gscale, d);
      }
    }
  }
  part[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) part[threadIdx.x] += part[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0 && loss) *loss = (float)(part[0] / (double)n);
}

// The training step's loss terms in one launch (model.py:265-270 / model_autodecoder.py:455-470):
// the two levels' img2mse against one target -- each with k_mse's arithmetic (the same per-thread
// element order, fp64 accumulation, reduction tree and rounding), the loads of both levels in
// flight together -- then loss = (loss1 + loss0) (+ extra): one launch for 2 k_mse launches and
// the add.  (mse2psnr stays torch's own log / mul / div, on both losses at once: torch's device
// log is not correctly rounded, tools/diag/psnr_ulp.py, so a restatement would sit 1 ulp off.)
__global__ __launch_bounds__(256) void k_loss_pair(const float* __restrict__ pred0,
                                                   const float* __restrict__ pred1,
                                                   const float* __restrict__ target, int64_t n,
                                                   const float* __restrict__ extra,
                                                   float* __restrict__ out, float* __restrict__ grad0,
                                                   float* __restrict__ grad1) {
  __shared__ double part[2][256];
  double s0 = 0.0, s1 = 0.0;
  const float gscale = __fdiv_rn(2.0f, (float)n);
  constexpr int kU = 8;
  for (int64_t i0 = threadIdx.x; i0 < n; i0 += 256 * kU) {
    float p0[kU], p1[kU], q[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t i = i0 + 256 * u;
      p0[u] = i < n ? pred0[i] : 0.f;
      p1[u] = i < n ? pred1[i] : 0.f;
      q[u] = i < n ? target[i] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t i = i0 + 256 * u;
      if (i < n) {
        const float d0 = __fsub_rn(p0[u], q[u]), d1 = __fsub_rn(p1[u], q[u]);
        s0 += (double)d0 * (double)d0;
        s1 += (double)d1 * (double)d1;
        if (grad0) grad0[i] = __fmul_rn(gscale, d0);
        if (grad1) grad1[i] = __fmul_rn(gscale, d1);
      }
    }
  }
  part[0][threadIdx.x] = s0;
  part[1][threadIdx.x] = s1;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      part[0][threadIdx.x] += part[0][threadIdx.x + o];
      part[1][threadIdx.x] += part[1][threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float l0 = (float)(part[0][0] / (double)n), l1 = (float)(part[1][0] / (double)n);
    float l = __fadd_rn(l1, l0);
    if (extra) l = __fadd_rn(l, *extra);
    out[0] = l;
    out[1] = l0;
    out[2] = l1;
  }
}

// its backward: d_i = grad_i * (g_loss + g_loss_i), absent (NULL) scalars taken as 0 -- what
// autograd forms for img2mse's `grad * g` after summing the two uses of loss_i
__global__ __launch_bounds__(256) void k_loss_pair_bwd(const float* __restrict__ grad0,
                                                       const float* __restrict__ grad1, int64_t n,
                                                       const float* __restrict__ g_loss,
                                                       const float* __restrict__ g_loss0,
                                                       const float* __restrict__ g_loss1,
                                                       float* __restrict__ d0, float* __restrict__ d1) {
  const float g = g_loss ? *g_loss : 0.f;
  const float a = g_loss0 ? (g_loss ? __fadd_rn(g, *g_loss0) : *g_loss0) : g;
  const float b = g_loss1 ? (g_loss ? __fadd_rn(g, *g_loss1) : *g_loss1) : g;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    d0[i] = __fmul_rn(grad0[i], a);
    d1[i] = __fmul_rn(grad1[i], b);
  }
}

// column sums out[n] (+)= sum_m X[m*ldx + n]: partials over row chunks, then a fixed-order sum
constexpr int kColRows = 1024;

__global__ __launch_bounds__(256) void k_colsum_part(const float* __restrict__ X, int64_t ldx,
                                                     int64_t M, int64_t N,
                                                     float* __restrict__ part) {
  // block (x: 64-column group, y: chunk of kColRows rows); 4 row phases x 64 columns
  __shared__ float red[4][64];
  const int c = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int64_t n = (int64_t)blockIdx.x * 64 + c;
  const int64_t r0 = (int64_t)blockIdx.y * kColRows;
  float s = 0.f;
  if (n < N) {
    const int64_t r1 = r0 + kColRows < M ? r0 + kColRows : M;
    for (int64_t m = r0 + ph; m < r1; m += 4) s = __fadd_rn(s, X[m * ldx + n]);
  }
  red[ph][c] = s;
  __syncthreads();
  if (ph == 0 && n < N)
    part[(int64_t)blockIdx.y * N + n] =
        __fadd_rn(__fadd_rn(__fadd_rn(red[0][c], red[1][c]), red[2][c]), red[3][c]);
}

__global__ void k_colsum_final(const float* __restrict__ part, int64_t chunks, int64_t N,
                               int accumulate, float* __restrict__ out) {
  const int64_t n = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (n >= N) return;
  float s = 0.f;
  for (int64_t z = 0; z < chunks; ++z) s = __fadd_rn(s, part[z * N + n]);
  out[n] = accumulate ? __fadd_rn(out[n], s) : s;
}

// Adam (torch.optim.Adam, no weight decay / amsgrad):
//   m = lerp(m, g, 1 - b1); v = b2 v + (1 - b2) g^2
//   p -= (lr / (1 - b1^t)) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)
struct AdamTable {
  float* p[AON_ADAM_MAX_TENSORS];
  const float* g[AON_ADAM_MAX_TENSORS];
  float* m[AON_ADAM_MAX_TENSORS];
  float* v[AON_ADAM_MAX_TENSORS];
  int64_t start[AON_ADAM_MAX_TENSORS + 1];  // prefix offsets of numel (k_adam4: of 4-element chunks)
  int64_t numel[AON_ADAM_MAX_TENSORS];
  int count;
};

struct AdamScalars {
  float step_size, one_minus_b1, b2, one_minus_b2, eps, bc2_sqrt;
};

__device__ __forceinline__ void adam_update(const AdamScalars& c, float g, float& p, float& m,
                                            float& v) {
  m = __fadd_rn(m, __fmul_rn(c.one_minus_b1, __fsub_rn(g, m)));
  v = __fadd_rn(__fmul_rn(v, c.b2), __fmul_rn(__fmul_rn(c.one_minus_b2, g), g));
  const float denom = __fadd_rn(__fdiv_rn(sqrtf(v), c.bc2_sqrt), c.eps);
  p = __fsub_rn(p, __fmul_rn(c.step_size, __fdiv_rn(m, denom)));
}

__global__ void k_adam(AdamTable t, AdamScalars c) {
  const int64_t total = t.start[t.count];
  int k = 0;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    while (e >= t.start[k + 1]) ++k;
    const int64_t i = e - t.start[k];
    float p = t.p[k][i], m = t.m[k][i], v = t.v[k][i];
    adam_update(c, t.g[k][i], p, m, v);
    t.p[k][i] = p;
    t.m[k][i] = m;
    t.v[k][i] = v;
  }
}

// The same update 4 elements per thread with 16-B loads and stores (every pointer 16-B aligned):
// t.start holds each tensor's first 4-element chunk, a tensor's last chunk runs its tail
// element by element.  One launch over ~1.2 M parameters was 28 us at one scalar element per
// thread (7 dependent 4-B accesses each, a linear search of the table per element).
__global__ void k_adam4(AdamTable t, AdamScalars c) {
  const int64_t chunks = t.start[t.count];
  int k = 0;
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < chunks;
       q += (int64_t)gridDim.x * blockDim.x) {
    while (q >= t.start[k + 1]) ++k;
    const int64_t i = 4 * (q - t.start[k]);
    const int64_t n = t.numel[k];
    if (i + 4 <= n) {
      const f4 p4 = *reinterpret_cast<const f4*>(t.p[k] + i);
      const f4 m4 = *reinterpret_cast<const f4*>(t.m[k] + i);
      const f4 v4 = *reinterpret_cast<const f4*>(t.v[k] + i);
      const f4 g4 = *reinterpret_cast<const f4*>(t.g[k] + i);
      float p[4], m[4], v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        p[u] = p4[u];
        m[u] = m4[u];
        v[u] = v4[u];
        adam_update(c, g4[u], p[u], m[u], v[u]);
      }
      *reinterpret_cast<f4*>(t.p[k] + i) = f4{p[0], p[1], p[2], p[3]};
      *reinterpret_cast<f4*>(t.m[k] + i) = f4{m[0], m[1], m[2], m[3]};
      *reinterpret_cast<f4*>(t.v[k] + i) = f4{v[0], v[1], v[2], v[3]};
    } else {
      for (int64_t e = i; e < n; ++e) {
        float p = t.p[k][e], m = t.m[k][e], v = t.v[k][e];
        adam_update(c, t.g[k][e], p, m, v);
        t.p[k][e] = p;
        t.m[k][e] = m;
        t.v[k][e] = v;
      }
    }
  }
}

}  // namespace aon

using namespace aon;

extern "C" int aon_composite_bwd(const float* rgb, int64_t rgb_stride, const float* sigma,
                                 int64_t sigma_stride, const float* t, const float* dirs,
                                 int64_t B, int S, int white_bkgd, int act, const float* g_rgb,
                                 const float* g_acc, const float* g_depth, float* d_rgb,
                                 float* d_sigma, int64_t d_stride, aon_stream_t stream) {
  AON_REQUIRE(rgb && sigma && t && dirs && g_rgb && d_rgb && d_sigma, "null pointer");
  AON_REQUIRE(B >= 0 && S >= 1 && S <= 512 && rgb_stride >= 3 && sigma_stride >= 1 && d_stride >= 1,
              "bad shape (1 <= S <= 512)");
  AON_REQUIRE(act >= AON_ACT_NONE && act <= AON_ACT_ARTIC, "bad activation");
  if (B == 0) return 0;
  const int grid = grid_for(B, kBwdWaves, 1 << 16);
  hipStream_t st = (hipStream_t)stream;
  switch ((S + 63) / 64) {
#define AON_BWD_CASE(nb)                                                                        \
  case nb:                                                                                      \
    hipLaunchKernelGGL(k_composite_bwd<nb>, grid, 64 * kBwdWaves, 0, st, rgb, rgb_stride,       \
                       sigma, sigma_stride, t, dirs, B, S, white_bkgd, act, g_rgb, g_acc,       \
                       g_depth, d_rgb, d_sigma, d_stride);                                      \
    break;
    AON_BWD_CASE(1)
    AON_BWD_CASE(2)
    AON_BWD_CASE(3)
    AON_BWD_CASE(4)
    AON_BWD_CASE(5)
    AON_BWD_CASE(6)
    AON_BWD_CASE(7)
    AON_BWD_CASE(8)
#undef AON_BWD_CASE
  }
  return launch_status(__func__);
}

extern "C" int aon_mse(const float* pred, const float* target, int64_t n, float grad_scale,
                       float* loss, float* grad, aon_stream_t stream) {
  AON_REQUIRE(pred && target && (loss || grad), "null pointer");
  AON_REQUIRE(n >= 1, "empty input");
  hipLaunchKernelGGL(k_mse, 1, 256, 0, (hipStream_t)stream, pred, target, n, grad_scale, loss, grad);
  return launch_status(__func__);
}

extern "C" int aon_loss_pair(const float* pred0, const float* pred1, const float* target,
                             int64_t n, const float* extra, float* out, float* grad0, float* grad1,
                             aon_stream_t stream) {
  AON_REQUIRE(pred0 && pred1 && target && out, "null pointer");
  AON_REQUIRE(n >= 1, "empty input");
  hipLaunchKernelGGL(k_loss_pair, 1, 256, 0, (hipStream_t)stream, pred0, pred1, target, n, extra,
                     out, grad0, grad1);
  return launch_status(__func__);
}

extern "C" int aon_loss_pair_bwd(const float* grad0, const float* grad1, int64_t n,
                                 const float* g_loss, const float* g_loss0, const float* g_loss1,
                                 float* d0, float* d1, aon_stream_t stream) {
  AON_REQUIRE(grad0 && grad1 && d0 && d1, "null pointer");
  AON_REQUIRE(n >= 0, "bad size");
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_loss_pair_bwd, grid_for(n, 256, 1024), 256, 0, (hipStream_t)stream, grad0,
                     grad1, n, g_loss, g_loss0, g_loss1, d0, d1);
  return launch_status(__func__);
}

extern "C" size_t aon_colsum_workspace_bytes(int64_t M, int64_t N) {
  return (size_t)((M + kColRows - 1) / kColRows) * (size_t)N * sizeof(float);
}

extern "C" int aon_colsum(const float* X, int64_t ldx, int64_t M, int64_t N, int accumulate,
                          float* out, void* work, size_t work_bytes, aon_stream_t stream) {
  AON_REQUIRE(X && out, "null pointer");
  AON_REQUIRE(M >= 0 && N >= 0 && ldx >= N, "bad shape");
  if (N == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const int64_t chunks = (M + kColRows - 1) / kColRows;
  if (chunks == 0) {
    if (!accumulate) {
      const hipError_t e = hipMemsetAsync(out, 0, N * sizeof(float), st);
      if (e != hipSuccess) return static_cast<int>(e);
    }
    return 0;
  }
  AON_REQUIRE(work && work_bytes >= aon_colsum_workspace_bytes(M, N),
              "needs aon_colsum_workspace_bytes() of workspace");
  AON_REQUIRE(chunks < 65536, "too many rows");
  hipLaunchKernelGGL(k_colsum_part, dim3((unsigned)((N + 63) / 64), (unsigned)chunks), 256, 0, st,
                     X, ldx, M, N, static_cast<float*>(work));
  hipLaunchKernelGGL(k_colsum_final, grid_for(N, 256), 256, 0, st,
                     static_cast<const float*>(work), chunks, N, accumulate, out);
  return launch_status(__func__);
}

extern "C" int aon_adam_step(const aon_adam_tensor* tensors, int count, double lr, double beta1,
                             double beta2, double eps, int64_t step, aon_stream_t stream) {
  AON_REQUIRE(tensors && count >= 1 && count <= AON_ADAM_MAX_TENSORS, "bad tensor list");
  AON_REQUIRE(step >= 1, "step counts from 1");
  AdamTable t;
  t.count = count;
  t.start[0] = 0;
  for (int i = 0; i < count; ++i) {
    AON_REQUIRE(tensors[i].param && tensors[i].grad && tensors[i].exp_avg && tensors[i].exp_avg_sq &&
                    tensors[i].numel >= 0,
                "null tensor");
    t.p[i] = tensors[i].param;
    t.g[i] = tensors[i].grad;
    t.m[i] = tensors[i].exp_avg;
    t.v[i] = tensors[i].exp_avg_sq;
    t.start[i + 1] = t.start[i] + tensors[i].numel;
    t.numel[i] = tensors[i].numel;
  }
  if (t.start[count] == 0) return 0;
  bool vec = true;  // every tensor 16-B aligned: k_adam4
  for (int i = 0; i < count; ++i)
    vec = vec && aligned16(t.p[i]) && aligned16(t.g[i]) && aligned16(t.m[i]) && aligned16(t.v[i]);
  // Every scalar is formed in double from the Python-float hyperparameters, as torch.optim.Adam
  // does (lerp weight 1 - beta1, addcmul value 1 - beta2, step size lr / bc1, sqrt(bc2)), and
  // only then rounded to fp32 where it meets the fp32 tensors.
  const double bc1 = 1.0 - std::pow(beta1, (double)step);
  const double bc2 = 1.0 - std::pow(beta2, (double)step);
  const AdamScalars c{(float)(lr / bc1), (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2),
                      (float)eps, (float)std::sqrt(bc2)};
  if (vec) {
    for (int i = 0; i < count; ++i) t.start[i + 1] = t.start[i] + (t.numel[i] + 3) / 4;
    hipLaunchKernelGGL(k_adam4, grid_for(t.start[count], 256, 4096), 256, 0, (hipStream_t)stream, t, c);
  } else {
    hipLaunchKernelGGL(k_adam, grid_for(t.start[count], 256, 4096), 256, 0, (hipStream_t)stream, t, c);
  }
  return launch_status(__func__);
}
