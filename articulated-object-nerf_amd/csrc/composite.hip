// Alpha compositing (reference models/vanilla_nerf/helper.py:157-195) -- HBM-bound.
//
// One 64-lane wave per ray; lane i owns samples i, i+64, ...: every load is a coalesced
// wave-wide read of the ray's contiguous (S, 4) raw block / (S,) t row, the transmittance is a
// wavefront prefix-product scan (6 __shfl_up steps per 64-sample block) carried across blocks.
// The scan runs in fp64 and rounds each prefix to fp32, which is what torch CPU's cumprod does
// (fp64 accumulator, measured), so T_i matches the reference bit-for-bit in practice.
// The per-ray sums (acc = sum w, depth = sum w*t, rgb = sum w*c) are staged in LDS and reduced
// in torch's CPU summation order (torch_sum.hpp), spread over lanes.
#include "aon_common.hpp"
#include "torch_sum.hpp"

namespace aon {

constexpr int kCompWaves = 4;
constexpr int kCompMaxS = 512;

struct CompLds {
  float w[kCompMaxS], wt[kCompMaxS], wc[3 * kCompMaxS];
};

__device__ __forceinline__ void wave_sync_c() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ float act_rgb(float x, int act) {
  if (act == AON_ACT_NONE) return x;
  const float s = __fdiv_rn(1.0f, __fadd_rn(1.0f, expf(-x)));
  return act == AON_ACT_ARTIC ? __fsub_rn(__fmul_rn(s, 1.002f), 0.001f) : s;
}

__device__ __forceinline__ float act_sigma(float x, int act) {
  if (act == AON_ACT_NONE) return x;
  if (act == AON_ACT_VANILLA) return fmaxf(x, 0.0f);
  // softplus(x - 1) with torch's threshold 20 (model_autodecoder.py:323)
  const float z = __fsub_rn(x, 1.0f);
  return z > 20.0f ? z : log1pf(expf(z));
}

__global__ __launch_bounds__(64 * kCompWaves) void k_composite_fwd(
    const float* __restrict__ rgb, int64_t rgb_stride, const float* __restrict__ sig,
    int64_t sig_stride, const float* __restrict__ tv, const float* __restrict__ dirs, int64_t B,
    int S, int white, int act, float* __restrict__ out_rgb, float* __restrict__ out_acc,
    float* __restrict__ out_w, float* __restrict__ out_depth) {
  __shared__ CompLds lds_all[kCompWaves];
  CompLds& Ls = lds_all[threadIdx.x >> 6];
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = (int64_t)gridDim.x * kCompWaves;
  for (int64_t ray = (int64_t)blockIdx.x * kCompWaves + (threadIdx.x >> 6); ray < B;
       ray += nwaves) {
    const float dx = dirs[3 * ray], dy = dirs[3 * ray + 1], dz = dirs[3 * ray + 2];
    const float dnorm = sqrtf(fmaf(dz, dz, fmaf(dy, dy, __fmul_rn(dx, dx))));
    const float* t = tv + ray * S;
    const int64_t row0 = ray * S;
    double carry = 1.0;  // prod_{j < block start} (1 - alpha_j + 1e-10)
    for (int base = 0; base < S; base += 64) {
      const int i = base + lane;
      const bool valid = i < S;
      float w = 0.f;
      double f = 1.0;
      float ti = 0.f, cr = 0.f, cg = 0.f, cb = 0.f;
      if (valid) {
        ti = t[i];
        const float dist = (i + 1 < S) ? __fsub_rn(t[i + 1], ti) : 1e10f;
        const float sgm = act_sigma(sig[(row0 + i) * sig_stride], act);
        const float alpha = __fsub_rn(1.0f, expf(__fmul_rn(-sgm, __fmul_rn(dist, dnorm))));
        if (i + 1 < S) f = (double)__fadd_rn(__fsub_rn(1.0f, alpha), 1e-10f);
        w = alpha;  // times T_i below
        const float* c = rgb + (row0 + i) * rgb_stride;
        cr = act_rgb(c[0], act);
        cg = act_rgb(c[1], act);
        cb = act_rgb(c[2], act);
      }
      // inclusive prefix product over the block, then exclusive via one more shift
      double incl = f;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const double v = __shfl_up(incl, o);
        if (lane >= o) incl *= v;
      }
      double excl = __shfl_up(incl, 1);
      if (lane == 0) excl = 1.0;
      const float T = (float)(carry * excl);
      carry *= __shfl(incl, 63);
      if (valid) {
        w = __fmul_rn(w, T);
        if (out_w) out_w[row0 + i] = w;
        Ls.w[i] = w;
        Ls.wt[i] = __fmul_rn(w, ti);
        Ls.wc[3 * i] = __fmul_rn(w, cr);
        Ls.wc[3 * i + 1] = __fmul_rn(w, cg);
        Ls.wc[3 * i + 2] = __fmul_rn(w, cb);
      }
    }
    wave_sync_c();
    // torch-order reductions, one partial per lane (torch_sum.hpp)
    const float* lw = Ls.w;
    const float* lwt = Ls.wt;
    const float* lwc = Ls.wc;
    float v = 0.f;
    const bool vec = S >= 8;
    if (lane < 8) {
      v = vec ? inner_sum_lane([&](int e) { return lw[e]; }, S, lane)
              : (lane == 0 ? row_sum_ilp4([&](int e) { return lw[e]; }, S) : 0.f);
    } else if (lane < 16) {
      v = vec ? inner_sum_lane([&](int e) { return lwt[e]; }, S, lane - 8)
              : (lane == 8 ? row_sum_ilp4([&](int e) { return lwt[e]; }, S) : 0.f);
    } else if (lane < 19) {
      const int ch = lane - 16;
      v = row_sum_ilp4([&](int e) { return lwc[3 * e + ch]; }, S);
    } else if (lane == 19) {
      v = vec ? inner_sum_tail([&](int e) { return lw[e]; }, S) : 0.f;
    } else if (lane == 20) {
      v = vec ? inner_sum_tail([&](int e) { return lwt[e]; }, S) : 0.f;
    }
    float sa, sd;
    if (vec) {
      sa = __shfl(v, 19);
      sd = __shfl(v, 20);
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        sa = __fadd_rn(sa, __shfl(v, c));
        sd = __fadd_rn(sd, __shfl(v, 8 + c));
      }
    } else {
      sa = __shfl(v, 0);
      sd = __shfl(v, 8);
    }
    float sr = __shfl(v, 16), sg = __shfl(v, 17), sb = __shfl(v, 18);
    wave_sync_c();  // LDS reuse by this wave's next ray
    if (lane == 0) {
      if (white) {
        const float bg = __fsub_rn(1.0f, sa);
        sr = __fadd_rn(sr, bg);
        sg = __fadd_rn(sg, bg);
        sb = __fadd_rn(sb, bg);
      }
      out_rgb[3 * ray] = sr;
      out_rgb[3 * ray + 1] = sg;
      out_rgb[3 * ray + 2] = sb;
      out_acc[ray] = sa;
      // nan_to_num(depth, nan=inf) then clamp(depth, min, max) over the chunk, which is the
      // identity on the resulting values (helper.py:182-183)
      out_depth[ray] = nan_to_num(sd, __builtin_inff());
    }
  }
}

}  // namespace aon

using namespace aon;

extern "C" int aon_composite_fwd(const float* rgb, int64_t rgb_stride, const float* sigma,
                                 int64_t sigma_stride, const float* t, const float* dirs,
                                 int64_t B, int S, int white_bkgd, int act, float* comp_rgb,
                                 float* acc, float* weights, float* depth, aon_stream_t stream) {
  AON_REQUIRE(rgb && sigma && t && dirs && comp_rgb && acc && depth, "null pointer");
  AON_REQUIRE(B >= 0 && S >= 1 && S <= kCompMaxS && rgb_stride >= 3 && sigma_stride >= 1,
              "bad shape (1 <= S <= 512)");
  AON_REQUIRE(act >= AON_ACT_NONE && act <= AON_ACT_ARTIC, "bad activation");
  if (B == 0) return 0;
  hipLaunchKernelGGL(k_composite_fwd, grid_for(B, kCompWaves, 1 << 16), 64 * kCompWaves, 0,
                     (hipStream_t)stream, rgb, rgb_stride, sigma, sigma_stride, t, dirs, B, S,
                     white_bkgd, act, comp_rgb, acc, weights, depth);
  return launch_status(__func__);
}
