// Kernels of the articulated training step (LitNeRF_AutoDecoder.training_step,
// models/vanilla_nerf/model_autodecoder.py:395-477) that the layer GEMMs (gemm_f16x3.hip) do
// not cover: the backward of pos_enc applied to the deformed points (model_autodecoder.py:205-212,
// helper.py:136-140), through which the trunk's input gradient reaches the deformation MLP, and
// the latent-code regulariser (model_autodecoder.py:456-466).
#include "aon_common.hpp"

#include <cmath>

namespace aon {

// dL/dx of enc = pos_enc(x) = cat[x, sin(x 2^d), sin(x 2^d + pi/2f)] for one (row, component):
// autograd of helper.py:136-140 — sin'(a) = cos(a) at each argument as the forward formed it
// (the cosine half's argument is fp32(x 2^d + 1.5707964)), the two halves' gradients meet on
// xb = x 2^d, the broadcast multiply by 2^d sums over degrees, and the identity channel adds last.
__global__ void k_pos_enc_bwd(const float* __restrict__ x, int64_t ldx,
                              const float* __restrict__ g, int64_t ldg, int64_t n, int min_deg,
                              int L, int accumulate, float* __restrict__ dx, int64_t lddx) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < 3 * n; i += stride) {
    const int64_t r = i / 3;
    const int c = (int)(i - 3 * r);
    const float xc = x[r * ldx + c];
    const float* gr = g + r * ldg;
    float acc = 0.0f;
    for (int d = 0; d < L; ++d) {
      const float s = __builtin_ldexpf(1.0f, min_deg + d);
      const float xb = __fmul_rn(xc, s);  // exact (power of two)
      const float g_xb = __fadd_rn(__fmul_rn(gr[3 + 3 * d + c], cos_cr(xb)),
                                   __fmul_rn(gr[3 + 3 * L + 3 * d + c], cos_cr(__fadd_rn(xb, kHalfPi))));
      acc = __fadd_rn(acc, __fmul_rn(g_xb, s));
    }
    float v = __fadd_rn(gr[c], acc);
    if (accumulate) v = __fadd_rn(dx[r * lddx + c], v);
    dx[r * lddx + c] = v;
  }
}

// loss (+)= weight * mean_c ||x[:, c]||_2 over an (n, c) code; grad = weight / C * x / ||x[:, c]||
// (0 where the column norm is 0, as torch's norm backward).  One workgroup, fixed order.
__global__ __launch_bounds__(256) void k_latent_reg(const float* __restrict__ x, int64_t n,
                                                    int64_t C, float weight, int accumulate,
                                                    float* __restrict__ loss,
                                                    float* __restrict__ grad) {
  __shared__ float part[256];
  float s = 0.0f;
  const float gscale = __fdiv_rn(weight, (float)C);
  for (int64_t c = threadIdx.x; c < C; c += blockDim.x) {
    float ss = 0.0f;
    for (int64_t r = 0; r < n; ++r) ss = fmaf(x[r * C + c], x[r * C + c], ss);
    const float nrm = sqrtf(ss);
    s = __fadd_rn(s, nrm);
    if (grad)
      for (int64_t r = 0; r < n; ++r)
        grad[r * C + c] = nrm > 0.0f ? __fmul_rn(gscale, __fdiv_rn(x[r * C + c], nrm)) : 0.0f;
  }
  part[threadIdx.x] = s;
  __syncthreads();
  for (int w = blockDim.x / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) part[threadIdx.x] = __fadd_rn(part[threadIdx.x], part[threadIdx.x + w]);
    __syncthreads();
  }
  if (threadIdx.x == 0 && loss) {
    const float v = __fmul_rn(weight, __fdiv_rn(part[0], (float)C));
    *loss = accumulate ? __fadd_rn(*loss, v) : v;
  }
}

}  // namespace aon

using namespace aon;

extern "C" int aon_pos_enc_bwd(const float* x, int64_t ldx, const float* g_enc, int64_t ldg,
                               int64_t n, int min_deg, int max_deg, int accumulate, float* dx,
                               int64_t lddx, aon_stream_t stream) {
  AON_REQUIRE(x && g_enc && dx, "null pointer");
  const int L = max_deg - min_deg;
  AON_REQUIRE(n >= 0 && L >= 0 && L <= 16, "bad shape");
  AON_REQUIRE(ldx >= 3 && lddx >= 3 && ldg >= 3 + 6 * L, "bad leading dimension");
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_pos_enc_bwd, grid_for(3 * n, 256, 65536), 256, 0, (hipStream_t)stream, x,
                     ldx, g_enc, ldg, n, min_deg, L, accumulate, dx, lddx);
  return launch_status(__func__);
}

extern "C" int aon_latent_reg(const float* code, int64_t n, int64_t c, float weight,
                              int accumulate, float* loss, float* grad, aon_stream_t stream) {
  AON_REQUIRE(code && (loss || grad), "null pointer");
  AON_REQUIRE(n >= 1 && c >= 1, "empty code");
  hipLaunchKernelGGL(k_latent_reg, 1, 256, 0, (hipStream_t)stream, code, n, c, weight, accumulate,
                     loss, grad);
  return launch_status(__func__);
}
