// Evaluation metrics and image output of the reference's test epoch (models/interface.py:54-62,
// 64-74, 124-139; models/utils.py:12-13, 21-27, 102-109; model.py:459-507).
#include "aon_common.hpp"

namespace aon {

// One workgroup per image: mean over the (masked) pixels' 3 channels of
// (clip(pred) - clip(gt))^2 (clip only when `clip`), accumulated in fp64; psnr = -10 ln(mse)/ln 10.
__global__ __launch_bounds__(256) void k_image_mse(const float* __restrict__ pred,
                                                   const float* __restrict__ gt, int64_t P,
                                                   const uint8_t* __restrict__ mask, int clip,
                                                   float* __restrict__ mse,
                                                   float* __restrict__ psnr) {
  __shared__ double s_sum[256];
  __shared__ long long s_cnt[256];
  const int64_t img = blockIdx.x;
  const float* p = pred + img * P * 3;
  const float* g = gt + img * P * 3;
  const uint8_t* m = mask ? mask + img * P : nullptr;
  double acc = 0.0;
  long long cnt = 0;
  for (int64_t e = threadIdx.x; e < P * 3; e += 256) {
    if (m && !m[e / 3]) continue;
    float a = p[e], b = g[e];
    if (clip) {
      a = fminf(fmaxf(a, 0.0f), 1.0f);
      b = fminf(fmaxf(b, 0.0f), 1.0f);
    }
    const float d = __fsub_rn(a, b);
    acc += (double)__fmul_rn(d, d);
    ++cnt;
  }
  s_sum[threadIdx.x] = acc;
  s_cnt[threadIdx.x] = cnt;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      s_sum[threadIdx.x] += s_sum[threadIdx.x + o];
      s_cnt[threadIdx.x] += s_cnt[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    // torch.mean of an empty selection is nan
    const float v = s_cnt[0] ? (float)(s_sum[0] / (double)s_cnt[0]) : __builtin_nanf("");
    mse[img] = v;
    if (psnr) psnr[img] = __fdiv_rn(__fmul_rn(-10.0f, logf(v)), 2.30258512f);
  }
}

// to8b (models/utils.py:12-13): uint8(255 * clip(x, 0, 1)), numpy's cast truncates
__global__ void k_to8b(const float* __restrict__ x, int64_t n, uint8_t* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float c = fminf(fmaxf(x[i], 0.0f), 1.0f);
    out[i] = static_cast<uint8_t>(__fmul_rn(255.0f, c));
  }
}

}  // namespace aon

using namespace aon;

extern "C" int aon_image_mse(const float* pred, const float* gt, int64_t n_images,
                             int64_t pixels, const uint8_t* mask, int clip, float* mse,
                             float* psnr, aon_stream_t stream) {
  AON_REQUIRE(pred && gt && mse && n_images >= 0 && pixels >= 0, "bad arguments");
  AON_REQUIRE(n_images < (1ll << 31), "too many images");
  if (n_images == 0) return 0;
  hipLaunchKernelGGL(k_image_mse, (unsigned)n_images, 256, 0, (hipStream_t)stream, pred, gt,
                     pixels, mask, clip, mse, psnr);
  return launch_status(__func__);
}

extern "C" int aon_to8b(const float* x, int64_t n, uint8_t* out, aon_stream_t stream) {
  AON_REQUIRE(x && out && n >= 0, "bad arguments");
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_to8b, grid_for(n, 256, 65536), 256, 0, (hipStream_t)stream, x, n, out);
  return launch_status(__func__);
}
