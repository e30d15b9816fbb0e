// Alpha compositing (reference models/vanilla_nerf/helper.py:157-195) -- HBM-bound.
//
// One 64-lane wave per ray; lane i owns samples i, i+64, ...: every load is a coalesced
// wave-wide read of the ray's contiguous (S, 4) raw block / (S,) t row, all issued before any
// math.  The transmittance is an fp64 prefix product (DPP row shifts/broadcasts, 6 steps per
// 64-sample block) carried across blocks and rounded per prefix to fp32, which is what torch
// CPU's cumprod does (fp64 accumulator, measured), so T_i matches the reference bit-for-bit in
// practice.  The per-ray sums (acc = sum w, depth = sum w*t, rgb = sum w*c) are staged in LDS
// and evaluated in torch's CPU summation order by the whole wave (torch_sum.hpp).
#include "composite_core.hpp"

namespace aon {

// One 64-lane wave per ray, NB = ceil(S/64) blocks of 64 samples (lane i owns samples i + 64b).
// All of a ray's loads are issued up front (NB x {16-B raw, 4-B t} per lane), the
// transmittance is an fp64 DPP prefix product per block (torch CPU's cumprod accumulates in
// fp64) carried across blocks, and the per-ray sums are evaluated in torch's CPU order by the
// whole wave (wave_row_sums) from planar LDS arrays w, w*t, w*r, w*g, w*b.
// RAW4: rgb and sigma interleaved as one (.., 4) fp32 row, 16-B aligned -> one dwordx4 load.
// SC > 0: the sample count as a compile-time constant (the render's 65 and 193), so the
// torch-order sum schedule (task split, chunk counts, tails) folds to constants.
template <int NB, bool RAW4, int SC = 0>
__global__ __launch_bounds__(64 * kCompWaves, SC > 0 ? (SC > 128 ? AON_COMP_OCC_FINE : 8) : 1) void k_composite_fwd(
    const float* __restrict__ rgb, int64_t rgb_stride, const float* __restrict__ sig,
    int64_t sig_stride, const float* __restrict__ tv, const float* __restrict__ dirs, int64_t B,
    int S_rt, int white, int act, float* __restrict__ out_rgb, float* __restrict__ out_acc,
    float* __restrict__ out_w, float* __restrict__ out_depth) {
  // LDS rows of SM floats; with the sample count known at compile time they are S long and the
  // scratch is exactly the sums' task count, so more waves fit per CU (LDS bounds occupancy)
  constexpr int SM = SC > 0 ? SC : 64 * NB;
  constexpr int kScratch = SC > 0 ? comp_scratch(SC) : kCompScratch;
  const int S = SC > 0 ? SC : S_rt;
  __shared__ float lds_all[kCompWaves][5 * SM + kScratch + 32];
  float* P = lds_all[threadIdx.x >> 6];  // P[q * SM + i]: q = 0 w, 1 w*t, 2..4 w*rgb
  float* scratch = P + 5 * SM;
  float* sums = scratch + kScratch;
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = (int64_t)gridDim.x * kCompWaves;
  for (int64_t ray = (int64_t)blockIdx.x * kCompWaves + (threadIdx.x >> 6); ray < B;
       ray += nwaves) {
    const int64_t row0 = ray * S;
    const float* t = tv + row0;
    float tt[NB];
    f4 raw[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int i = 64 * b + lane;
      tt[b] = 0.f;
      raw[b] = f4{0.f, 0.f, 0.f, 0.f};
      if (i < S) {
        tt[b] = t[i];
        if (RAW4) {
          raw[b] = *reinterpret_cast<const f4*>(rgb + (row0 + i) * 4);
        } else {
          const float* c = rgb + (row0 + i) * rgb_stride;
          raw[b] = f4{c[0], c[1], c[2], sig[(row0 + i) * sig_stride]};
        }
      }
    }
    composite_ray<NB, SC>(tt, raw, dirs, ray, S, lane, act, white, P, SM, scratch, sums, out_rgb,
                          out_acc, out_w, out_depth);
    wave_sync_c();  // LDS reuse by this wave's next ray
  }
}

template <int NB, int SC = 0>
static void launch_composite(bool raw4, int grid, hipStream_t st, const float* rgb,
                             int64_t rgb_stride, const float* sig, int64_t sig_stride,
                             const float* t, const float* dirs, int64_t B, int S, int white,
                             int act, float* comp, float* acc, float* w, float* depth) {
  if (raw4)
    hipLaunchKernelGGL((k_composite_fwd<NB, true, SC>), grid, 64 * kCompWaves, 0, st, rgb,
                       rgb_stride, sig, sig_stride, t, dirs, B, S, white, act, comp, acc, w, depth);
  else
    hipLaunchKernelGGL((k_composite_fwd<NB, false, SC>), grid, 64 * kCompWaves, 0, st, rgb,
                       rgb_stride, sig, sig_stride, t, dirs, B, S, white, act, comp, acc, w,
                       depth);
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
  const bool raw4 = rgb_stride == 4 && sigma_stride == 4 && sigma == rgb + 3 && aligned16(rgb);
  const int grid = grid_for(B, kCompWaves, 1 << 16);
  hipStream_t st = (hipStream_t)stream;
  if (S == 193 || S == 65) {  // the render's levels (64 + 1 coarse, 64 + 1 + 128 fine)
    if (S == 193)
      launch_composite<4, 193>(raw4, grid, st, rgb, rgb_stride, sigma, sigma_stride, t, dirs, B,
                               S, white_bkgd, act, comp_rgb, acc, weights, depth);
    else
      launch_composite<2, 65>(raw4, grid, st, rgb, rgb_stride, sigma, sigma_stride, t, dirs, B,
                              S, white_bkgd, act, comp_rgb, acc, weights, depth);
    return launch_status(__func__);
  }
  switch ((S + 63) / 64) {
#define AON_COMP_CASE(nb)                                                                       \
  case nb:                                                                                      \
    launch_composite<nb>(raw4, grid, st, rgb, rgb_stride, sigma, sigma_stride, t, dirs, B, S,   \
                         white_bkgd, act, comp_rgb, acc, weights, depth);                       \
    break;
    AON_COMP_CASE(1)
    AON_COMP_CASE(2)
    AON_COMP_CASE(3)
    AON_COMP_CASE(4)
    AON_COMP_CASE(5)
    AON_COMP_CASE(6)
    AON_COMP_CASE(7)
    AON_COMP_CASE(8)
#undef AON_COMP_CASE
  }
  return launch_status(__func__);
}
