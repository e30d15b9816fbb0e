// Alpha compositing (reference models/vanilla_nerf/helper.py:157-195) -- HBM-bound.
//
// One 64-lane wave per ray; lane i owns samples i, i+64, ...: every load is a coalesced
// wave-wide read of the ray's contiguous (S, 4) raw block / (S,) t row, all issued before any
// math.  The transmittance is an fp64 prefix product (DPP row shifts/broadcasts, 6 steps per
// 64-sample block) carried across blocks and rounded per prefix to fp32, which is what torch
// CPU's cumprod does (fp64 accumulator, measured), so T_i matches the reference bit-for-bit in
// practice.  The per-ray sums (acc = sum w, depth = sum w*t, rgb = sum w*c) are staged in LDS
// and evaluated in torch's CPU summation order by the whole wave (torch_sum.hpp).
#include "aon_common.hpp"
#include "torch_sum.hpp"

namespace aon {

#ifndef AON_COMP_OCC_FINE
#define AON_COMP_OCC_FINE 6  // waves per SIMD the fine-level (S = 193) instantiation is built for (7: 72 VGPRs, 8: spills; both no faster)
#endif

constexpr int kCompWaves = 4;
constexpr int kCompMaxS = 512;
constexpr int kCompScratch = 256;  // wave_row_sums task partials (<= 236 at S = 512)

// wave_row_sums task partials the compositor's sums need at S samples (3 rgb sums over S terms,
// 16 vector-lane sums over S/8 terms; torch_sum.hpp)
constexpr int comp_scratch(int S) {
  return S < 8 ? 256
               : 3 * 4 * ((S >> 2 >> 4) + 1) + 16 * 4 * (((S / 8) >> 2 >> 4) + 1);
}

__device__ __forceinline__ void wave_sync_c() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// ---- DPP lane moves (gfx9 controls).  Lanes whose source is outside the pattern keep `old`.
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ double dpp_f64(double src, double old) {
  const long long s = __builtin_bit_cast(long long, src), o = __builtin_bit_cast(long long, old);
  const int lo = __builtin_amdgcn_update_dpp((int)o, (int)s, CTRL, ROW_MASK, 0xF, false);
  const int hi =
      __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(s >> 32), CTRL, ROW_MASK, 0xF, false);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
}

__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const long long s = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_readlane((int)s, lane);
  const int hi = __builtin_amdgcn_readlane((int)(s >> 32), lane);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
}

// inclusive prefix product over the 64 lanes: row_shr 1/2/4/8 inside 16-lane rows, then
// row_bcast:15 (rows 1, 3) and row_bcast:31 (rows 2, 3) -- VALU lane moves, no LDS
__device__ __forceinline__ double wave_incl_prod(double x) {
  x *= dpp_f64<0x111>(x, 1.0);
  x *= dpp_f64<0x112>(x, 1.0);
  x *= dpp_f64<0x114>(x, 1.0);
  x *= dpp_f64<0x118>(x, 1.0);
  x *= dpp_f64<0x142, 0xA>(x, 1.0);
  x *= dpp_f64<0x143, 0xC>(x, 1.0);
  return x;
}

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
  const bool inner8 = S >= 8;
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
    const float dx = dirs[3 * ray], dy = dirs[3 * ray + 1], dz = dirs[3 * ray + 2];
    const float dnorm = sqrtf(fmaf(dz, dz, fmaf(dy, dy, __fmul_rn(dx, dx))));
    double carry = 1.0;  // prod_{j < block start} (1 - alpha_j + 1e-10)
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int i = 64 * b + lane;
      const bool valid = i < S;
      // t[i + 1]: lane i + 1 of this block, or lane 0 of the next (wave_shl:1)
      const float tnext0 = b + 1 < NB ? __builtin_bit_cast(float, __builtin_amdgcn_readlane(
                                                                      __builtin_bit_cast(int, tt[b + 1]), 0))
                                      : 0.f;
      const float tn = __builtin_bit_cast(
          float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, tnext0),
                                             __builtin_bit_cast(int, tt[b]), 0x130, 0xF, 0xF, false));
      const float ti = tt[b];
      float alpha = 0.f;
      double f = 1.0;
      if (valid) {
        const float dist = (i + 1 < S) ? __fsub_rn(tn, ti) : 1e10f;
        const float sgm = act_sigma(raw[b].w, act);
        alpha = __fsub_rn(1.0f, expf(__fmul_rn(-sgm, __fmul_rn(dist, dnorm))));
        if (i + 1 < S) f = (double)__fadd_rn(__fsub_rn(1.0f, alpha), 1e-10f);
      }
      const double incl = wave_incl_prod(f);
      const double excl = dpp_f64<0x138>(incl, 1.0);  // wave_shr:1, lane 0 -> 1
      const float T = (float)(carry * excl);
      if (b + 1 < NB) carry *= readlane_f64(incl, 63);
      if (valid) {
        const float w = __fmul_rn(alpha, T);
        if (out_w) out_w[row0 + i] = w;
        P[i] = w;
        P[SM + i] = __fmul_rn(w, ti);
        P[2 * SM + i] = __fmul_rn(w, act_rgb(raw[b].x, act));
        P[3 * SM + i] = __fmul_rn(w, act_rgb(raw[b].y, act));
        P[4 * SM + i] = __fmul_rn(w, act_rgb(raw[b].z, act));
      }
    }
    wave_sync_c();
    // torch-order sums (torch_sum.hpp): specs 0..2 = rgb over S terms (stride-3 outer sum);
    // S >= 8: specs 3..18 = the 8 vector lanes of the inner sums of w (3..10) and w*t (11..18)
    // over S/8 terms each; S < 8: specs 3, 4 = scalar sums of w, w*t.
    wave_row_sums(
        [&](int sp, const float*& base, int& str) {
          if (sp < 3) {
            base = P + (2 + sp) * SM;
            str = 1;
          } else if (inner8) {
            base = P + ((sp - 3) >> 3) * SM + ((sp - 3) & 7);
            str = 8;
          } else {
            base = P + (sp - 3) * SM;
            str = 1;
          }
        },
        3, S, inner8 ? 16 : 2, inner8 ? S / 8 : S, scratch, sums, lane, wave_sync_c);
    if (lane < 2) {
      // acc (lane 0) / depth (lane 1): tail x[8m..S) from 0, then + vector lanes 0..7
      float s;
      if (inner8) {
        s = 0.f;
        for (int e = (S / 8) * 8; e < S; ++e) s = __fadd_rn(s, P[lane * SM + e]);
#pragma unroll
        for (int c = 0; c < 8; ++c) s = __fadd_rn(s, sums[3 + 8 * lane + c]);
      } else {
        s = sums[3 + lane];
      }
      if (lane == 0) {
        float sr = sums[0], sg = sums[1], sb = sums[2];
        if (white) {
          const float bg = __fsub_rn(1.0f, s);
          sr = __fadd_rn(sr, bg);
          sg = __fadd_rn(sg, bg);
          sb = __fadd_rn(sb, bg);
        }
        out_rgb[3 * ray] = sr;
        out_rgb[3 * ray + 1] = sg;
        out_rgb[3 * ray + 2] = sb;
        out_acc[ray] = s;
      } else {
        // nan_to_num(depth, nan=inf) then clamp(depth, min, max) over the chunk, which is the
        // identity on the resulting values (helper.py:182-183)
        out_depth[ray] = nan_to_num(s, __builtin_inff());
      }
    }
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
