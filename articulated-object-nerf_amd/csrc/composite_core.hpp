// Alpha compositing device code (reference models/vanilla_nerf/helper.py:157-195), shared by
// k_composite_fwd (composite.hip) and the fused coarse composite + resample kernel (march.hip).
#pragma once

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

// The compositor's math for one ray, its inputs in registers (lane i: sample 64 b + i's t and
// raw [r, g, b, sigma]): alpha, the fp64 DPP transmittance scan, weights into the planar LDS
// arrays P (and out_w when given), the torch-order sums and the ray's rgb / acc / depth.  Leaves
// the weights in P[0 .. S) (the fused march kernel resamples from there).
template <int NB, int SC>
__device__ __forceinline__ void composite_ray(const float (&tt)[NB], const f4 (&raw)[NB],
                                              const float* __restrict__ dirs, int64_t ray, int S,
                                              int lane, int act, int white, float* P, int SM,
                                              float* scratch, float* sums,
                                              float* __restrict__ out_rgb,
                                              float* __restrict__ out_acc,
                                              float* __restrict__ out_w,
                                              float* __restrict__ out_depth) {
  const int64_t row0 = ray * S;
  const bool inner8 = S >= 8;
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
      alpha = __fsub_rn(1.0f, exp_cr(__fmul_rn(-sgm, __fmul_rn(dist, dnorm))));
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
}

}  // namespace aon
