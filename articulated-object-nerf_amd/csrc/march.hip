// Coarse-level compositing fused with the hierarchical resampling that consumes its weights
// ("march"): reference models/vanilla_nerf/helper.py:157-195 (volumetric_rendering) then
// helper.py:203-252 (sample_pdf on mids of t and weights[..., 1:-1]) and the merge of
// model.py:163-172, for one ray per 64-lane wave.
//
// The separate kernels round-trip the coarse weights through HBM (written by the compositor,
// read back with t by k_sample_pdf).  Here the weights never leave the wave: the compositor
// leaves them in its planar LDS row (composite_ray), the resampler reads weights[1 : S-1] from
// that row and t from the registers the compositor loaded, so a ray moves only raw + t + dirs
// in and rgb / acc / depth + the merged fine t out (weights too only when the caller asks).
// Same device code as k_composite_fwd and k_sample_pdf: outputs are bit-identical to the
// two-kernel path.
#include "composite_core.hpp"
#include "pdf_core.hpp"

namespace aon {

// LDS of one wave: the compositor's planar rows + sum scratch, then the resampler's rows
template <int SM, int SCR, int NBX, int NO>
struct MarchLds {
  float P[5 * SM + SCR + 32];
  PdfLds<NBX> L;
  float orow[NO];  // the merged fine t row, written out by coalesced stores
};

#ifndef AON_MARCH_OCC
#define AON_MARCH_OCC 7  // waves per SIMD the S = 65 instantiation is built for (6 / 8 slower: profiles/r02/ab_march)
#endif

template <int NB, int SC, int NBX>
__global__ __launch_bounds__(64 * kCompWaves, SC > 0 ? AON_MARCH_OCC : 1) void k_composite_march(
    const float* __restrict__ raw4, const float* __restrict__ tv, const float* __restrict__ dirs,
    int64_t B, int S_rt, int white, int act, const float* __restrict__ u_g, int64_t u_stride,
    int Ns, int Ns_pow2, float* __restrict__ out_rgb, float* __restrict__ out_acc,
    float* __restrict__ out_w, float* __restrict__ out_depth, float* __restrict__ t_out) {
  constexpr int SM = SC > 0 ? SC : 64 * NB;
  constexpr int kScratch = SC > 0 ? comp_scratch(SC) : kCompScratch;
  const int S = SC > 0 ? SC : S_rt;
  __shared__ MarchLds<SM, kScratch, NBX, SM + 64 * NBX> lds_all[kCompWaves];
  MarchLds<SM, kScratch, NBX, SM + 64 * NBX>& M = lds_all[threadIdx.x >> 6];
  float* P = M.P;
  float* scratch = P + 5 * SM;
  float* sums = scratch + kScratch;
  PdfLds<NBX>& L = M.L;
  const int lane = threadIdx.x & 63;
  const int nb = S - 1;  // bins = mids of t
  const int64_t nwaves = (int64_t)gridDim.x * kCompWaves;
  for (int64_t ray = (int64_t)blockIdx.x * kCompWaves + (threadIdx.x >> 6); ray < B;
       ray += nwaves) {
    const int64_t row0 = ray * S;
    // every load of the ray up front: raw rows and t (compositor layout), the fine uniforms
    float tt[NB];
    f4 raw[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int i = 64 * b + lane;
      tt[b] = 0.f;
      raw[b] = f4{0.f, 0.f, 0.f, 0.f};
      if (i < S) {
        tt[b] = tv[row0 + i];
        raw[b] = *reinterpret_cast<const f4*>(raw4 + (row0 + i) * 4);
      }
    }
    float cu[NBX];
#pragma unroll
    for (int b = 0; b < NBX; ++b) {
      const int i = 64 * b + lane;
      cu[b] = i < Ns ? u_g[ray * u_stride + i] : 0.f;
    }
#ifdef AON_MARCH_ABL_NOCOMP  // timing-only ablation: weights = raw sigma, no compositing
#pragma unroll
    for (int b = 0; b < NB; ++b)
      if (64 * b + lane < S) P[64 * b + lane] = raw[b].w;
    wave_sync();
    if (false)
#endif
    composite_ray<NB, SC>(tt, raw, dirs, ray, S, lane, act, white, P, SM, scratch, sums, out_rgb,
                          out_acc, out_w, out_depth);
    // the resampler's rows: t_merge = this ray's t (already in registers), bins = its mids
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int i = 64 * b + lane;
      if (i < S) L.tm[i] = tt[b];
    }
    wave_sync();
    for (int k = lane; k < nb; k += 64) L.bins[k] = __fmul_rn(0.5f, __fadd_rn(L.tm[k + 1], L.tm[k]));
    // weights[..., 1:-1] straight from the compositor's LDS row (P[0 .. S) = w)
#ifndef AON_MARCH_ABL_NOPDF  // timing-only ablation (wrong t_fine)
    pdf_ray<NBX>(L, P + 1, nb, Ns, Ns_pow2, cu, true, S, ray, lane, M.orow, nullptr, nullptr,
                 nullptr);
#endif
    wave_sync();
    // the merged row leaves in wave-contiguous stores (the merge scatters within it)
    const int No = S + Ns;
    float* orow_g = t_out + ray * No;
    for (int i = lane; i < No; i += 64) orow_g[i] = M.orow[i];
    wave_sync();  // LDS reuse by this wave's next ray
  }
}

// ---------------------------------------------------------------------------------------------
// The render's shape (S = 65 coarse samples, Ns = 128 fine) at FOUR rays per wave: ray r of the
// wave owns lanes 16 r .. 16 r + 15 (one DPP row).  Lane q of the row holds coarse samples
// q + 16 m (m = 0..3) and lane 0 also sample 64 ("m = 4"); fine samples j = q + 16 n (n = 0..7).
// The one-ray-per-wave kernel above spends most of its ~800 issued instructions per ray on a few
// lanes (torch-order sums on 9-19 lanes, the fp64 scans, a 1-sample second block); here every
// reduction runs on the row's own lanes, for four rays per instruction:
//   * transmittance: the same fp64 association as wave_incl_prod over a 64-lane block (Hillis-
//     Steele inside each 16-sample block m, then the block totals combined exactly as
//     row_bcast:15 / row_bcast:31 combine rows), so T is bit-identical to k_composite_fwd's;
//   * torch-order sums (torch_sum.hpp): the rgb sums' four 16-term folds x[4 s + k] advance as
//     DPP row_ror:4 chains, the inner sums of w and w t pair registers m, m + 2 and lanes c, c + 8
//     exactly as SumKernel's 8-lane vectors do, the final 9-term chains run along row_ror:1;
//   * the pdf's weight sum and fp64 CDF scan likewise, on the weights shifted by one sample;
//   * inverse CDF: 8 independent branch-free searches per lane (count_lift), the merge by the
//     bin hint and a per-row ballot fill -- pdf_ray's algorithm, row-local.
// Outputs are bit-identical to composite_ray + pdf_ray (tests: test_composite_march_*).
namespace rowm {

constexpr int kS = 65, kNs = 128, kNo = kS + kNs, kWaves = 2;

// Every cross-lane value below is "laundered" through an empty volatile asm: the move then
// stays where it is written, in uniform control flow.  Without it hipcc turned
// `q == 15 ? ror<1>(tl) : part` into a branch taken by lane 15 alone, folded tl to its lane-15
// value inside it and ran the DPP there -- reading the inactive lane 14 (a wrong weight sum).
template <typename T>
__device__ __forceinline__ T fence_v(T v) {
  asm volatile("" : "+v"(v));
  return v;
}
template <int CTRL>
__device__ __forceinline__ float dpp(float src, float old) {
  return fence_v(__builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
                                               __builtin_bit_cast(int, old),
                                               __builtin_bit_cast(int, src), CTRL, 0xF, 0xF, false)));
}
template <int CTRL>
__device__ __forceinline__ double dpp64(double src, double old) {
  return fence_v(dpp_f64<CTRL>(src, old));
}
// lane q of each 16-lane row <- lane (q - n) mod 16 of that row
template <int N> __device__ __forceinline__ float ror(float v) { return dpp<0x120 + N>(v, v); }
template <int N> __device__ __forceinline__ double ror64(double v) { return dpp64<0x120 + N>(v, v); }
// every lane of a 16-lane row <- lane L of that row (ds_swizzle bitmask mode, no LDS access)
template <int L>
__device__ __forceinline__ int row_bcast_i(int v) {
  return fence_v(__builtin_amdgcn_ds_swizzle(v, 0x10 | (L << 5)));
}
template <int L>
__device__ __forceinline__ float row_bcast(float v) {
  return __builtin_bit_cast(float, row_bcast_i<L>(__builtin_bit_cast(int, v)));
}
template <int L>
__device__ __forceinline__ double row_bcast64(double v) {
  const long long s = __builtin_bit_cast(long long, v);
  const int lo = row_bcast_i<L>((int)s), hi = row_bcast_i<L>((int)(s >> 32));
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
}
// Hillis-Steele inside the 16-lane rows (the first four steps of wave_incl_prod / _sum)
__device__ __forceinline__ double row_incl_prod(double x) {
  x *= dpp64<0x111>(x, 1.0);
  x *= dpp64<0x112>(x, 1.0);
  x *= dpp64<0x114>(x, 1.0);
  x *= dpp64<0x118>(x, 1.0);
  return x;
}
__device__ __forceinline__ double row_incl_sum(double x) {
  x += dpp64<0x111>(x, 0.0);
  x += dpp64<0x112>(x, 0.0);
  x += dpp64<0x114>(x, 0.0);
  x += dpp64<0x118>(x, 0.0);
  return x;
}

#ifndef AON_MARCH_DIRECT
#define AON_MARCH_DIRECT 1  // 0: merged rows staged in LDS and copied out (more LDS per wave)
#endif
#ifndef AON_MARCH_PIPE
#define AON_MARCH_PIPE 0  // 1: the next group's inputs loaded during this group's resampling (resident grid): 7% slower (profiles/r03/ab_march)
#endif
#ifndef AON_MARCH_ROWS_OCC
#define AON_MARCH_ROWS_OCC 5  // waves per SIMD the register budget is built for (92 VGPRs, no spills; 6 and 7 spill and run slower: profiles/r03/ab_march)
#endif

struct RayLds {
  float tm[68];      // t (65): the merge's t row
  float cdf[64];     // the CDF; after the inverse CDF: the merge's filled-slot bytes (193)
  float bins[64];    // mids of t (the sort path's samples overwrite cdf + bins: 128 floats)
#if !AON_MARCH_DIRECT
  float samp[kNs];
#endif
};
struct WaveLds {
  RayLds r[4];
#if !AON_MARCH_DIRECT
  float orow[4 * kNo];  // the four rays' merged rows, contiguous as in t_fine
#endif
};

// sorted a[0 .. 64) (a[63] = 1 for a CDF): entries <= x, count_lift<true>(a, 64, x) exactly --
// the top probe decides 64 / below, the six lower probes do not depend on it
__device__ __forceinline__ int count_le64(const float* a, float x) {
  const bool all = a[63] <= x;
  int c = 0;
#pragma unroll
  for (int step = 32; step > 0; step >>= 1) c = a[c + step - 1] <= x ? c + step : c;
  return all ? 64 : c;
}

template <int ACT>
__global__ __launch_bounds__(64 * kWaves, AON_MARCH_ROWS_OCC) void k_march_rows(
    const float* __restrict__ raw4, const float* __restrict__ tv, const float* __restrict__ dirs,
    int64_t B, int white, const float* __restrict__ u_g, int64_t u_stride,
    float* __restrict__ out_rgb, float* __restrict__ out_acc, float* __restrict__ out_w,
    float* __restrict__ out_depth, float* __restrict__ t_out) {
  constexpr int act = ACT;
  __shared__ WaveLds lds_all[kWaves];
  WaveLds& WL = lds_all[threadIdx.x >> 6];
  const int lane = threadIdx.x & 63, row = lane >> 4, q = lane & 15;
  RayLds& L = WL.r[row];
  const int64_t ngroups = (B + 3) >> 2;
  const int64_t gstride = (int64_t)gridDim.x * kWaves;
  // a group's per-ray inputs: t and raw of samples q + 16 m and sample 64 ("m = 4", every lane;
  // lane 0's copy is the one used), rays_d.  The last group's rows past B read the last ray (no
  // branches around the loads) and store nothing; 32-bit offsets (the host checks B * (S + Ns)
  // < 2^31).  AON_MARCH_PIPE: the next group's inputs are loaded while this group resamples
  // (its t / raw registers are dead by then), so a wave streaming several groups does not wait
  // on HBM at the top of each.
  auto load_group = [&](int64_t g, float (&t5)[5], f4 (&r5)[5], float (&d3)[3]) {
    const int64_t ry = 4 * g + row;
    const uint32_t rr = static_cast<uint32_t>(ry < B ? ry : B - 1);
#pragma unroll
    for (int m = 0; m < 5; ++m) {
      const uint32_t i = rr * kS + (m < 4 ? 16 * m + q : 64);
      t5[m] = tv[i];
      r5[m] = *reinterpret_cast<const f4*>(raw4 + 4 * i);
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) d3[c] = dirs[3 * rr + c];
  };
  int64_t grp = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  float ntt[5], nd[3];
  f4 nrw[5];
  if (AON_MARCH_PIPE && grp < ngroups) load_group(grp, ntt, nrw, nd);
  for (; grp < ngroups; grp += gstride) {
    const int64_t ray = 4 * grp + row;
    const bool valid = ray < B;
    const uint32_t rc = static_cast<uint32_t>(valid ? ray : B - 1);
    const uint32_t r0 = rc * kS;
    float tt[5], d3[3];
    f4 rw[5];
    if (AON_MARCH_PIPE) {
#pragma unroll
      for (int m = 0; m < 5; ++m) {
        tt[m] = ntt[m];
        rw[m] = nrw[m];
      }
#pragma unroll
      for (int c = 0; c < 3; ++c) d3[c] = nd[c];
    } else {
      load_group(grp, tt, rw, d3);
    }
    const float dx = d3[0], dy = d3[1], dz = d3[2];
    const float dnorm = sqrtf(fmaf(dz, dz, fmaf(dy, dy, __fmul_rn(dx, dx))));
    // ---- t[i + 1] of sample i = q + 16 m: lane q + 1, or lane 0's block m + 1 (row_ror:15)
    float tn[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) tn[m] = ror<15>(q == 0 ? tt[m + 1] : tt[m]);
    // ---- alpha, f = 1 - alpha + 1e-10 (helper.py:166-176)
    float alpha[5];
    double f[4];
#pragma unroll
    for (int m = 0; m < 5; ++m) {
      const float dist = m < 4 ? __fsub_rn(tn[m], tt[m]) : 1e10f;
      const float sgm = act_sigma(rw[m].w, act);
      alpha[m] = __fsub_rn(1.0f, exp_cr(__fmul_rn(-sgm, __fmul_rn(dist, dnorm))));
      if (m < 4) f[m] = (double)__fadd_rn(__fsub_rn(1.0f, alpha[m]), 1e-10f);
    }
    // ---- transmittance: wave_incl_prod's association over samples 0..63 (block m = row m of
    // the 64-lane scan), then T_i = excl_i (carry 1); sample 64: T = incl_63
    double hs[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) hs[m] = row_incl_prod(f[m]);
    const double e0 = row_bcast64<15>(hs[0]), e1 = row_bcast64<15>(hs[1]),
                 e2 = row_bcast64<15>(hs[2]);
    const double e01 = e1 * e0;  // lane 31 after the row_bcast:15 step
    double incl[4];
    incl[0] = hs[0];
    incl[1] = hs[1] * e0;
    incl[2] = hs[2] * e01;
    incl[3] = (hs[3] * e2) * e01;
    float w[5];
#pragma unroll
    for (int m = 0; m < 5; ++m) {
      // exclusive: lane q - 1 of block m, lane 0 <- lane 15 of block m - 1 (1.0 for m = 0)
      const double sel = m == 4 ? incl[3] : (q == 15 ? (m == 0 ? 1.0 : incl[m - 1]) : incl[m]);
      const float T = (float)ror64<1>(sel);  // (float)(carry 1.0 * excl) = (float)excl
      w[m] = __fmul_rn(alpha[m], T);
    }
    if (out_w && valid) {
#pragma unroll
      for (int m = 0; m < 5; ++m)
        if (m < 4 || q == 0) out_w[r0 + (m < 4 ? 16 * m + q : 64)] = w[m];
    }
    // ---- rgb: row_sum_ilp4 over 65 terms x_i = w_i rgb_i: folds C_k = x[k] + x[4+k] + ...
    // + x[60+k] as row_ror:4 chains (term s of fold k sits at lane 4 (s % 4) + k, block s / 4),
    // p_k = ((0 + (0 + C_k)) + 0) + 0, p_0 += x[64], ((p0 + p1) + p2) + p3
    float rgb_out[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      float x[5];
#pragma unroll
      for (int m = 0; m < 5; ++m) x[m] = __fmul_rn(w[m], act_rgb(c == 0 ? rw[m].x : (c == 1 ? rw[m].y : rw[m].z), act));
      float acc = __fadd_rn(0.f, x[0]);
#pragma unroll
      for (int s = 1; s < 16; ++s) acc = __fadd_rn(ror<4>(acc), x[s >> 2]);
      // lanes 12..15: C_0..C_3
      float p = __fadd_rn(__fadd_rn(__fadd_rn(0.f, __fadd_rn(0.f, acc)), 0.f), 0.f);
      const float x64 = ror<12>(x[4]);  // lane 12 <- lane 0's sample 64
      if (q == 12) p = __fadd_rn(p, x64);
      float r = p;
      r = __fadd_rn(ror<1>(r), p);  // lane 13: p0 + p1
      const float r13 = r;
      r = __fadd_rn(ror<1>(r13), p);  // lane 14
      const float r14 = r;
      r = __fadd_rn(ror<1>(r14), p);  // lane 15: ((p0 + p1) + p2) + p3
      rgb_out[c] = r;
    }
    // ---- acc / depth: inner sums of w and w t over 65 terms (8-lane vectors v_j = x[8j..8j+7]:
    // lane c's partial over j < 8 is ((((0 + y0) + y4) + ((0 + y1) + y5)) + ((0 + y2) + y6))
    // + ((0 + y3) + y7) with y_j = x[8 j + c]; j even -> block j / 2 lane c, j odd -> lane 8 + c)
    float sums2[2];
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      float y[5];
#pragma unroll
      for (int m = 0; m < 5; ++m) y[m] = v == 0 ? w[m] : __fmul_rn(w[m], tt[m]);
      const float a = __fadd_rn(__fadd_rn(0.f, y[0]), y[2]);
      const float b = __fadd_rn(__fadd_rn(0.f, y[1]), y[3]);
      const float part = __fadd_rn(__fadd_rn(__fadd_rn(a, ror<8>(a)), b), ror<8>(b));  // lanes 0..7
      // ((((tail + L0) + L1) ... + L7), tail = 0 + x[64] (lane 0) moved to lane 15
      const float tail = ror<15>(__fadd_rn(0.f, y[4]));
      float s = q == 15 ? tail : part;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float nx = __fadd_rn(ror<1>(s), part);
        s = q == k ? nx : s;
      }
      sums2[v] = s;  // lane 7
    }
    {
      const float accv = ror<8>(sums2[0]);  // lane 15 <- lane 7
      if (valid && q == 15) {
        float sr = rgb_out[0], sg = rgb_out[1], sb = rgb_out[2];
        if (white) {
          const float bg = __fsub_rn(1.0f, accv);
          sr = __fadd_rn(sr, bg);
          sg = __fadd_rn(sg, bg);
          sb = __fadd_rn(sb, bg);
        }
        out_rgb[3 * ray] = sr;
        out_rgb[3 * ray + 1] = sg;
        out_rgb[3 * ray + 2] = sb;
      }
      if (valid && q == 7) {
        out_acc[ray] = sums2[0];
        out_depth[ray] = nan_to_num(sums2[1], __builtin_inff());
      }
    }
    // ==== resampling (pdf_ray): bins = mids of t, weights[1 .. 63]
    // LDS rows: t (the merge), bins (inverse CDF)
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      L.tm[16 * m + q] = tt[m];
      L.bins[16 * m + q] = __fmul_rn(0.5f, __fadd_rn(tn[m], tt[m]));
    }
    if (q == 0) L.tm[64] = tt[4];
    if (AON_MARCH_PIPE && grp + gstride < ngroups) load_group(grp + gstride, ntt, nrw, nd);
    // wn[m] at lane q = w[q + 16 m + 1] = the pdf's weight w'[q + 16 m]
    float wn[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) wn[m] = ror<15>(q == 0 ? w[m + 1] : w[m]);
    // weight sum (helper.py:206): inner sum over nw = 63 terms w'[k]: 7 vectors of 8, lane c
    // (c < 8): row_sum_ilp4 over y_j = w'[8 j + c], j < 7 (j even: wn[j/2] lane c; odd: lane 8 + c)
    float ws;
    {
      const float y0 = wn[0], y1 = ror<8>(wn[0]), y2 = wn[1], y3 = ror<8>(wn[1]), y4 = wn[2],
                  y5 = ror<8>(wn[2]), y6 = wn[3];
      auto z3 = [](float v) { return __fadd_rn(__fadd_rn(__fadd_rn(__fadd_rn(0.f, v), 0.f), 0.f), 0.f); };
      float p0 = z3(y0);
      p0 = __fadd_rn(__fadd_rn(__fadd_rn(p0, y4), y5), y6);
      const float part = __fadd_rn(__fadd_rn(__fadd_rn(p0, z3(y1)), z3(y2)), z3(y3));  // lanes 0..7
      // tail: w'[56 .. 62] = wn[3] lanes 8..14, summed from 0 in order -> lane 14
      float tl = __fadd_rn(0.f, wn[3]);  // lane 8
#pragma unroll
      for (int k = 9; k < 15; ++k) {
        const float nx = __fadd_rn(ror<1>(tl), wn[3]);
        tl = q == k ? nx : tl;
      }
      const float tl14 = ror<1>(tl);
      float s = q == 15 ? tl14 : part;  // the tail at lane 15 (<- lane 14)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float nx = __fadd_rn(ror<1>(s), part);
        s = q == k ? nx : s;
      }
      ws = row_bcast<7>(s);
    }
    const float pad = fmaxf(0.0f, __fsub_rn(1e-5f, ws));
    const float padw = __fdiv_rn(pad, 63.0f);
    const float wsum = __fadd_rn(ws, pad);
    // CDF (helper.py:213-223): fp64 scan of pdf[0 .. 61], wave_incl_sum's association
    {
      double hp[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int k = 16 * m + q;
        const double v = k < 62 ? (double)__fdiv_rn(__fadd_rn(wn[m], padw), wsum) : 0.0;
        hp[m] = row_incl_sum(v);
      }
      const double s0 = row_bcast64<15>(hp[0]), s1 = row_bcast64<15>(hp[1]),
                   s2 = row_bcast64<15>(hp[2]);
      const double s01 = s1 + s0;
      double inc[4];
      inc[0] = hp[0];
      inc[1] = hp[1] + s0;
      inc[2] = hp[2] + s01;
      inc[3] = (hp[3] + s2) + s01;
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int k = 16 * m + q;
        if (k < 62) L.cdf[k + 1] = fminf(1.0f, (float)(0.0 + inc[m]));
      }
      if (q == 0) {
        L.cdf[0] = 0.0f;
        L.cdf[63] = 1.0f;
      }
    }
    wave_sync();
#ifdef AON_MARCH_DEBUG  // debug build: out_w row = [ws, padw, wsum, cdf[0..61]] instead of w
    if (out_w && valid) {
      if (q == 0) {
        out_w[r0] = ws;
        out_w[r0 + 1] = padw;
        out_w[r0 + 2] = wsum;
      }
      for (int k = q; k < 62; k += 16) out_w[r0 + 3 + k] = L.cdf[k + 1];
    }
#endif
    // inverse CDF (helper.py:232-241) for u_j, j = 16 n + q (u loaded here, not with the
    // compositor's inputs: 8 fewer registers live across the compositor; eval mode reads one
    // shared L2-resident row).  The eight searches run level by level (count_le64's probes, all
    // eight samples' LDS reads of a level issued together): sample by sample, each probe waited
    // for its own read and the chain of dependent LDS round trips set the kernel's pace.
    float uu[8];
    const uint32_t u0 = rc * static_cast<uint32_t>(u_stride);
#pragma unroll
    for (int n = 0; n < 8; ++n) uu[n] = u_g[u0 + 16 * n + q];
    float smp[8];
    int hint[8];
    {
      const float top = L.cdf[63];
      int c[8];
#pragma unroll
      for (int n = 0; n < 8; ++n) c[n] = 0;
#pragma unroll
      for (int step = 32; step > 0; step >>= 1) {
        float v[8];
#pragma unroll
        for (int n = 0; n < 8; ++n) v[n] = L.cdf[c[n] + step - 1];
#pragma unroll
        for (int n = 0; n < 8; ++n) c[n] = v[n] <= uu[n] ? c[n] + step : c[n];
      }
      // the interpolation in two halves of four samples (register budget)
#pragma unroll
      for (int h = 0; h < 8; h += 4) {
        float c0[4], c1[4], b0[4], b1[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int n = h + e;
          const int idx = top <= uu[n] ? 64 : c[n];  // = count_le(cdf, 64, u)
          const int i0 = idx - 1 < 0 ? 0 : (idx - 1 > 63 ? 63 : idx - 1);
          const int i1 = idx > 63 ? 63 : idx;
          hint[n] = i0;
          c0[e] = L.cdf[i0];
          c1[e] = L.cdf[i1];
          b0[e] = L.bins[i0];
          b1[e] = L.bins[i1];
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float qq = nan_to_num(__fdiv_rn(__fsub_rn(uu[h + e], c0[e]), __fsub_rn(c1[e], c0[e])), 0.0f);
          qq = fminf(fmaxf(qq, 0.0f), 1.0f);
          smp[h + e] = __fadd_rn(b0[e], __fmul_rn(qq, __fsub_rn(b1[e], b0[e])));
        }
      }
    }
    // sorted already (u ascending: always in eval mode)?  NaN compares unordered -> sort
    bool unsorted = false;
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      const float nxt = ror<15>(q == 0 ? smp[n < 7 ? n + 1 : 7] : smp[n]);
      if (!(n == 7 && q == 15)) unsorted |= !(smp[n] <= nxt);
    }
    const uint64_t ub = __builtin_amdgcn_ballot_w64(unsorted);
#if AON_MARCH_DIRECT
    // the merged row goes straight to t_fine: a row's stores land in one ~772-B window, nearly
    // consecutive per instruction (slot j + rank of sample j)
    float* orow = t_out + rc * kNo;
    float* samp = L.cdf;  // cdf + bins, dead after the inverse CDF
#else
    float* orow = WL.orow + row * kNo;
    float* samp = L.samp;
#endif
    wave_sync();  // the CDF row is read by every search above before it is reused
    if (ub == 0) {
      // merge by the bin hint: sample j's rank in t starts at its lower bin i0 + 1 (t[i0] <=
      // bins[i0] <= sample); t fills the remaining slots in order (per-row ballot + popcount)
      uint8_t* filled = reinterpret_cast<uint8_t*>(L.cdf);
      for (int p = q; p < kNo; p += 16) filled[p] = 0;
      wave_sync();
      // t[i0] <= bins[i0] <= s <= bins[i0 + 1] <= t[i0 + 2]: the rank is i0 + 1 .. i0 + 3 --
      // t[c - 1 .. c + 2] read at once, the two steps as selects; pdf_ray's fallback rule (t[c - 1]
      // > s, which a NaN sample never meets) or a third step still possible takes the search
      int pos[8];
      bool slow = false;
#pragma unroll
      for (int h = 0; h < 8; h += 4) {
        float ta[4], tb[4], tc[4], td[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = hint[h + e] + 1;  // 1 .. 64
          ta[e] = L.tm[c - 1];
          tb[e] = L.tm[c];
          tc[e] = L.tm[c + 1 < kS ? c + 1 : kS - 1];
          td[e] = L.tm[c + 2 < kS ? c + 2 : kS - 1];
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int n = h + e;
          const float sv = smp[n];
          const int c = hint[n] + 1;
          const bool s1 = c < kS && tb[e] <= sv;
          const bool s2 = s1 && c + 1 < kS && tc[e] <= sv;
          const bool s3 = s2 && c + 2 < kS && td[e] <= sv;
          const bool bad = ta[e] > sv || s3;
          pos[n] = 16 * n + q + c + (s1 ? 1 : 0) + (s2 ? 1 : 0);
          if (bad) pos[n] = -1;
          slow |= bad;
        }
      }
      if (__builtin_amdgcn_ballot_w64(slow)) {  // (never on rows whose bins are t's mids)
#pragma unroll
        for (int n = 0; n < 8; ++n)
          if (pos[n] < 0) pos[n] = 16 * n + q + count_le(L.tm, kS, smp[n]);
      }
#pragma unroll
      for (int n = 0; n < 8; ++n) {
        filled[pos[n]] = 1;
        if (!AON_MARCH_DIRECT || valid) orow[pos[n]] = smp[n];
      }
      wave_sync();
      // the remaining slots take t in order: slot p's rank among the row's empty slots from a
      // per-row ballot + popcount, all 13 blocks of 16 slots' flags read at once
      constexpr int kBlk = (kNo + 15) / 16;
      int carry = 0;
      const uint32_t below = (1u << q) - 1u;
#pragma unroll
      for (int i0 = 0; i0 < kBlk; i0 += 7) {  // two passes of <= 7 blocks (register budget)
        uint32_t fl[7];
        int rank[7];
        float tvv[7];
#pragma unroll
        for (int e = 0; e < 7; ++e) {
          const int i = i0 + e;
          fl[e] = (i < kBlk && 16 * i + q < kNo) ? filled[16 * i + q] : 1u;
        }
#pragma unroll
        for (int e = 0; e < 7; ++e) {
          const uint32_t m = static_cast<uint32_t>(__builtin_amdgcn_ballot_w64(fl[e] == 0) >> (16 * row)) & 0xFFFFu;
          rank[e] = fl[e] == 0 ? carry + __builtin_popcount(m & below) : -1;
          carry += __builtin_popcount(m);
        }
#pragma unroll
        for (int e = 0; e < 7; ++e) tvv[e] = L.tm[rank[e] < 0 ? 0 : rank[e]];
#pragma unroll
        for (int e = 0; e < 7; ++e)
          if (rank[e] >= 0 && (!AON_MARCH_DIRECT || valid)) orow[16 * (i0 + e) + q] = tvv[e];
      }
    } else {
      // some ray of the wave needs the sort: bitonic sort of every row's 128 samples (a sorted
      // row is left bit for bit as it is), then the merge by searches
#pragma unroll
      for (int n = 0; n < 8; ++n) samp[16 * n + q] = smp[n];
      wave_sync();
      for (int k = 2; k <= kNs; k <<= 1) {
        for (int jj = k >> 1; jj > 0; jj >>= 1) {
          for (int i = q; i < kNs; i += 16) {
            const int p = i ^ jj;
            if (p > i) {
              const float a = samp[i], b = samp[p];
              const bool up = (i & k) == 0;
              if ((a > b) == up) {
                samp[i] = b;
                samp[p] = a;
              }
            }
          }
          wave_sync();
        }
      }
      for (int j = q; j < kNs; j += 16) {
        const float s = samp[j];
        if (!AON_MARCH_DIRECT || valid) orow[j + count_le(L.tm, kS, s)] = s;
      }
      for (int i = q; i < kS; i += 16) {
        const float tvv = L.tm[i];
        if (!AON_MARCH_DIRECT || valid) orow[i + count_lt(samp, kNs, tvv)] = tvv;
      }
    }
    wave_sync();
#if !AON_MARCH_DIRECT
    // the four merged rows leave as one contiguous run
    const int64_t nvalid = B - 4 * grp < 4 ? B - 4 * grp : 4;
    float* og = t_out + 4 * grp * kNo;
    const int n_out = static_cast<int>(nvalid) * kNo;
    for (int i = lane; i < n_out; i += 64) og[i] = WL.orow[i];
    wave_sync();  // LDS reuse by this wave's next group
#endif
  }
}

}  // namespace rowm

#ifndef AON_MARCH_ROWS
#define AON_MARCH_ROWS 1  // 0: the one-ray-per-wave kernel for the render's S = 65 / Ns = 128 too
#endif

template <int NB, int SC, int NBX>
static void launch_march(hipStream_t st, const float* raw, const float* t, const float* dirs,
                         int64_t B, int S, int white, int act, const float* u, int64_t u_stride,
                         int Ns, int p2, float* comp, float* acc, float* w, float* depth,
                         float* t_out) {
  hipLaunchKernelGGL((k_composite_march<NB, SC, NBX>), grid_for(B, kCompWaves, 1 << 16),
                     64 * kCompWaves, 0, st, raw, t, dirs, B, S, white, act, u, u_stride, Ns, p2,
                     comp, acc, w, depth, t_out);
}

}  // namespace aon

using namespace aon;

extern "C" int aon_composite_march(const float* raw, const float* t, const float* dirs, int64_t B,
                                   int S, int white_bkgd, int act, const float* u,
                                   int64_t u_stride, int Ns, float* comp_rgb, float* acc,
                                   float* weights, float* depth, float* t_fine,
                                   aon_stream_t stream) {
  AON_REQUIRE(raw && t && dirs && u && comp_rgb && acc && depth && t_fine, "null pointer");
  AON_REQUIRE(aligned16(raw), "raw must be a 16-byte aligned (B*S, 4) [r, g, b, sigma] array");
  AON_REQUIRE(B >= 0 && S >= 3 && S <= 256 && Ns >= 1 && Ns <= 256, "bad shape (3 <= S, Ns <= 256)");
  AON_REQUIRE(act >= AON_ACT_NONE && act <= AON_ACT_ARTIC, "bad activation");
  if (B == 0) return 0;
  int p2 = 1;
  while (p2 < Ns) p2 <<= 1;
  const int need = S > p2 ? S : p2;  // LDS rows: t_merge (S), bins (S - 1), padded samples
  const int nbx = need <= 64 ? 1 : (need <= 128 ? 2 : 4);
  const int nb = (S + 63) / 64;
  hipStream_t st = (hipStream_t)stream;
#define AON_MARCH(NB_, SC_, NBX_)                                                                 \
  launch_march<NB_, SC_, NBX_>(st, raw, t, dirs, B, S, white_bkgd, act, u, u_stride, Ns, p2,      \
                               comp_rgb, acc, weights, depth, t_fine)
  if (AON_MARCH_ROWS && S == rowm::kS && Ns == rowm::kNs && B * rowm::kNo < (int64_t(1) << 31) &&
      (u_stride == 0 || B * u_stride < (int64_t(1) << 31))) {
    // the render's coarse level (64 + 1 samples, 128 fine): four rays per wave
    const int64_t groups = (B + 3) / 4;
#define AON_ROWS(A_)                                                                              \
  hipLaunchKernelGGL(rowm::k_march_rows<A_>,                                                      \
                     AON_MARCH_PIPE ? resident_grid(rowm::k_march_rows<A_>, 64 * rowm::kWaves,     \
                                                    (groups + rowm::kWaves - 1) / rowm::kWaves)    \
                                    : grid_for(groups, rowm::kWaves, 1 << 16),                     \
                     64 * rowm::kWaves, 0, st, raw, t, dirs, B, white_bkgd, u, u_stride, comp_rgb, \
                     acc, weights, depth, t_fine)
    if (act == AON_ACT_NONE) AON_ROWS(AON_ACT_NONE);
    else if (act == AON_ACT_VANILLA) AON_ROWS(AON_ACT_VANILLA);
    else AON_ROWS(AON_ACT_ARTIC);
#undef AON_ROWS
  } else if (S == 65 && nbx == 2) {
    AON_MARCH(2, 65, 2);  // S = 65 with other fine counts: 64 + 1 samples
  } else {
#define AON_MARCH_NBX(NB_)                     \
  if (nbx == 1) AON_MARCH(NB_, 0, 1);          \
  else if (nbx == 2) AON_MARCH(NB_, 0, 2);     \
  else AON_MARCH(NB_, 0, 4);
    switch (nb) {
      case 1: AON_MARCH_NBX(1) break;
      case 2: AON_MARCH_NBX(2) break;
      case 3: AON_MARCH_NBX(3) break;
      default: AON_MARCH_NBX(4) break;
    }
#undef AON_MARCH_NBX
  }
#undef AON_MARCH
  return launch_status(__func__);
}
