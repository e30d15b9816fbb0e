// Inverse-CDF resampling device code (reference models/vanilla_nerf/helper.py:203-252), shared by
// k_sample_pdf (pdf.hip) and the fused coarse composite + resample kernel (march.hip).
#pragma once

#include "aon_common.hpp"
#include "torch_sum.hpp"

namespace aon {

#ifndef AON_PDF_PIPE
#define AON_PDF_PIPE 0  // 1: next ray's inputs loaded one ray ahead on a resident grid (7% slower)
#endif

constexpr int kPdfWaves = 4;
constexpr int kMaxBins = 256;
constexpr int kMaxNs = 512;
constexpr int kMaxNt = 512;

// order this wave's LDS writes before its later LDS reads (lanes exchange data through LDS)
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// Two-level counts in a sorted LDS row, 2 dependent LDS round trips instead of log2(n): the
// every-8th "pivots" a[8m + 7] (the same address on every lane: broadcast reads) give the first
// bucket q whose pivot is not counted; buckets before it count whole, bucket q entry by entry,
// everything after it is past x (sorted).  Equal to the binary searches below for any x
// (NaN x: 0; +inf entries sort last).
template <bool LE>
__device__ __forceinline__ int count_sorted(const float* a, int n, float x) {
  const int nfull = n >> 3;
  int q = 0;
  for (int m = 0; m < nfull; ++m) {
    const float p = a[8 * m + 7];
    q += LE ? (p <= x) : (p < x);
  }
  int c = 8 * q;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int i = 8 * q + e;
    if (i < n) {
      const float v = a[i];
      c += LE ? (v <= x) : (v < x);
    }
  }
  return c;
}

// Branch-free binary lifting: the largest c with a[c-1] <= x (LE) / < x, one probe per power of
// two below n -- a trip count uniform across the wave (no divergent loop exits).  Equal to the
// while-loop searches below on sorted rows (NaN x: 0).
template <bool LE>
__device__ __forceinline__ int count_lift(const float* a, int n, float x) {
  int c = 0;
  if (n <= 0) return 0;
  for (int step = 1 << (31 - __builtin_clz(n)); step > 0; step >>= 1) {
    const int j = c + step;
    const float v = a[(j < n ? j : n) - 1];
    const bool ok = j <= n && (LE ? v <= x : v < x);
    c = ok ? j : c;
  }
  return c;
}

#ifndef AON_PDF_SEARCH2
#define AON_PDF_SEARCH2 2  // 2: count_lift (fused march 0.418 -> 0.394 ms); 1: two-level searches (more LDS reads: 5-15% slower); 0: while-loop binary searches (profiles/r02/ab_march)
#endif

// number of entries of sorted a[0..n) that are <= x  (upper bound)
__device__ __forceinline__ int count_le_bin(const float* a, int n, float x) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] <= x) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// number of entries of sorted a[0..n) that are < x  (lower bound)
__device__ __forceinline__ int count_lt_bin(const float* a, int n, float x) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] < x) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ int count_le(const float* a, int n, float x) {
  return AON_PDF_SEARCH2 == 2 ? count_lift<true>(a, n, x)
         : AON_PDF_SEARCH2 ? count_sorted<true>(a, n, x) : count_le_bin(a, n, x);
}
__device__ __forceinline__ int count_lt(const float* a, int n, float x) {
  return AON_PDF_SEARCH2 == 2 ? count_lift<false>(a, n, x)
         : AON_PDF_SEARCH2 ? count_sorted<false>(a, n, x) : count_lt_bin(a, n, x);
}

#ifndef AON_PDF_HINT_MERGE
#define AON_PDF_HINT_MERGE 1  // 0: merge by binary searches on both sides
#endif

#ifndef AON_PDF_DPP_SCAN
#define AON_PDF_DPP_SCAN 1  // 0: the shuffle (ds_bpermute) scan
#endif

// per-wave LDS, sized for rows of up to 64 * NBX entries (bins, weights, samples, t_merge)
template <int NBX>
struct PdfLds {
  float bins[64 * NBX];
  float cdf[64 * NBX];
  float w[64 * NBX];
  float samp[64 * NBX];
  float tm[64 * NBX];
};

// The resampling of one ray once its LDS rows are staged (L.bins; L.tm when merging; the nb - 1
// weights at w, any LDS row): torch-order weight sum + padding, fp64 CDF scan, inverse CDF per u
// (cu[b] = u[64 b + lane]), the sort when needed, and the (merged) output row o (global, or an
// LDS row the caller copies out); xyz optional.
template <int NBX>
__device__ __forceinline__ void pdf_ray(PdfLds<NBX>& L, const float* w, int nb, int Ns,
                                        int Ns_pow2, const float (&cu)[NBX], bool merge, int Nt,
                                        int64_t ray, int lane, float* __restrict__ o,
                                        float* __restrict__ xyz, const float* __restrict__ ro,
                                        const float* __restrict__ rd) {
  const int nw = nb - 1;
  // ---- weight sum (torch CPU order, torch_sum.hpp) + padding (helper.py:206-212)
  float part = 0.f;
  if (nw >= 8) {
    if (lane < 8) part = inner_sum_lane([&](int e) { return w[e]; }, nw, lane);
    else if (lane == 8) part = inner_sum_tail([&](int e) { return w[e]; }, nw);
  } else if (lane == 0) {
    part = row_sum_ilp4([&](int e) { return w[e]; }, nw);
  }
  // lane partials gathered by v_readlane (SGPR broadcasts; the lane index is uniform)
  auto lane_val = [&](int c) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, part), c));
  };
  float ws = lane_val(nw >= 8 ? 8 : 0);
  if (nw >= 8) {
#pragma unroll
    for (int c = 0; c < 8; ++c) ws = __fadd_rn(ws, lane_val(c));
  }
  const float pad = fmaxf(0.0f, __fsub_rn(1e-5f, ws));
  const float padw = __fdiv_rn(pad, static_cast<float>(nw));
  const float wsum = __fadd_rn(ws, pad);
  // ---- cdf (helper.py:213-223): fp64 scan of pdf[0 .. nw-2]
  double carry = 0.0;
  for (int base = 0; base < nw - 1; base += 64) {
    const int k = base + lane;
    double v = 0.0;
    if (k < nw - 1) v = (double)__fdiv_rn(__fadd_rn(w[k], padw), wsum);
#if AON_PDF_DPP_SCAN
    v = wave_incl_sum(v);  // DPP lane moves, no LDS round trips
#else
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const double x = __shfl_up(v, o);
      if (lane >= o) v += x;
    }
#endif
    if (k < nw - 1) L.cdf[k + 1] = fminf(1.0f, (float)(carry + v));
    carry += readlane_f64(v, 63);
  }
  if (lane == 0) {
    L.cdf[0] = 0.0f;
    L.cdf[nb - 1] = 1.0f;
  }
  wave_sync();
  // ---- inverse cdf (helper.py:232-241)
  int hint[NBX];  // sample j's lower bin i0: t_merge[0 .. i0] <= sample (the merge's start)
#pragma unroll
  for (int b = 0; b < NBX; ++b) {
    const int j = 64 * b + lane;
    hint[b] = 0;
    if (j >= Ns_pow2) break;
    float s = __builtin_inff();  // sort padding
    if (j < Ns) {
      const float uj = cu[b];
      const int idx = count_le(L.cdf, nb, uj);
      const int i0 = idx - 1 < 0 ? 0 : (idx - 1 > nb - 1 ? nb - 1 : idx - 1);
      hint[b] = i0;
      const int i1 = idx > nb - 1 ? nb - 1 : idx;
      const float c0 = L.cdf[i0], c1 = L.cdf[i1];
      const float b0 = L.bins[i0], b1 = L.bins[i1];
      float q = nan_to_num(__fdiv_rn(__fsub_rn(uj, c0), __fsub_rn(c1, c0)), 0.0f);
      q = fminf(fmaxf(q, 0.0f), 1.0f);
      s = __fadd_rn(b0, __fmul_rn(q, __fsub_rn(b1, b0)));
    }
    L.samp[j] = s;
  }
  wave_sync();
  // ---- bitonic sort of the samples (ascending), skipped when they already are (sorted u,
  // e.g. the eval-mode linspace, maps to nondecreasing samples); a NaN compares unordered
  // and keeps the sort on, as before
  bool unsorted = false;
  for (int j = lane; j + 1 < Ns; j += 64) unsorted |= !(L.samp[j] <= L.samp[j + 1]);
  const bool need_sort = __any(unsorted);
  for (int k = 2; need_sort && k <= Ns_pow2; k <<= 1) {
    for (int jj = k >> 1; jj > 0; jj >>= 1) {
      for (int i = lane; i < Ns_pow2; i += 64) {
        const int p = i ^ jj;
        if (p > i) {
          const float a = L.samp[i], b = L.samp[p];
          const bool up = (i & k) == 0;
          if ((a > b) == up) {
            L.samp[i] = b;
            L.samp[p] = a;
          }
        }
      }
      wave_sync();
    }
  }
  // ---- write (merged) output
  const int No = merge ? Nt + Ns : Ns;
  float ox = 0.f, oy = 0.f, oz = 0.f, dx = 0.f, dy = 0.f, dz = 0.f;
  if (xyz) {
    ox = ro[3 * ray]; oy = ro[3 * ray + 1]; oz = ro[3 * ray + 2];
    dx = rd[3 * ray]; dy = rd[3 * ray + 1]; dz = rd[3 * ray + 2];
  }
  float* xo = xyz ? xyz + ray * No * 3 : nullptr;
#if AON_PDF_HINT_MERGE
  if (merge && !need_sort) {
    // Samples in u order are ascending: sample j's bin i0 bounds its rank in t_merge from below
    // (t_merge[i0] <= bins[i0] <= sample, bins = mids of t_merge), and it lies below
    // t_merge[i0 + 2] but for ties, so a short walk replaces the binary search.  The merged
    // row's remaining slots then take t_merge in order: slot p's rank among the empty slots
    // comes from a ballot + mbcnt per 64 slots (no search over the samples).  Same positions as
    // the searches below (ties: count_le / count_lt put samples after equal t, t before).
    uint8_t* filled = reinterpret_cast<uint8_t*>(L.cdf);  // free after the inverse cdf
    for (int p = lane; p < No; p += 64) filled[p] = 0;
    wave_sync();
#pragma unroll
    for (int b = 0; b < NBX; ++b) {
      const int j = 64 * b + lane;
      if (j < Ns) {
        const float s = L.samp[j];
        int c = hint[b] + 1;
        if (c > Nt || L.tm[c - 1] > s) {
          c = count_le(L.tm, Nt, s);  // bins that are not t_merge's mids: no bound, search
        } else {
          while (c < Nt && L.tm[c] <= s) ++c;
        }
        const int pos = j + c;
        filled[pos] = 1;
        o[pos] = s;
        if (xo) {
          xo[3 * pos] = __fadd_rn(ox, __fmul_rn(s, dx));
          xo[3 * pos + 1] = __fadd_rn(oy, __fmul_rn(s, dy));
          xo[3 * pos + 2] = __fadd_rn(oz, __fmul_rn(s, dz));
        }
      }
    }
    wave_sync();
    int carry = 0;  // empty slots before this 64-slot block
    for (int p0 = 0; p0 < No; p0 += 64) {
      const int p = p0 + lane;
      const bool empty = p < No && filled[p] == 0;
      const uint64_t m = __builtin_amdgcn_ballot_w64(empty);
      if (empty) {
        const int rank = carry + __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m >> 32),
                                                           __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), 0));
        const float tv = L.tm[rank];
        o[p] = tv;
        if (xo) {
          xo[3 * p] = __fadd_rn(ox, __fmul_rn(tv, dx));
          xo[3 * p + 1] = __fadd_rn(oy, __fmul_rn(tv, dy));
          xo[3 * p + 2] = __fadd_rn(oz, __fmul_rn(tv, dz));
        }
      }
      carry += __builtin_popcountll(m);
    }
    return;
  }
#endif
  for (int j = lane; j < Ns; j += 64) {
    const float s = L.samp[j];
    const int pos = merge ? j + count_le(L.tm, Nt, s) : j;
    o[pos] = s;
    if (xo) {
      xo[3 * pos] = __fadd_rn(ox, __fmul_rn(s, dx));
      xo[3 * pos + 1] = __fadd_rn(oy, __fmul_rn(s, dy));
      xo[3 * pos + 2] = __fadd_rn(oz, __fmul_rn(s, dz));
    }
  }
  if (merge) {
    for (int i = lane; i < Nt; i += 64) {
      const float tv = L.tm[i];
      const int pos = i + count_lt(L.samp, Ns, tv);
      o[pos] = tv;
      if (xo) {
        xo[3 * pos] = __fadd_rn(ox, __fmul_rn(tv, dx));
        xo[3 * pos + 1] = __fadd_rn(oy, __fmul_rn(tv, dy));
        xo[3 * pos + 2] = __fadd_rn(oz, __fmul_rn(tv, dz));
      }
    }
  }
}

}  // namespace aon
