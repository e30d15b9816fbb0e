// Inverse-CDF hierarchical sampling (reference models/vanilla_nerf/helper.py:203-252, called
// from models/vanilla_nerf/model.py:163-172).
//
// One 64-lane wave per ray, everything staged in LDS:
//   1. weight_sum by a wave reduction, the eps padding, pdf = w / sum;
//   2. cdf = [0, fmin(1, cumsum(pdf[:-1])), 1] by an fp64 wavefront scan rounded per prefix
//      (torch CPU's cumsum accumulates fp32 in fp64);
//   3. per u: idx = #{cdf <= u} (binary search == the reference's (B,64,128) mask reduction,
//      proven bit-exact in oracle/nerf_oracle.py) and the clipped linear interpolation;
//   4. samples are bitonic-sorted in LDS (randomized u is unsorted) and merged with the sorted
//      coarse t by rank (position = own index + rank in the other list) -- the values equal
//      torch.sort(cat[t, samples]) exactly; xyz = o + t*d optionally.
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

// number of entries of sorted a[0..n) that are <= x  (upper bound)
__device__ __forceinline__ int count_le(const float* a, int n, float x) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] <= x) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// number of entries of sorted a[0..n) that are < x  (lower bound)
__device__ __forceinline__ int count_lt(const float* a, int n, float x) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] < x) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// per-wave LDS, sized for rows of up to 64 * NBX entries (bins, weights, samples, t_merge)
template <int NBX>
struct PdfLds {
  float bins[64 * NBX];
  float cdf[64 * NBX];
  float w[64 * NBX];
  float samp[64 * NBX];
  float tm[64 * NBX];
};

// A ray's inputs -- its t_merge row (or bins), weights and u, NBX 64-entry blocks of each -- are
// read by coalesced wave-wide loads, all issued before any math, and staged in LDS (the weight
// sum reads LDS, not HBM).  One ray per wave on a grid of up to 65,536 workgroups: many short
// waves hide HBM latency better than AON_PDF_PIPE's resident grid with ray r + 1's loads issued
// before ray r's math (measured 0.40 vs 0.43 ms per frame).
template <int NBX>
__global__ __launch_bounds__(64 * kPdfWaves) void k_sample_pdf(
    const float* __restrict__ bins_g, int64_t bins_stride, const float* __restrict__ w_g,
    int64_t w_stride, int64_t B, int nb, int Ns, int Ns_pow2, const float* __restrict__ u_g,
    int64_t u_stride, const float* __restrict__ tm_g, int Nt, const float* __restrict__ ro,
    const float* __restrict__ rd, float* __restrict__ out, float* __restrict__ xyz) {
  __shared__ PdfLds<NBX> lds_all[kPdfWaves];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  PdfLds<NBX>& L = lds_all[wid];
  const int nw = nb - 1;
  const int64_t nwaves = (int64_t)gridDim.x * kPdfWaves;
  // this lane's entries 64 b + lane of t_merge, bins, weights and u: current ray, next ray
  float ct[NBX], cb[NBX], cw[NBX], cu[NBX];
  float pt[NBX], pb[NBX], pw[NBX], pu[NBX];
  auto load_ray = [&](int64_t r, float(&tv)[NBX], float(&bv)[NBX], float(&wv)[NBX],
                      float(&uv)[NBX]) {
#pragma unroll
    for (int b = 0; b < NBX; ++b) {
      const int i = 64 * b + lane;
      tv[b] = tm_g && i < Nt ? tm_g[r * Nt + i] : 0.f;
      bv[b] = bins_g && i < nb ? bins_g[r * bins_stride + i] : 0.f;
      wv[b] = i < nw ? w_g[r * w_stride + i] : 0.f;
      uv[b] = i < Ns ? u_g[r * u_stride + i] : 0.f;
    }
  };
  int64_t ray = (int64_t)blockIdx.x * kPdfWaves + wid;
  if (AON_PDF_PIPE && ray < B) load_ray(ray, ct, cb, cw, cu);
  for (; ray < B; ray += nwaves) {
    if (!AON_PDF_PIPE)
      load_ray(ray, ct, cb, cw, cu);
    else if (ray + nwaves < B)
      load_ray(ray + nwaves, pt, pb, pw, pu);
    // ---- stage t_merge, bins and the weights
#pragma unroll
    for (int b = 0; b < NBX; ++b) {
      const int i = 64 * b + lane;
      if (tm_g && i < Nt) L.tm[i] = ct[b];
      if (bins_g && i < nb) L.bins[i] = cb[b];
      if (i < nw) L.w[i] = cw[b];
    }
    wave_sync();
    if (!bins_g) {  // bins = mids of t_merge (model.py:163)
      for (int k = lane; k < nb; k += 64) L.bins[k] = __fmul_rn(0.5f, __fadd_rn(L.tm[k + 1], L.tm[k]));
    }
    // ---- weight sum (torch CPU order, torch_sum.hpp) + padding (helper.py:206-212)
    const float* w = L.w;
    float part = 0.f;
    if (nw >= 8) {
      if (lane < 8) part = inner_sum_lane([&](int e) { return w[e]; }, nw, lane);
      else if (lane == 8) part = inner_sum_tail([&](int e) { return w[e]; }, nw);
    } else if (lane == 0) {
      part = row_sum_ilp4([&](int e) { return w[e]; }, nw);
    }
    float ws = __shfl(part, nw >= 8 ? 8 : 0);
    if (nw >= 8) {
#pragma unroll
      for (int c = 0; c < 8; ++c) ws = __fadd_rn(ws, __shfl(part, c));
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
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const double x = __shfl_up(v, o);
        if (lane >= o) v += x;
      }
      if (k < nw - 1) L.cdf[k + 1] = fminf(1.0f, (float)(carry + v));
      carry += __shfl(v, 63);
    }
    if (lane == 0) {
      L.cdf[0] = 0.0f;
      L.cdf[nb - 1] = 1.0f;
    }
    wave_sync();
    // ---- inverse cdf (helper.py:232-241)
#pragma unroll
    for (int b = 0; b < NBX; ++b) {
      const int j = 64 * b + lane;
      if (j >= Ns_pow2) break;
      float s = __builtin_inff();  // sort padding
      if (j < Ns) {
        const float uj = cu[b];
        const int idx = count_le(L.cdf, nb, uj);
        const int i0 = idx - 1 < 0 ? 0 : (idx - 1 > nb - 1 ? nb - 1 : idx - 1);
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
    const int No = tm_g ? Nt + Ns : Ns;
    float* o = out + ray * No;
    float ox = 0.f, oy = 0.f, oz = 0.f, dx = 0.f, dy = 0.f, dz = 0.f;
    if (xyz) {
      ox = ro[3 * ray]; oy = ro[3 * ray + 1]; oz = ro[3 * ray + 2];
      dx = rd[3 * ray]; dy = rd[3 * ray + 1]; dz = rd[3 * ray + 2];
    }
    float* xo = xyz ? xyz + ray * No * 3 : nullptr;
    for (int j = lane; j < Ns; j += 64) {
      const float s = L.samp[j];
      const int pos = tm_g ? j + count_le(L.tm, Nt, s) : j;
      o[pos] = s;
      if (xo) {
        xo[3 * pos] = __fadd_rn(ox, __fmul_rn(s, dx));
        xo[3 * pos + 1] = __fadd_rn(oy, __fmul_rn(s, dy));
        xo[3 * pos + 2] = __fadd_rn(oz, __fmul_rn(s, dz));
      }
    }
    if (tm_g) {
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
    wave_sync();  // LDS reuse by the next ray of this wave
    if (AON_PDF_PIPE) {
#pragma unroll
    for (int b = 0; b < NBX; ++b) {
      ct[b] = pt[b];
      cb[b] = pb[b];
      cw[b] = pw[b];
      cu[b] = pu[b];
    }
    }
  }
}

template <int NBX>
static void launch_pdf(hipStream_t st, const float* bins, int64_t bins_stride, const float* w,
                       int64_t w_stride, int64_t B, int nb, int Ns, int p2, const float* u,
                       int64_t u_stride, const float* tm, int Nt, const float* ro,
                       const float* rd, float* out, float* xyz) {
  const int grid = AON_PDF_PIPE
                       ? resident_grid(k_sample_pdf<NBX>, 64 * kPdfWaves, (B + kPdfWaves - 1) / kPdfWaves)
                       : grid_for(B, kPdfWaves, 1 << 16);
  hipLaunchKernelGGL(k_sample_pdf<NBX>, grid, 64 * kPdfWaves, 0, st, bins, bins_stride, w,
                     w_stride, B, nb, Ns, p2, u, u_stride, tm, Nt, ro, rd, out, xyz);
}

}  // namespace aon

using namespace aon;

extern "C" int aon_sample_pdf(const float* bins, int64_t bins_stride, const float* weights,
                              int64_t w_stride, int64_t B, int nb, int Ns, const float* u,
                              int64_t u_stride, const float* t_merge, int Nt,
                              const float* rays_o, const float* rays_d, float* out, float* xyz,
                              aon_stream_t stream) {
  AON_REQUIRE(weights && u && out, "null pointer");
  AON_REQUIRE(B >= 0 && nb >= 2 && nb <= kMaxBins && Ns >= 1 && Ns <= kMaxNs, "bad shape");
  AON_REQUIRE(bins || (t_merge && Nt == nb + 1), "bins == NULL needs t_merge with nb+1 entries");
  AON_REQUIRE(!t_merge || (Nt >= 1 && Nt <= kMaxNt), "bad Nt");
  AON_REQUIRE(!xyz || (rays_o && rays_d), "xyz needs rays_o/rays_d");
  if (B == 0) return 0;
  int p2 = 1;
  while (p2 < Ns) p2 <<= 1;
  // LDS rows of 64 * NBX entries hold the bins, t_merge and the (power-of-two padded) samples
  int need = nb > p2 ? nb : p2;
  if (t_merge && Nt > need) need = Nt;
  const int nbx = need <= 64 ? 1 : (need <= 128 ? 2 : (need <= 256 ? 4 : 8));
  hipStream_t st = (hipStream_t)stream;
  const int nt = t_merge ? Nt : 0;
  switch (nbx) {
    case 1: launch_pdf<1>(st, bins, bins_stride, weights, w_stride, B, nb, Ns, p2, u, u_stride, t_merge, nt, rays_o, rays_d, out, xyz); break;
    case 2: launch_pdf<2>(st, bins, bins_stride, weights, w_stride, B, nb, Ns, p2, u, u_stride, t_merge, nt, rays_o, rays_d, out, xyz); break;
    case 4: launch_pdf<4>(st, bins, bins_stride, weights, w_stride, B, nb, Ns, p2, u, u_stride, t_merge, nt, rays_o, rays_d, out, xyz); break;
    default: launch_pdf<8>(st, bins, bins_stride, weights, w_stride, B, nb, Ns, p2, u, u_stride, t_merge, nt, rays_o, rays_d, out, xyz); break;
  }
  return launch_status(__func__);
}
