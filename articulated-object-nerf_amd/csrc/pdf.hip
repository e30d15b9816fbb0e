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
#include "pdf_core.hpp"

namespace aon {

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
    pdf_ray<NBX>(L, L.w, nb, Ns, Ns_pow2, cu, tm_g != nullptr, Nt, ray, lane,
                 out + ray * (tm_g ? Nt + Ns : Ns), xyz, ro, rd);
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
