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
  if (S == 65 && nbx == 2) {
    AON_MARCH(2, 65, 2);  // the render's coarse level: 64 + 1 samples, 128 fine
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
