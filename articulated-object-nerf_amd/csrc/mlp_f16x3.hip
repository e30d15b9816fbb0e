// Fused NeRFMLP forward on fp16 MFMA with a 3-product hi/lo split ("fp16x3").
//
// Every operand x is carried as x_hi = fp16(x) and x_lo = fp16((x - x_hi) * 2^11): together
// ~22 significant bits.  A weight-activation product is w_hi*x_hi + 2^-11 (w_hi*x_lo + w_lo*x_hi)
// (the dropped w_lo*x_lo term is 2^-22 relative), each on v_mfma_f32_16x16x32_f16 with fp32
// accumulation into two accumulators (hi*hi, and the 2^11-scaled cross terms).  That is 3 fp16
// MFMAs per 32-deep k-step where the fp32 path needs 8 v_mfma_f32_16x16x4_f32 of twice the
// cycles: 16/3 = 5.3x the arithmetic rate at fp32-class accuracy (measured against the
// reference in tests/test_gpu_parity.py).  Activations and biases are carried at 2^-8 scale so
// fp16 cannot overflow below |x| = 1.6e7; the scaling is exact (powers of two).
//
// Structure (mlp_layout.hpp kLayersH): feature-major tiles as in mlp.hip; a wave owns 16*NCOL
// samples; output tiles are produced in pairs (u, u+1) whose accumulators, converted in the
// epilogue, ARE the next layer's B operand for one 32-feature k-step (lane group g holds rows
// 4g..4g+3 of both tiles) -- no LDS round trip; the epilogue of pair p overlaps the MFMAs of
// pair p+1.  Weights stream through the same chunked LDS pipeline (mlp_pipe.hpp).
#include "aon_common.hpp"
#include "mlp_layout.hpp"
#include "mlp_pipe.hpp"

namespace aon {
namespace mlp {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));

#ifndef AON_FMA_MIX
#define AON_FMA_MIX 1
#endif

__device__ __forceinline__ f4 mfma16(h8 a, h8 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ h8 as_h8(f4 v) { return __builtin_bit_cast(h8, v); }

// fp32 value (already at activation scale) -> (hi, lo) fp16 pair: V2 lo = x - hi (exact in
// fp32, normal in fp16 for |x| >= 2^-3 at scale); V1 lo = (x - hi) * 2^11
__device__ __forceinline__ _Float16 lo_of(float v, _Float16 h) {
#if AON_F16X3_V2
  // v - hi is exact in fp32; as an fma with the fp16 operand widened in the instruction it can
  // issue as one v_fma_mix_f32 instead of v_cvt_f32_f16 + v_sub_f32
  return static_cast<_Float16>(__builtin_fmaf(static_cast<float>(h), -1.0f, v));
#else
  return static_cast<_Float16>(__fmul_rn(__fsub_rn(v, static_cast<float>(h)), kLoScale));
#endif
}

// 8 fp32 values (already at activation scale) -> (hi, lo) fp16 fragments
__device__ __forceinline__ void split8(const float (&v)[8], h8& hi, h8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const _Float16 h = static_cast<_Float16>(v[j]);
    hi[j] = h;
    lo[j] = lo_of(v[j], h);
  }
}

// One-step-ahead fragment prefetch over the weight stream: blocks are consumed strictly in
// stream order (2 per (u, k-step)), so the step after block b is always b + 2.  The hi/lo pair
// of the NEXT step is read from LDS before the MFMAs of the current step are issued, hiding the
// LDS latency behind 3*NCOL MFMAs (hipcc issues ds_read -> lgkmcnt(0) -> MFMA otherwise).
#ifndef AON_SCHED_MASK
#define AON_SCHED_MASK 0
#endif

#ifndef AON_PREFETCH
#define AON_PREFETCH 2
#endif

template <typename P, int D = AON_PREFETCH>
struct FragPipe {
  P& p;
  f4 nh[D], nl[D];  // fragments of the next D steps
  __device__ __forceinline__ explicit FragPipe(P& pp) : p(pp) {}
  __device__ __forceinline__ void fetch_into(int blk, f4& h, f4& l) {
    if (blk >= kBlocks) return;
#ifdef AON_ABLATE_LDS  // timing-only build: reuse the first fragments (no LDS reads, wrong results)
    if (blk >= 2 * D) {
      if (blk % P::kChunk == 0) p.begin(blk / P::kChunk);
      return;
    }
#endif
    if (blk % P::kChunk == 0) p.begin(blk / P::kChunk);
    h = p.block(blk);
    l = p.block(blk + 1);
  }
  __device__ __forceinline__ void start() {
#pragma unroll
    for (int i = 0; i < D; ++i) fetch_into(2 * i, nh[i], nl[i]);
  }
  // fragments of block pair `blk` (fetched D steps earlier); prefetches blk + 2D
  __device__ __forceinline__ void take(int blk, h8& wh, h8& wl) {
    wh = as_h8(nh[0]);
    wl = as_h8(nl[0]);
#pragma unroll
    for (int i = 0; i + 1 < D; ++i) {
      nh[i] = nh[i + 1];
      nl[i] = nl[i + 1];
    }
    fetch_into(blk + 2 * D, nh[D - 1], nl[D - 1]);
    // keep the prefetch reads above this step's MFMAs (hipcc otherwise sinks them to their use)
    __builtin_amdgcn_sched_barrier(AON_SCHED_MASK);
  }
};

template <int N, int NCOL>
struct Frag {
  h8 hi[N][NCOL], lo[N][NCOL];
};

// epilogue of a finished pair, in 4 parts of 2 values (so it can ride between MFMA steps):
// part q converts v[2q], v[2q+1] of the pair's 8 per-lane values (v[4uu + r] = tile uu, reg r)
template <bool RELU, int NCOL, int NO>
__device__ __forceinline__ void epi_part(int q, const f4 (&hh)[2][NCOL], const f4 (&xx)[2][NCOL],
                                         const f4 (&bias)[2], Frag<NO, NCOL>& out, int pr) {
  const int uu = q >> 1, r0 = (q & 1) * 2;
#pragma unroll
  for (int c = 0; c < NCOL; ++c) {
    float vv[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
#if AON_F16X3_V2
      // one accumulator at scale 2^9 -> activation scale 2^3, plus the (pre-scaled) bias
      float v = fmaf(hh[uu][c][r0 + e], 1.0f / kWS, bias[uu][r0 + e]);
      (void)xx;
#else
      float v = fmaf(xx[uu][c][r0 + e], 1.0f / kLoScale, hh[uu][c][r0 + e]);
      (void)bias;
#endif
      if (RELU) v = fmaxf(v, 0.0f);
      vv[e] = v;
    }
#if AON_F16X3_V2 && AON_FMA_MIX
    // hi pair by one v_cvt_pk_f16_f32; lo_e = v_e - hi_e by v_fma_mix_f32 reading the fp16 half
    // in place (exact in fp32), then one more cvt_pk
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    const h2 hp = {static_cast<_Float16>(vv[0]), static_cast<_Float16>(vv[1])};
    const uint32_t hu = __builtin_bit_cast(uint32_t, hp);
    float d0, d1;
    asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(d0) : "v"(hu), "v"(vv[0]));
    asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(d1) : "v"(hu), "v"(vv[1]));
    out.hi[pr][c][2 * q] = hp[0];
    out.hi[pr][c][2 * q + 1] = hp[1];
    out.lo[pr][c][2 * q] = static_cast<_Float16>(d0);
    out.lo[pr][c][2 * q + 1] = static_cast<_Float16>(d1);
#else
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const _Float16 h = static_cast<_Float16>(vv[e]);
      out.hi[pr][c][2 * q + e] = h;
      out.lo[pr][c][2 * q + e] = lo_of(vv[e], h);
    }
#endif
  }
}

// one layer with U >= 2 output tiles: out = act(W . [a ; b] + bias) as next-layer fragments.
// Pair p's epilogue is spread over the first k-steps of pair p+1 (compute[cur] || finish[prev]).
template <int LAYER, bool RELU, typename P, int NCOL, int NA, int NB, int NO>
__device__ __forceinline__ void layer_h(P& p, const Frag<NA, NCOL>& a,
                                        const Frag<NB, NCOL>& b, Frag<NO, NCOL>& out,
                                        const float* bias_s, int g) {
  constexpr LayerDesc d = kLayersH[LAYER];
  constexpr int K = d.ka + d.kb;
  constexpr int NP = d.u / 2;
  static_assert(d.u % 2 == 0 && NP <= NO && d.ka <= NA && d.kb <= NB, "layer shape");
  f4 phh[2][NCOL], pxx[2][NCOL];  // accumulators of the pair whose epilogue is pending
  f4 pbias[2];                     // V2: that pair's biases, added in its epilogue
#pragma unroll
  for (int pr = 0; pr < NP; ++pr) {
    f4 hh[2][NCOL], xx[2][NCOL], bias[2];
#pragma unroll
    for (int uu = 0; uu < 2; ++uu) {
      bias[uu] = *reinterpret_cast<const f4*>(bias_s + d.bias0 + 16 * (2 * pr + uu) + 4 * g);
#pragma unroll
      for (int c = 0; c < NCOL; ++c) {
#if AON_F16X3_V2
        hh[uu][c] = f4{0.f, 0.f, 0.f, 0.f};  // bias joins in the epilogue: no LDS read to wait on
#else
        hh[uu][c] = bias[uu];
#endif
        xx[uu][c] = f4{0.f, 0.f, 0.f, 0.f};
      }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
#pragma unroll
      for (int uu = 0; uu < 2; ++uu) {
        const int blk = d.blk0 + 2 * ((pr * K + k) * 2 + uu);
        h8 wh, wl;
        p.take(blk, wh, wl);
#pragma unroll
        for (int c = 0; c < NCOL; ++c) {
          const int ia = k < NA ? k : 0, ib = (k >= d.ka && k - d.ka < NB) ? k - d.ka : 0;
          const h8 xh = k < d.ka ? a.hi[ia][c] : b.hi[ib][c];
          const h8 xl = k < d.ka ? a.lo[ia][c] : b.lo[ib][c];
#if AON_F16X3_V2
          hh[uu][c] = mfma16(wh, xh, hh[uu][c]);
          hh[uu][c] = mfma16(wh, xl, hh[uu][c]);
          hh[uu][c] = mfma16(wl, xh, hh[uu][c]);
#else
          hh[uu][c] = mfma16(wh, xh, hh[uu][c]);
          xx[uu][c] = mfma16(wh, xl, xx[uu][c]);
          xx[uu][c] = mfma16(wl, xh, xx[uu][c]);
#endif
        }
      }
      if (pr > 0 && k < 4) epi_part<RELU>(k, phh, pxx, pbias, out, pr - 1);
    }
    if (pr > 0) {
#pragma unroll
      for (int q = K; q < 4; ++q) epi_part<RELU>(q, phh, pxx, pbias, out, pr - 1);
    }
#pragma unroll
    for (int uu = 0; uu < 2; ++uu) {
      pbias[uu] = bias[uu];
#pragma unroll
      for (int c = 0; c < NCOL; ++c) {
        phh[uu][c] = hh[uu][c];
        pxx[uu][c] = xx[uu][c];
      }
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) epi_part<RELU>(q, phh, pxx, pbias, out, NP - 1);
}

// single-tile head (density / rgb): returns the 16-row tile at activation scale
template <int LAYER, typename P, int NCOL, int NA>
__device__ __forceinline__ void head_h(P& p, const Frag<NA, NCOL>& a, f4 (&res)[NCOL],
                                       const float* bias_s, int g) {
  constexpr LayerDesc d = kLayersH[LAYER];
  static_assert(d.u == 1 && d.kb == 0 && d.ka <= NA, "head shape");
  f4 hh[NCOL], xx[NCOL];
  const f4 bias = *reinterpret_cast<const f4*>(bias_s + d.bias0 + 4 * g);
#pragma unroll
  for (int c = 0; c < NCOL; ++c) {
#if AON_F16X3_V2
    hh[c] = f4{0.f, 0.f, 0.f, 0.f};
#else
    hh[c] = bias;
#endif
    xx[c] = f4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int k = 0; k < d.ka; ++k) {
    const int blk = d.blk0 + 2 * k;
    h8 wh, wl;
    p.take(blk, wh, wl);
#pragma unroll
    for (int c = 0; c < NCOL; ++c) {
#if AON_F16X3_V2
      hh[c] = mfma16(wh, a.hi[k][c], hh[c]);
      hh[c] = mfma16(wh, a.lo[k][c], hh[c]);
      hh[c] = mfma16(wl, a.hi[k][c], hh[c]);
#else
      hh[c] = mfma16(wh, a.hi[k][c], hh[c]);
      xx[c] = mfma16(wh, a.lo[k][c], xx[c]);
      xx[c] = mfma16(wl, a.hi[k][c], xx[c]);
#endif
    }
  }
#pragma unroll
  for (int c = 0; c < NCOL; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#if AON_F16X3_V2
      res[c][r] = fmaf(hh[c][r], 1.0f / (kWS * kActS), bias[r]);  // true scale (head bias unscaled)
#else
      res[c][r] = fmaf(xx[c][r], 1.0f / kLoScale, hh[c][r]);
#endif
}

#ifndef AON_RING
#define AON_RING 3
#endif
#ifndef AON_CHUNK_H
#define AON_CHUNK_H 32
#endif
constexpr int kRing = AON_RING;      // LDS-DMA ring depth (chunks in LDS)
constexpr int kChunkH = AON_CHUNK_H;  // 1-KB blocks per chunk
// Weight pipeline: the LDS-DMA ring, or (AON_PIPE_REG) the register-staged double buffer.
// hipcc drains lgkmcnt to 0 before every LDS read while any global_load_lds is in flight, which
// defeats the fragment prefetch; the register-staged pipe keeps precise lgkmcnt(N) waits.
#ifdef AON_PIPE_REG
template <int THREADS>
using WeightPipe = Pipe<THREADS>;
constexpr int kLdsWeights = 2 * kChunk * 64;  // f4
#else
template <int THREADS>
using WeightPipe = DmaPipe<THREADS, kRing, kChunkH>;
constexpr int kLdsWeights = kRing * kChunkH * 64;
#endif

template <int NCOL>
struct GeomH {
  static constexpr int kWaves = NCOL == 1 ? 8 : 4;
  static constexpr int kThreads = 64 * kWaves;
  static constexpr int kRowsPerWave = 16 * NCOL;
  static constexpr int kRowsPerBlock = kRowsPerWave * kWaves;
};

// MODE 0: (rays_o, rays_d, viewdirs, t) inputs; MODE 1: encoded x (N, 63), condition (B, 27)
template <int MODE, int NCOL>
__global__ __launch_bounds__(GeomH<NCOL>::kThreads, NCOL == 1 ? 2 : 1) void k_mlp_fwd_f16x3(
    const f4* __restrict__ wstream, const float* __restrict__ bias_g, const float* __restrict__ in0,
    const float* __restrict__ in1, const float* __restrict__ in2, const float* __restrict__ in3,
    int64_t B, int S, int act, float* __restrict__ raw) {
  using G = GeomH<NCOL>;
  // ONE __shared__ object: weight ring | bias table | per-lane stash of the encodings
  constexpr int kStash = G::kWaves * 64 * 6 * NCOL;  // f4: enc 2 k-steps + venc 1, hi & lo
  __shared__ f4 smem[kLdsWeights + kBiasFloats / 4 + kStash];
  float* bias_s = reinterpret_cast<float*>(smem + kLdsWeights);
  f4* stash = smem + kLdsWeights + kBiasFloats / 4 + (threadIdx.x >> 6) * 64 * 6 * NCOL +
              (threadIdx.x & 63);  // lane-private slots: written and read by the same lane

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, j = lane & 15;
  const int64_t N = B * S;

  WeightPipe<G::kThreads> p;
  p.wbuf = smem;
  p.src = wstream;
  p.tid = tid;
  p.lane = lane;
  p.start();
  for (int i = tid; i < kBiasFloats; i += G::kThreads) bias_s[i] = bias_g[i];

  // layer-0 (enc) and view-layer (enc_dir) fragments: k-step k, lane group g, element e
  // <-> feature 32k + 8g + e of the encoding
  Frag<2, NCOL> enc;
  Frag<1, NCOL> venc;
  int64_t rows[NCOL];
#pragma unroll
  for (int c = 0; c < NCOL; ++c) {
    const int64_t row = (int64_t)blockIdx.x * G::kRowsPerBlock + wave * G::kRowsPerWave + 16 * c + j;
    rows[c] = row;
    const int64_t rr = row < N ? row : N - 1;
    const int64_t ray = rr / S;
    float ev[2][8], vv[8];
    if (MODE == 0) {
      const float* ro = in0 + 3 * ray;
      const float* rd = in1 + 3 * ray;
      const float* vd = in2 + 3 * ray;
      const float tt = in3[rr];
      const float x0 = __fadd_rn(ro[0], __fmul_rn(tt, rd[0]));
      const float x1 = __fadd_rn(ro[1], __fmul_rn(tt, rd[1]));
      const float x2 = __fadd_rn(ro[2], __fmul_rn(tt, rd[2]));
#pragma unroll
      for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int e = 0; e < 8; ++e) ev[k][e] = pos_enc_feature(x0, x1, x2, 32 * k + 8 * g + e, 0, 10);
#pragma unroll
      for (int e = 0; e < 8; ++e) vv[e] = pos_enc_feature(vd[0], vd[1], vd[2], 8 * g + e, 0, 4);
    } else {
      const float* x = in0 + rr * 63;
      const float* cd = in1 + ray * 27;
#pragma unroll
      for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int f = 32 * k + 8 * g + e;
          ev[k][e] = f < 63 ? x[f] : 0.f;
        }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int f = 8 * g + e;
        vv[e] = f < 27 ? cd[f] : 0.f;
      }
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
#pragma unroll
      for (int e = 0; e < 8; ++e) ev[k][e] *= (AON_F16X3_V2 ? kActS : kActScale);
      split8(ev[k], enc.hi[k][c], enc.lo[k][c]);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) vv[e] *= (AON_F16X3_V2 ? kActS : kActScale);
    split8(vv, venc.hi[0][c], venc.lo[0][c]);
  }

  // park the encodings in LDS until the skip / view layers need them (frees 24 VGPRs for the
  // fragment prefetch); only the owning lane ever touches its slots
#pragma unroll
  for (int c = 0; c < NCOL; ++c) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      stash[64 * (6 * c + 2 * k)] = __builtin_bit_cast(f4, enc.hi[k][c]);
      stash[64 * (6 * c + 2 * k + 1)] = __builtin_bit_cast(f4, enc.lo[k][c]);
    }
    stash[64 * (6 * c + 4)] = __builtin_bit_cast(f4, venc.hi[0][c]);
    stash[64 * (6 * c + 5)] = __builtin_bit_cast(f4, venc.lo[0][c]);
  }

  FragPipe<WeightPipe<G::kThreads>> fp(p);
  fp.start();  // begin(0): chunk 0 landed; the barrier also publishes bias_s

  Frag<8, NCOL> x, y;
  Frag<1, NCOL> none;
  layer_h<L0, true>(fp, none, enc, x, bias_s, g);
  layer_h<L1, true>(fp, x, none, y, bias_s, g);
  layer_h<L2, true>(fp, y, none, x, bias_s, g);
  layer_h<L3, true>(fp, x, none, y, bias_s, g);
  layer_h<L4, true>(fp, y, none, x, bias_s, g);
#pragma unroll
  for (int c = 0; c < NCOL; ++c)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      enc.hi[k][c] = __builtin_bit_cast(h8, stash[64 * (6 * c + 2 * k)]);
      enc.lo[k][c] = __builtin_bit_cast(h8, stash[64 * (6 * c + 2 * k + 1)]);
    }
  layer_h<L5, true>(fp, x, enc, y, bias_s, g);  // skip: cat[h, enc] (model.py:102-103)
  layer_h<L6, true>(fp, y, none, x, bias_s, g);
  layer_h<L7, true>(fp, x, none, y, bias_s, g);
  f4 dens[NCOL], rgb[NCOL];
  head_h<LDEN>(fp, y, dens, bias_s, g);             // model.py:105-107
  layer_h<LBOT, false>(fp, y, none, x, bias_s, g);  // bottleneck, no activation (model.py:109)
#pragma unroll
  for (int c = 0; c < NCOL; ++c) {
    venc.hi[0][c] = __builtin_bit_cast(h8, stash[64 * (6 * c + 4)]);
    venc.lo[0][c] = __builtin_bit_cast(h8, stash[64 * (6 * c + 5)]);
  }
  layer_h<LVIEW, true>(fp, x, venc, y, bias_s, g);  // cat[bottleneck, enc_dir] + ReLU (:110-116)
  head_h<LRGB>(fp, y, rgb, bias_s, g);              // model.py:118

  if (g == 0) {
#pragma unroll
    for (int c = 0; c < NCOL; ++c) {
      if (rows[c] < N) {
        const float s = AON_F16X3_V2 ? 1.0f : 1.0f / kActScale;  // V2 heads are at true scale
        const f4 o = {act_rgb(rgb[c][0] * s, act), act_rgb(rgb[c][1] * s, act),
                      act_rgb(rgb[c][2] * s, act), act_sigma(dens[c][0] * s, act)};
        *reinterpret_cast<f4*>(raw + 4 * rows[c]) = o;
      }
    }
  }
}

// ---- packing: torch [out][in] fp32 -> hi/lo fp16 blocks (+ biases at activation scale)
__global__ void k_pack_f16x3(PackArgs a, float* __restrict__ out_f) {
  const int64_t nhalf = (int64_t)kStreamBlocks * 512;  // fp16 elements of the stream
  _Float16* out = reinterpret_cast<_Float16*>(out_f);
  float* bias_out = out_f + (int64_t)kStreamBlocks * 256;
  const int64_t total = nhalf + kBiasFloats;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    if (e < nhalf) {
      const int blk = static_cast<int>(e >> 9);
      const int l = static_cast<int>((e >> 3) & 63), jj = static_cast<int>(e & 7);
      float w = 0.f;
      bool lo_part = false;
      if (blk < kBlocks) {
        int li = 0;
        while (li + 1 < kNumLayers && a.layers[li + 1].blk0 <= blk) ++li;
        const LayerDesc d = a.layers[li];
        const int K = d.ka + d.kb;
        const int q = (blk - d.blk0) >> 1;
        lo_part = ((blk - d.blk0) & 1) != 0;
        int u, k;
        if (d.u == 1) {
          u = 0;
          k = q;
        } else {
          u = 2 * ((q >> 1) / K) + (q & 1);
          k = (q >> 1) % K;
        }
        const int o = 16 * u + (l & 15), gg = l >> 4;
        int col = -1;
        if (k < d.ka) {  // previous-layer output fragment order
          const int f = 32 * k + 16 * (jj >> 2) + 4 * gg + (jj & 3);
          col = f < d.len_a ? f : -1;
        } else {  // in-register encodings: natural order
          const int f = 32 * (k - d.ka) + 8 * gg + jj;
          col = f < d.len_b ? d.len_a + f : -1;
        }
        if (o < d.out_real && col >= 0) w = a.w[li][(int64_t)o * (d.len_a + d.len_b) + col];
      }
#if AON_F16X3_V2
      w *= kWS;  // exact (power of two)
      const _Float16 h = static_cast<_Float16>(w);
      out[e] = lo_part ? static_cast<_Float16>(w - static_cast<float>(h)) : h;
#else
      const _Float16 h = static_cast<_Float16>(w);
      out[e] = lo_part ? static_cast<_Float16>((w - static_cast<float>(h)) * kLoScale) : h;
#endif
    } else {
      const int i = static_cast<int>(e - nhalf);
      int li = 0;
      while (li + 1 < kNumLayers && a.layers[li + 1].bias0 <= i) ++li;
      const int o = i - a.layers[li].bias0;
#if AON_F16X3_V2
      // hidden layers add the bias at activation scale; the 1-tile heads at true scale
      const float bs = a.layers[li].u == 1 ? 1.0f : kActS;
#else
      const float bs = kActScale;
#endif
      bias_out[i] = o < a.layers[li].out_real ? a.b[li][o] * bs : 0.f;
    }
  }
}

int pack_f16x3(const PackArgs& a, void* packed, hipStream_t stream) {
  const int64_t total = (int64_t)kStreamBlocks * 512 + kBiasFloats;
  hipLaunchKernelGGL(k_pack_f16x3, grid_for(total, 256, 4096), 256, 0, stream, a,
                     static_cast<float*>(packed));
  return launch_status("aon_mlp_pack");
}

int launch_f16x3(int mode, int ncol, const void* packed, const float* a0, const float* a1,
                 const float* a2, const float* a3, int64_t B, int S, int act, float* raw,
                 hipStream_t stream) {
  const int64_t N = B * S;
  const f4* ws = static_cast<const f4*>(packed);
  const float* bias = reinterpret_cast<const float*>(static_cast<const char*>(packed) + kStreamBytesF32);
#define AON_LAUNCH_H(M, C)                                                                       \
  hipLaunchKernelGGL((k_mlp_fwd_f16x3<M, C>),                                                    \
                     static_cast<int>((N + GeomH<C>::kRowsPerBlock - 1) / GeomH<C>::kRowsPerBlock), \
                     GeomH<C>::kThreads, 0, stream, ws, bias, a0, a1, a2, a3, B, S, act, raw)
  if (mode == 0 && ncol == 1) AON_LAUNCH_H(0, 1);
  else if (mode == 0) AON_LAUNCH_H(0, 2);
  else if (ncol == 1) AON_LAUNCH_H(1, 1);
  else AON_LAUNCH_H(1, 2);
#undef AON_LAUNCH_H
  return launch_status("aon_mlp_fwd");
}

}  // namespace mlp
}  // namespace aon
