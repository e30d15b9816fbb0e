// Fused NeRFMLP forward on fp16x3 MFMA, WEIGHT-STREAMED dataflow ("ws") -- the render path's
// alternative to k_mlp_fwd_f16x3 (mlp_f16x3.hip), same numerics, bit-identical outputs.
//
// Why ("Fine MLP: LDS bytes per MAC"): k_mlp_fwd_f16x3 keeps each wave's 16
// samples in registers and streams the WEIGHTS through LDS, so every wave reads the whole 2.37-MB
// stream per 16 samples: 683 B of LDS per MFMA, 19 MB per 128-sample pass per CU -- with the
// ring's DMA writes ~100k LDS cycles against ~112k MFMA cycles.  The LDS is co-critical with the
// matrix cores (MFMA busy 0.69; a build without the fragment reads runs in half the time).
//
// Here the roles swap.  A workgroup (8 waves, 2 per SIMD) owns 128 samples whose activations
// live in LDS (hi / lo planes, 128 KB) and are shared by all its waves; each wave owns 32 OUTPUT
// rows (one pair of 16-row tiles) of a layer and reads its weight fragments straight from the
// packed stream in global memory (L2-resident: every CU reads the same 2.37 MB) into registers.
// Per 32-deep k-step a wave loads 4 KB of A from L2 and 16 KB of B (8 sample tiles, hi + lo) from
// LDS for 48 MFMAs: 341 B of LDS per MFMA (half of the streamed kernel's) and 21 B/clk/CU of
// L2 -> CU traffic.  A layer ends with two barriers: all waves past their reads of the input
// planes -> epilogue (bias, ReLU, fp16 hi/lo split) written in place -> all waves past their
// writes.  The accumulator tile (2 pr + uu, sample tile t) of lane (g, j) holds rows
// 16 (2 pr + uu) + 4 g + r, which are exactly elements 4 uu + r of the next layer's k-step-pr
// B fragment of that lane (the stream's feature order, mlp_layout.hpp) -- the epilogue writes
// each lane's own 16 B, no shuffles.
//
// Accumulation order per output: k-steps in order, hi*hi, hi*lo, lo*hi into ONE fp32 accumulator,
// the same epilogue arithmetic -- every raw value equals k_mlp_fwd_f16x3's bit for bit
// (tests/test_gpu_parity.py::test_mlp_ws_equals_streamed).  MODE 0 (rays + t) inference only;
// selected by AON_MLP_WS (env, mlp.hip) for the A/B.
#include <utility>

#include "mlp_f16x3_core.hpp"

namespace aon {
namespace mlp {
namespace ws {

#ifndef AON_WS_PREFETCH
#define AON_WS_PREFETCH 3  // k-steps of A fragments in flight ahead of the one in use (8 waves)
#endif

// Workgroup geometry.  WAVES = 8: one workgroup of 128 samples per CU (160 KB of LDS), 2 waves
// per SIMD; WAVES = 4: 64 samples (80 KB), two workgroups per CU, one wave of each per SIMD --
// their barriers and epilogues fall at different times, so one workgroup's MFMAs run while the
// other's waves wait (the 8-wave kernel's SIMD-mates reach every barrier and epilogue together).
template <int WAVES>
struct Geo {
  static constexpr int kWaves = WAVES;
  static constexpr int kThreads = 64 * WAVES;
  static constexpr int kTiles = WAVES;              // 16-sample tiles per workgroup pass
  static constexpr int kNb = 16 * kTiles;           // samples per pass
  static constexpr int kActPlane = 8 * 4 * kNb;     // f4: [k-step 8][lane group 4][sample]
  static constexpr int kEncPlane = 2 * 4 * kNb;     // f4: segment B, 2 k-steps
  static constexpr int kLdsF4 = 2 * kActPlane + 2 * kEncPlane;
  static constexpr int kWavesPerSimd = 2;           // __launch_bounds__: 256 VGPRs per wave
  // A-fragment k-steps in flight (AON_WS_PREFETCH): 4 row tiles per wave at WAVES = 4 hold twice
  // the registers per k-step, so one step less fits in 256 VGPRs without spills
  static constexpr int kPrefetch = WAVES == 8 ? AON_WS_PREFETCH : AON_WS_PREFETCH - 1;
  static_assert(kLdsF4 * 16 * (8 / WAVES) <= 160 * 1024, "LDS");
  // the rows a wave computes in a layer of u row tiles: row tiles [rt0, rt0 + TU) over sample
  // tiles [T0, T0 + NT).  Pairs per layer P = u / 2; P >= WAVES: P / WAVES pairs each over every
  // sample tile; P < WAVES: WAVES / P waves share a pair, splitting the sample tiles.
  __host__ __device__ static constexpr int tu(int u) { return u / 2 >= WAVES ? u / WAVES : 2; }
  __host__ __device__ static constexpr int nt(int u) { return u / 2 >= WAVES ? kTiles : kTiles * (u / 2) / WAVES; }
  __host__ __device__ static constexpr int rt0(int u, int w) {
    return u / 2 >= WAVES ? tu(u) * w : 2 * (w % (u / 2));
  }
  __host__ __device__ static constexpr int t0(int u, int w) {
    return u / 2 >= WAVES ? 0 : nt(u) * (w / (u / 2));
  }
};

// The per-wave step sequence of a network: its layers in table order (both layer tables list
// them in execution order), each ka + kb 32-deep k-steps.
template <typename Net>
__host__ __device__ constexpr int layer_k(int l) { return Net::layer(l).ka + Net::layer(l).kb; }
template <typename Net>
__host__ __device__ constexpr int step0_of(int l) { return l == 0 ? 0 : step0_of<Net>(l - 1) + layer_k<Net>(l - 1); }
template <typename Net>
__host__ __device__ constexpr int layer_of_step(int s) {
  int l = 0;
  while (l + 1 < Net::kNumLayers && step0_of<Net>(l + 1) <= s) ++l;
  return l;
}
template <typename Net>
constexpr int kStepsOf = step0_of<Net>(Net::kNumLayers);

// A fragments straight from the packed stream (global, L2-resident), D k-steps ahead: the
// wave's TU row tiles of each k-step (a 1-tile head: tile 0, on every wave).
template <typename Net, typename G, int D>
struct APipe {
  static constexpr int TM = G::tu(16);  // most row tiles a wave holds
  const f4* __restrict__ ws;
  int lane, w;
  f4 qh[D][TM], ql[D][TM];
  __device__ __forceinline__ void fetch(int s, f4 (&h)[TM], f4 (&l)[TM]) {
    if (s >= kStepsOf<Net>) return;
    const int L = layer_of_step<Net>(s);
    const int k = s - step0_of<Net>(L);
    const LayerDesc d = Net::layer(L);
    const int K = d.ka + d.kb;
    if (d.u == 1) {
      const int b = d.blk0 + 2 * k;
      h[0] = ws[(size_t)b * 64 + lane];
      l[0] = ws[(size_t)(b + 1) * 64 + lane];
      return;
    }
    const int r0 = G::rt0(d.u, w);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      if (i >= G::tu(d.u)) break;
      const int u = r0 + i;
      const int b = d.blk0 + 2 * (((u >> 1) * K + k) * 2 + (u & 1));
      h[i] = ws[(size_t)b * 64 + lane];
      l[i] = ws[(size_t)(b + 1) * 64 + lane];
    }
  }
  __device__ __forceinline__ void start() {
#pragma unroll
    for (int i = 0; i < D; ++i) fetch(i, qh[i], ql[i]);
  }
  __device__ __forceinline__ void take(int s, h8 (&wh)[TM], h8 (&wl)[TM]) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      wh[i] = as_h8(qh[0][i]);
      wl[i] = as_h8(ql[0][i]);
    }
#pragma unroll
    for (int q = 0; q + 1 < D; ++q)
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        qh[q][i] = qh[q + 1][i];
        ql[q][i] = ql[q + 1][i];
      }
    fetch(s + D, qh[D - 1], ql[D - 1]);
  }
};

// every wave's LDS writes (and reads) done, then the workgroup barrier; the A prefetch (global
// loads into registers) stays in flight across it
__device__ __forceinline__ void lds_barrier() {
  asm volatile("" ::: "memory");  // no LDS access moves across (the builtin itself is IntrNoMem)
  wait_vm<0>(31);
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// LDS plane pointers: each plane gets its own base register (opaque to the compiler), so every
// access is base + an immediate offset < 64 KB -- ds_read / ds_write's offset field stops at
// 64 KB, and past it hipcc materialises one address VGPR per access (40+ registers here)
typedef __attribute__((address_space(3))) f4 lds_f4w;
__device__ __forceinline__ lds_f4w* lds_base(f4* p) {
  uint32_t a = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(p));
  asm volatile("" : "+v"(a));
  return reinterpret_cast<lds_f4w*>(static_cast<uintptr_t>(a));
}
struct Planes {
  lds_f4w* act_hi;  // [8][4][kNb] (+ g * kNb + j applied)
  lds_f4w* act_lo;
  lds_f4w* enc_hi;  // [2][4][kNb]: segment B (pos_enc(x), pos_enc(x'), xyz, pos_enc(dir))
  lds_f4w* enc_lo;
};

#ifndef AON_WS_VENC_EARLY
#define AON_WS_VENC_EARLY 0
#endif

#ifndef AON_WS_BPF
#define AON_WS_BPF 2  // B fragments (one sample tile's hi + lo) read from LDS ahead of their MFMAs
#endif

// MFMAs of one layer for NT sample tiles from T0 and TU row tiles: acc[i][t] = sum_k W[k] . B[k]
// (3 products per k-step into one accumulator, k-steps in order).  The (k, t) loop runs flat
// with the B fragments of the next AON_WS_BPF (k, t) steps already read from LDS (the
// sched_barrier keeps those reads above the current step's MFMAs: left alone, hipcc sinks each
// ds_read to its use and waits lgkmcnt(0) in front of every sample tile's MFMAs).
template <typename Net, typename G, int L, int NT, int TU, typename AP>
__device__ __forceinline__ void layer_mfma(AP& ap, const Planes& pl, int T0, f4 (&acc)[TU][NT]) {
  constexpr LayerDesc d = Net::layer(L);
  constexpr int K = d.ka + d.kb;
  constexpr int NS = K * NT;
  constexpr int P = AON_WS_BPF < NS ? AON_WS_BPF : NS;
  constexpr int S0 = step0_of<Net>(L);
  constexpr int kNb = G::kNb;
#pragma unroll
  for (int i = 0; i < TU; ++i)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[i][t] = f4{0.f, 0.f, 0.f, 0.f};
  auto bsrc = [&](int s, f4& xh, f4& xl) {
    const int k = s / NT, t = s % NT;
    const lds_f4w* bh = k < d.ka ? pl.act_hi + k * 4 * kNb : pl.enc_hi + (k - d.ka) * 4 * kNb;
    const lds_f4w* bl = k < d.ka ? pl.act_lo + k * 4 * kNb : pl.enc_lo + (k - d.ka) * 4 * kNb;
    xh = bh[16 * (T0 + t)];
    xl = bl[16 * (T0 + t)];
  };
  f4 qh[P], ql[P];
#pragma unroll
  for (int s = 0; s < P; ++s) bsrc(s, qh[s], ql[s]);
  h8 wh[AP::TM], wl[AP::TM];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int t = s % NT;
    if (t == 0) ap.take(S0 + s / NT, wh, wl);
    const h8 xh = as_h8(qh[0]), xl = as_h8(ql[0]);
#pragma unroll
    for (int p = 0; p + 1 < P; ++p) {
      qh[p] = qh[p + 1];
      ql[p] = ql[p + 1];
    }
    if (s + P < NS) bsrc(s + P, qh[P - 1], ql[P - 1]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < TU; ++i) {
      acc[i][t] = mfma16(wh[i], xh, acc[i][t]);
      acc[i][t] = mfma16(wh[i], xl, acc[i][t]);
      acc[i][t] = mfma16(wl[i], xh, acc[i][t]);
    }
  }
}

// epilogue of the wave's row tiles: bias at activation scale, ReLU, fp16 hi / lo split
// (mlp_f16x3_core.hpp epi_part, V2 + fma_mix), written as the lanes' B fragments of the next
// layer (row tiles 2 pr, 2 pr + 1 = k-step pr); m16: the range guard's packed max of the hi bits
template <typename G, bool RELU, int NT, int TU>
__device__ __forceinline__ void pair_epilogue(const f4 (&acc)[TU][NT], const f4 (&bias)[TU],
                                              const Planes& pl, int rt0, int T0, uint32_t& m16) {
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  constexpr int kNb = G::kNb;
#pragma unroll
  for (int p = 0; p < TU / 2; ++p)
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      u4 hw, lw;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int uu = q >> 1, r0 = (q & 1) * 2;
        float vv[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          float v = fmaf(acc[2 * p + uu][t][r0 + e], 1.0f / kWS, bias[2 * p + uu][r0 + e]);
          // no activation: pinned, else hipcc folds this fma and the fp16 conversion of the hi
          // part into one v_fma_mixlo_f16 -- ONE rounding of the exact fma to fp16 where the
          // split (and k_mlp_fwd_f16x3) rounds to fp32 first: 1-ulp different hi / lo pairs in
          // the bottleneck (tools/diag/ws_diff2.py).  (With ReLU the max stands between them;
          // a pin there would also cost a canonicalising v_max per value.)
          if (!RELU) asm("" : "+v"(v));
          if (RELU) v = fmaxf(v, 0.0f);
          vv[e] = v;
        }
        const h2 hp = {static_cast<_Float16>(vv[0]), static_cast<_Float16>(vv[1])};
        const uint32_t hu = __builtin_bit_cast(uint32_t, hp);
        m16 = pk_max_i16(m16, RELU ? hu : (hu & 0x7FFF7FFFu));
        asm("" : "+v"(m16));
        float d0, d1;
        asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(d0) : "v"(hu), "v"(vv[0]));
        asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(d1) : "v"(hu), "v"(vv[1]));
        const h2 lp = {static_cast<_Float16>(d0), static_cast<_Float16>(d1)};
        hw[q] = hu;
        lw[q] = __builtin_bit_cast(uint32_t, lp);
      }
      const int pr = rt0 / 2 + p;
      pl.act_hi[pr * 4 * kNb + 16 * (T0 + t)] = __builtin_bit_cast(f4, hw);
      pl.act_lo[pr * 4 * kNb + 16 * (T0 + t)] = __builtin_bit_cast(f4, lw);
    }
}

__device__ __forceinline__ f4 ldg_f4(const float* p) { return *reinterpret_cast<const f4*>(p); }

// One hidden layer (256 or 128 rows) of the wave's rows and sample tiles (Geo), output in
// place: MFMAs; barrier (every wave past its reads of the input planes); epilogue; `mid` (work
// that needs the input planes free, e.g. the next segment B into the enc planes); barrier.
struct NoMid {
  __device__ __forceinline__ void operator()() const {}
};
template <typename Net, typename G, int L, bool RELU, typename AP, typename MID = NoMid>
__device__ __forceinline__ void hidden_layer(AP& ap, const Planes& pl, const float* bias_g, int w,
                                             int g, uint32_t& m16, const MID& mid = MID{}) {
  constexpr LayerDesc d = Net::layer(L);
  static_assert(d.u == 16 || d.u == 8, "hidden layer of 256 or 128 rows");
  constexpr int NT = G::nt(d.u), TU = G::tu(d.u);
  const int r0 = G::rt0(d.u, w), T0 = G::t0(d.u, w);
  f4 bias[TU];
#pragma unroll
  for (int i = 0; i < TU; ++i) bias[i] = ldg_f4(bias_g + d.bias0 + 16 * (r0 + i) + 4 * g);
  f4 acc[TU][NT];
  layer_mfma<Net, G, L, NT, TU>(ap, pl, T0, acc);
  lds_barrier();
  pair_epilogue<G, RELU, NT, TU>(acc, bias, pl, r0, T0, m16);
  mid();
  lds_barrier();
}

// a 1-tile head (density / rgb / deformation) on the wave's own sample tile: 4 rows at true scale
template <typename Net, typename G, int L, typename AP>
__device__ __forceinline__ f4 head(AP& ap, const Planes& pl, const float* bias_g, int w, int g) {
  constexpr LayerDesc d = Net::layer(L);
  static_assert(d.u == 1 && d.kb == 0, "head");
  const f4 bias = ldg_f4(bias_g + d.bias0 + 4 * g);
  f4 acc[1][1];
  layer_mfma<Net, G, L, 1, 1>(ap, pl, w, acc);
  f4 res;
#pragma unroll
  for (int r = 0; r < 4; ++r) res[r] = fmaf(acc[0][0][r], 1.0f / (kWS * kActS), bias[r]);
  return res;
}

// 8 fp32 features (true scale) of a segment-B k-step of this lane -> the enc planes (hi / lo at
// activation scale, split8's range test into ovf)
template <typename G>
__device__ __forceinline__ void put_segb(const Planes& pl, int k, int w, const float (&v)[8],
                                         uint64_t& ovf) {
  float ev[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) ev[e] = v[e] * kActS;
  h8 hi, lo;
  split8<false>(ev, hi, lo, ovf);
  pl.enc_hi[k * 4 * G::kNb + 16 * w] = __builtin_bit_cast(f4, hi);
  pl.enc_lo[k * 4 * G::kNb + 16 * w] = __builtin_bit_cast(f4, lo);
}

struct WsSetup {
  Planes pl;
  int lane, w, g, j;
  int64_t row, rr, ray;
};
template <typename G>
__device__ __forceinline__ WsSetup ws_setup(f4* smem, int64_t N, int S) {
  WsSetup c;
  const int tid = threadIdx.x;
  c.lane = tid & 63;
  c.w = __builtin_amdgcn_readfirstlane(tid >> 6);
  c.g = c.lane >> 4;
  c.j = c.lane & 15;
  const int gj = c.g * G::kNb + c.j;
  c.pl.act_hi = lds_base(smem + gj);
  c.pl.act_lo = lds_base(smem + G::kActPlane + gj);
  c.pl.enc_hi = lds_base(smem + 2 * G::kActPlane + gj);
  c.pl.enc_lo = lds_base(smem + 2 * G::kActPlane + G::kEncPlane + gj);
  c.row = (int64_t)blockIdx.x * G::kNb + 16 * c.w + c.j;  // this lane's sample (wave w's tile)
  c.rr = c.row < N ? c.row : N - 1;
  c.ray = c.rr / S;
  return c;
}

// ---- vanilla NeRFMLP (model.py:95-120), MODE 0 inputs: rays_o, rays_d, viewdirs, t
template <int WAVES>
__global__ __launch_bounds__(64 * WAVES, 2) void k_mlp_ws_f16x3(
    const f4* __restrict__ wstream, const float* __restrict__ bias_g, const float* __restrict__ in0,
    const float* __restrict__ in1, const float* __restrict__ in2, const float* __restrict__ in3,
    int64_t B, int S, int act, float* __restrict__ raw) {
  using Net = NetVanillaH;
  using G = Geo<WAVES>;
  __shared__ f4 smem[G::kLdsF4];
  const int64_t N = B * S;
  const WsSetup c = ws_setup<G>(smem, N, S);
  const int w = c.w, g = c.g;
  const Planes& pl = c.pl;
  APipe<Net, G, G::kPrefetch> ap;
  ap.ws = wstream;
  ap.lane = c.lane;
  ap.w = w;
  ap.start();

  // pos_enc(x) of this wave's sample tile, natural feature order (segment B)
  uint64_t ovf = 0;
  {
    const float* ro = in0 + 3 * c.ray;
    const float* rd = in1 + 3 * c.ray;
    const float tt = in3[c.rr];
    const float x0 = __fadd_rn(ro[0], __fmul_rn(tt, rd[0]));
    const float x1 = __fadd_rn(ro[1], __fmul_rn(tt, rd[1]));
    const float x2 = __fadd_rn(ro[2], __fmul_rn(tt, rd[2]));
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      float ev[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) ev[e] = pos_enc_feature(x0, x1, x2, 32 * k + 8 * g + e, 0, 10);
      put_segb<G>(pl, k, w, ev, ovf);
    }
  }
  lds_barrier();

  uint32_t m16 = 0;
  hidden_layer<Net, G, L0, true>(ap, pl, bias_g, w, g, m16);
  hidden_layer<Net, G, L1, true>(ap, pl, bias_g, w, g, m16);
  hidden_layer<Net, G, L2, true>(ap, pl, bias_g, w, g, m16);
  hidden_layer<Net, G, L3, true>(ap, pl, bias_g, w, g, m16);
  hidden_layer<Net, G, L4, true>(ap, pl, bias_g, w, g, m16);
  // skip layer cat[h4, enc]; once it has read the enc planes, pos_enc(viewdirs) of this wave's
  // tile goes to enc k-step 0 for the view layer
  hidden_layer<Net, G, L5, true>(ap, pl, bias_g, w, g, m16, [&] {
    const float* vd = in2 + 3 * c.ray;
    float vv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) vv[e] = pos_enc_feature(vd[0], vd[1], vd[2], 8 * g + e, 0, 4);
    put_segb<G>(pl, 0, w, vv, ovf);
  });
  hidden_layer<Net, G, L6, true>(ap, pl, bias_g, w, g, m16);
  hidden_layer<Net, G, L7, true>(ap, pl, bias_g, w, g, m16);
  // density head on h7 (this wave's tile), then the bottleneck (no activation) on h7
  const f4 dens = head<Net, G, LDEN>(ap, pl, bias_g, w, g);
  hidden_layer<Net, G, LBOT, false>(ap, pl, bias_g, w, g, m16);
  hidden_layer<Net, G, LVIEW, true>(ap, pl, bias_g, w, g, m16);  // cat[bottleneck, enc_dir] + ReLU
  const f4 rgb = head<Net, G, LRGB>(ap, pl, bias_g, w, g);
  if (g == 0 && c.row < N) {
    const f4 o = {act_rgb(rgb[0], act), act_rgb(rgb[1], act), act_rgb(rgb[2], act), act_sigma(dens[0], act)};
    *reinterpret_cast<f4*>(raw + 4 * c.row) = o;
  }
  const bool bad = (m16 & 0x7FFFu) >= 0x7C00u || ((m16 >> 16) & 0x7FFFu) >= 0x7C00u;
  range_report(bias_g + Net::kBiasFloats, ovf | __builtin_amdgcn_ballot_w64(bad));
}

// ---- articulated NeRFMLP (model_autodecoder.py:168-239, latents folded into the biases as in
// mlp_art.hip), MODE 0 inputs.  The deformation head gives each wave its tile's delta in lane
// group 0, broadcast to the sample's lanes (as mlp_art.hip does), x' = delta + xyz in fp32,
// pos_enc(x') into the enc planes.
template <int WAVES>
__global__ __launch_bounds__(64 * WAVES, 2) void k_mlp_art_ws_f16x3(
    const f4* __restrict__ wstream, const float* __restrict__ bias_g, const float* __restrict__ in0,
    const float* __restrict__ in1, const float* __restrict__ in2, const float* __restrict__ in3,
    int64_t B, int S, int act, float* __restrict__ raw) {
  using Net = NetArtH;
  using G = Geo<WAVES>;
  __shared__ f4 smem[G::kLdsF4];
  const int64_t N = B * S;
  const WsSetup c = ws_setup<G>(smem, N, S);
  const int w = c.w, g = c.g;
  const Planes& pl = c.pl;
  APipe<Net, G, G::kPrefetch> ap;
  ap.ws = wstream;
  ap.lane = c.lane;
  ap.w = w;
  ap.start();

  uint64_t ovf = 0;
  float px[3];
  {
    const float* ro = in0 + 3 * c.ray;
    const float* rd = in1 + 3 * c.ray;
    const float tt = in3[c.rr];
#pragma unroll
    for (int q = 0; q < 3; ++q) px[q] = __fadd_rn(ro[q], __fmul_rn(tt, rd[q]));
    // deformation input: xyz in lane group 0, elements 0..2 (natural order), the rest 0
    float dv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) dv[e] = (g == 0 && e < 3) ? px[e < 3 ? e : 0] : 0.f;
    put_segb<G>(pl, 0, w, dv, ovf);
  }
  lds_barrier();

  uint32_t m16 = 0;
  hidden_layer<Net, G, A_D0, true>(ap, pl, bias_g, w, g, m16);
  hidden_layer<Net, G, A_D1, true>(ap, pl, bias_g, w, g, m16);
  hidden_layer<Net, G, A_D2, true>(ap, pl, bias_g, w, g, m16);
  hidden_layer<Net, G, A_D3, true>(ap, pl, bias_g, w, g, m16);
  {
    const f4 dlt = head<Net, G, A_DOUT>(ap, pl, bias_g, w, g);
    // x' = deformation + xyz (:205), pos_enc(x') (:207-212) of this wave's tile -> enc planes
    // (the xyz segment there was last read by deformations_linear.0, long past its barriers)
    float q3[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) q3[q] = __fadd_rn(__shfl(dlt[q], c.j, 64), px[q]);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      float ev[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) ev[e] = pos_enc_feature(q3[0], q3[1], q3[2], 32 * k + 8 * g + e, 0, 10);
      put_segb<G>(pl, k, w, ev, ovf);
    }
    lds_barrier();
  }
  hidden_layer<Net, G, A_P0, true>(ap, pl, bias_g, w, g, m16);
  hidden_layer<Net, G, A_P1, true>(ap, pl, bias_g, w, g, m16);
  hidden_layer<Net, G, A_P2, true>(ap, pl, bias_g, w, g, m16);
  hidden_layer<Net, G, A_P3, true>(ap, pl, bias_g, w, g, m16);
  hidden_layer<Net, G, A_P4, true>(ap, pl, bias_g, w, g, m16);
  hidden_layer<Net, G, A_P5, true>(ap, pl, bias_g, w, g, m16, [&] {
    const float* vd = in2 + 3 * c.ray;
    float vv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) vv[e] = pos_enc_feature(vd[0], vd[1], vd[2], 8 * g + e, 0, 4);
    put_segb<G>(pl, 0, w, vv, ovf);
  });
  hidden_layer<Net, G, A_P6, true>(ap, pl, bias_g, w, g, m16);
  hidden_layer<Net, G, A_P7, true>(ap, pl, bias_g, w, g, m16);
  const f4 dens = head<Net, G, A_DEN>(ap, pl, bias_g, w, g);
  hidden_layer<Net, G, A_BOT, false>(ap, pl, bias_g, w, g, m16);
  hidden_layer<Net, G, A_V0, true>(ap, pl, bias_g, w, g, m16);  // cat[bottleneck, enc_dir, app]
  hidden_layer<Net, G, A_V1, true>(ap, pl, bias_g, w, g, m16);
  hidden_layer<Net, G, A_V2, true>(ap, pl, bias_g, w, g, m16);
  hidden_layer<Net, G, A_V3, true>(ap, pl, bias_g, w, g, m16);
  const f4 rgb = head<Net, G, A_RGB>(ap, pl, bias_g, w, g);
  if (g == 0 && c.row < N) {
    const f4 o = {act_rgb(rgb[0], act), act_rgb(rgb[1], act), act_rgb(rgb[2], act), act_sigma(dens[0], act)};
    *reinterpret_cast<f4*>(raw + 4 * c.row) = o;
  }
  const bool bad = (m16 & 0x7FFFu) >= 0x7C00u || ((m16 >> 16) & 0x7FFFu) >= 0x7C00u;
  range_report(bias_g + Net::kBiasFloats, ovf | __builtin_amdgcn_ballot_w64(bad));
}


// compile-time loop: f(std::integral_constant<int, I>) for I in [0, N) -- the step indices that
// select blocks and layers must be constants, or hipcc evaluates layer_of_step's loop at run
// time in VGPRs (hundreds of spilled registers in the pipelined kernel)
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// ---- pipelined schedule (AON_WS_PIPE): every hidden layer in two halves of the workgroup's
// sample tiles (half h = tiles h kTiles / 2 ..), one barrier per half.  The epilogue of the half
// just finished runs in small units between the MFMAs of the next half (MFMAs issue
// asynchronously: the wave's VALU and LDS writes fill the matrix pipe's 16-cycle slots), instead
// of after a barrier with every wave of the SIMD idle in it together.  Safe in place: the units
// of half h of layer l write tiles of half h, which every wave finished reading before the
// barrier that ends half h; the next half's MFMAs read the other half's tiles (or, across a
// layer boundary, half 0 of layer l's output, completed by the previous phase's units).  The
// weight fragments of a layer stream twice (once per half): 2x the L2 -> CU bytes.
template <typename Net>
__host__ __device__ constexpr bool hidden_of(int l) { return Net::layer(l).u > 1; }
template <typename Net>
__host__ __device__ constexpr int pstep0_of(int l) {
  return l == 0 ? 0 : pstep0_of<Net>(l - 1) + (hidden_of<Net>(l - 1) ? 2 * layer_k<Net>(l - 1) : 0);
}
template <typename Net>
__host__ __device__ constexpr int player_of_step(int s) {
  int l = 0;
  while (l + 1 < Net::kNumLayers && pstep0_of<Net>(l + 1) <= s) ++l;
  return l;
}
template <typename Net>
constexpr int kPStepsOf = pstep0_of<Net>(Net::kNumLayers);

// APipe over the pipelined sequence (hidden layers twice, no heads)
template <typename Net, typename G, int D>
struct APipeP {
  static constexpr int TM = G::tu(16);
  const f4* __restrict__ ws;
  int lane, w;
  f4 qh[D][TM], ql[D][TM];
  template <int S>
  __device__ __forceinline__ void fetch(f4 (&h)[TM], f4 (&l)[TM]) {
    if constexpr (S < kPStepsOf<Net>) {
      constexpr int L = player_of_step<Net>(S);
      constexpr LayerDesc d = Net::layer(L);
      constexpr int K = d.ka + d.kb;
      constexpr int k = (S - pstep0_of<Net>(L)) % K;
      constexpr int TU = G::tu(d.u);
      const int r0 = G::rt0(d.u, w);
#pragma unroll
      for (int i = 0; i < TU; ++i) {
        const int u = r0 + i;
        const int b = d.blk0 + 2 * (((u >> 1) * K + k) * 2 + (u & 1));
        h[i] = ws[(size_t)b * 64 + lane];
        l[i] = ws[(size_t)(b + 1) * 64 + lane];
      }
    }
  }
  __device__ __forceinline__ void start() {
    static_for<D>([&](auto I) { fetch<decltype(I)::value>(qh[decltype(I)::value], ql[decltype(I)::value]); });
  }
  template <int S>
  __device__ __forceinline__ void take(h8 (&wh)[TM], h8 (&wl)[TM]) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      wh[i] = as_h8(qh[0][i]);
      wl[i] = as_h8(ql[0][i]);
    }
#pragma unroll
    for (int q = 0; q + 1 < D; ++q)
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        qh[q][i] = qh[q + 1][i];
        ql[q][i] = ql[q + 1][i];
      }
    fetch<S + D>(qh[D - 1], ql[D - 1]);
  }
};

// the wave's part of half H of layer L: TU row tiles from rt0 over NTh sample tiles from T0
template <typename Net, typename G, int L>
struct LG {
  static constexpr LayerDesc d = Net::layer(L);
  static constexpr int K = d.ka + d.kb;
  static constexpr int TU = G::tu(d.u), NTh = G::nt(d.u) / 2;
  __device__ __forceinline__ static int rt0(int w) { return G::rt0(d.u, w); }
  __device__ __forceinline__ static int T0(int w, int H) { return H * (G::kTiles / 2) + G::t0(d.u, w) / 2; }
};

// a finished half waiting for its epilogue: accumulators, biases, where the output goes
template <typename Net, typename G, int L, bool RELU>
struct Job {
  using LGt = LG<Net, G, L>;
  static constexpr int TU = LGt::TU, NTh = LGt::NTh;
  static constexpr int kUnits = TU / 2 * NTh;  // (pair, sample tile) units
  f4 acc[TU][NTh];
  f4 bias[TU];
  int rt0, T0;
  __device__ __forceinline__ void load_bias(const float* bias_g, int g) {
#pragma unroll
    for (int i = 0; i < TU; ++i) bias[i] = ldg_f4(bias_g + LGt::d.bias0 + 16 * (rt0 + i) + 4 * g);
  }
  // epilogue unit I: pair I / NTh of the wave's rows, sample tile I % NTh (pair_epilogue's body)
  template <int I>
  __device__ __forceinline__ void unit(const Planes& pl, uint32_t& m16) const {
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    constexpr int p = I / NTh, t = I % NTh;
    u4 hw, lw;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int uu = q >> 1, r0 = (q & 1) * 2;
      float vv[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        float v = fmaf(acc[2 * p + uu][t][r0 + e], 1.0f / kWS, bias[2 * p + uu][r0 + e]);
        if (!RELU) asm("" : "+v"(v));  // (pair_epilogue: no fma + fp16-convert fold)
        if (RELU) v = fmaxf(v, 0.0f);
        vv[e] = v;
      }
      const h2 hp = {static_cast<_Float16>(vv[0]), static_cast<_Float16>(vv[1])};
      const uint32_t hu = __builtin_bit_cast(uint32_t, hp);
      m16 = pk_max_i16(m16, RELU ? hu : (hu & 0x7FFF7FFFu));
      asm("" : "+v"(m16));
      float d0, d1;
      asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(d0) : "v"(hu), "v"(vv[0]));
      asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(d1) : "v"(hu), "v"(vv[1]));
      const h2 lp = {static_cast<_Float16>(d0), static_cast<_Float16>(d1)};
      hw[q] = hu;
      lw[q] = __builtin_bit_cast(uint32_t, lp);
    }
    const int pr = rt0 / 2 + p;
    pl.act_hi[pr * 4 * G::kNb + 16 * (T0 + t)] = __builtin_bit_cast(f4, hw);
    pl.act_lo[pr * 4 * G::kNb + 16 * (T0 + t)] = __builtin_bit_cast(f4, lw);
  }
  __device__ __forceinline__ void all(const Planes& pl, uint32_t& m16) const {
    static_for<kUnits>([&](auto I) { unit<decltype(I)::value>(pl, m16); });
  }
};
struct NoJob {
  static constexpr int kUnits = 0;
  template <int I>
  __device__ __forceinline__ void unit(const Planes&, uint32_t&) const {}
};

// MFMAs of half H of layer L (as layer_mfma, over the pipelined step sequence) with the
// pending job's epilogue units after the MFMAs of every other (k, t) step; then the job's
// remaining units
template <typename Net, typename G, int L, int H, typename AP, typename J>
__device__ __forceinline__ void half_mfma(AP& ap, const Planes& pl, int w,
                                          f4 (&acc)[LG<Net, G, L>::TU][LG<Net, G, L>::NTh],
                                          const J& job, uint32_t& m16) {
  using LGt = LG<Net, G, L>;
  constexpr LayerDesc d = LGt::d;
  constexpr int K = LGt::K, NT = LGt::NTh, TU = LGt::TU;
  constexpr int NS = K * NT;
  constexpr int P = AON_WS_BPF < NS ? AON_WS_BPF : NS;
  constexpr int S0 = pstep0_of<Net>(L) + H * K;
  constexpr int kNb = G::kNb;
  const int T0 = LGt::T0(w, H);
#pragma unroll
  for (int i = 0; i < TU; ++i)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[i][t] = f4{0.f, 0.f, 0.f, 0.f};
  auto bsrc = [&](int s, f4& xh, f4& xl) {
    const int k = s / NT, t = s % NT;
    const lds_f4w* bh = k < d.ka ? pl.act_hi + k * 4 * kNb : pl.enc_hi + (k - d.ka) * 4 * kNb;
    const lds_f4w* bl = k < d.ka ? pl.act_lo + k * 4 * kNb : pl.enc_lo + (k - d.ka) * 4 * kNb;
    xh = bh[16 * (T0 + t)];
    xl = bl[16 * (T0 + t)];
  };
  f4 qh[P], ql[P];
#pragma unroll
  for (int s = 0; s < P; ++s) bsrc(s, qh[s], ql[s]);
  h8 wh[AP::TM], wl[AP::TM];
  constexpr int kEvery = J::kUnits > 0 && NS / J::kUnits >= 2 ? NS / J::kUnits : 1;
  static_for<NS>([&](auto I) {
    constexpr int s = decltype(I)::value;
    constexpr int t = s % NT;
    if constexpr (t == 0) ap.template take<S0 + s / NT>(wh, wl);
    const h8 xh = as_h8(qh[0]), xl = as_h8(ql[0]);
#pragma unroll
    for (int p = 0; p + 1 < P; ++p) {
      qh[p] = qh[p + 1];
      ql[p] = ql[p + 1];
    }
    if constexpr (s + P < NS) bsrc(s + P, qh[P - 1], ql[P - 1]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < TU; ++i) {
      acc[i][t] = mfma16(wh[i], xh, acc[i][t]);
      acc[i][t] = mfma16(wh[i], xl, acc[i][t]);
      acc[i][t] = mfma16(wl[i], xh, acc[i][t]);
    }
#ifndef AON_WS_DBG_NOUNITS
    if constexpr (s % kEvery == kEvery - 1 && s / kEvery < J::kUnits)
      job.template unit<s / kEvery>(pl, m16);
#endif
  });
  static_for<(J::kUnits > NS / kEvery ? J::kUnits - NS / kEvery : 0)>([&](auto I) {
    job.template unit<NS / kEvery + decltype(I)::value>(pl, m16);
  });
}

// a finished half -> its job (biases loaded now: read by the units during the next half)
template <typename Net, typename G, int L, bool RELU, int H>
__device__ __forceinline__ Job<Net, G, L, RELU> make_job(
    const f4 (&acc)[LG<Net, G, L>::TU][LG<Net, G, L>::NTh], const float* bias_g, int w, int g) {
  Job<Net, G, L, RELU> j;
#pragma unroll
  for (int i = 0; i < LG<Net, G, L>::TU; ++i)
#pragma unroll
    for (int t = 0; t < LG<Net, G, L>::NTh; ++t) j.acc[i][t] = acc[i][t];
  j.rt0 = LG<Net, G, L>::rt0(w);
  j.T0 = LG<Net, G, L>::T0(w, H);
  j.load_bias(bias_g, g);
  return j;
}

// a 1-tile head on the wave's own sample tile, its weight fragments loaded straight from global
// (two k-steps at a time; not in the prefetch sequence)
template <typename Net, typename G, int L>
__device__ __forceinline__ f4 head_direct(const Planes& pl, const f4* __restrict__ wstream,
                                          const float* bias_g, int w, int g, int lane) {
#ifdef AON_WS_DBG_NOHEADS
  return f4{0.f, 0.f, 0.f, 0.f};
#endif
  constexpr LayerDesc d = Net::layer(L);
  static_assert(d.u == 1 && d.kb == 0, "head");
  const f4 bias = ldg_f4(bias_g + d.bias0 + 4 * g);
  f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k0 = 0; k0 < d.ka; k0 += 2) {
    f4 ah[2], al[2], bh[2], bl[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int b = d.blk0 + 2 * (k0 + k);
      ah[k] = wstream[(size_t)b * 64 + lane];
      al[k] = wstream[(size_t)(b + 1) * 64 + lane];
      bh[k] = pl.act_hi[(k0 + k) * 4 * G::kNb + 16 * w];
      bl[k] = pl.act_lo[(k0 + k) * 4 * G::kNb + 16 * w];
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      acc = mfma16(as_h8(ah[k]), as_h8(bh[k]), acc);
      acc = mfma16(as_h8(ah[k]), as_h8(bl[k]), acc);
      acc = mfma16(as_h8(al[k]), as_h8(bh[k]), acc);
    }
  }
  f4 res;
#pragma unroll
  for (int r = 0; r < 4; ++r) res[r] = fmaf(acc[r], 1.0f / (kWS * kActS), bias[r]);
  return res;
}

// one hidden layer, pipelined: half 0 (finishing `prev`), half 1 (finishing half 0); returns
// the job of half 1, to be finished by the next layer's half 0
#define AON_WS_HALVES(L_, RELU_, PREV, OUT)                                                  \
  f4 OUT##_a0[LG<Net, G, L_>::TU][LG<Net, G, L_>::NTh];                                     \
  half_mfma<Net, G, L_, 0>(ap, pl, w, OUT##_a0, PREV, m16);                                  \
  lds_barrier();                                                                             \
  const auto OUT##_j0 = make_job<Net, G, L_, RELU_, 0>(OUT##_a0, bias_g, w, g);              \
  f4 OUT##_a1[LG<Net, G, L_>::TU][LG<Net, G, L_>::NTh];                                     \
  half_mfma<Net, G, L_, 1>(ap, pl, w, OUT##_a1, OUT##_j0, m16);                              \
  lds_barrier();                                                                             \
  const auto OUT = make_job<Net, G, L_, RELU_, 1>(OUT##_a1, bias_g, w, g);

template <int WAVES>
__global__ __launch_bounds__(64 * WAVES, 2) void k_mlp_ws_pipe_f16x3(
    const f4* __restrict__ wstream, const float* __restrict__ bias_g, const float* __restrict__ in0,
    const float* __restrict__ in1, const float* __restrict__ in2, const float* __restrict__ in3,
    int64_t B, int S, int act, float* __restrict__ raw) {
  using Net = NetVanillaH;
  using G = Geo<WAVES>;
  __shared__ f4 smem[G::kLdsF4];
  const int64_t N = B * S;
  const WsSetup c = ws_setup<G>(smem, N, S);
  const int w = c.w, g = c.g;
  const Planes& pl = c.pl;
  APipeP<Net, G, G::kPrefetch> ap;
  ap.ws = wstream;
  ap.lane = c.lane;
  ap.w = w;
  ap.start();
  const bool first_half = w < G::kTiles / 2;  // the wave's own sample tile (heads) is in half 0

  uint64_t ovf = 0;
  {
    const float* ro = in0 + 3 * c.ray;
    const float* rd = in1 + 3 * c.ray;
    const float tt = in3[c.rr];
    const float x0 = __fadd_rn(ro[0], __fmul_rn(tt, rd[0]));
    const float x1 = __fadd_rn(ro[1], __fmul_rn(tt, rd[1]));
    const float x2 = __fadd_rn(ro[2], __fmul_rn(tt, rd[2]));
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      float ev[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) ev[e] = pos_enc_feature(x0, x1, x2, 32 * k + 8 * g + e, 0, 10);
      put_segb<G>(pl, k, w, ev, ovf);
    }
  }
  lds_barrier();

  uint32_t m16 = 0;
  const NoJob none;
  AON_WS_HALVES(L0, true, none, j0)
  AON_WS_HALVES(L1, true, j0, j1)
  AON_WS_HALVES(L2, true, j1, j2)
  AON_WS_HALVES(L3, true, j2, j3)
  AON_WS_HALVES(L4, true, j3, j4)
  AON_WS_HALVES(L5, true, j4, j5)  // the skip layer reads the enc planes (both halves)
  // L6 half 0: every wave is past L5's reads of the enc planes -> pos_enc(viewdirs) of the
  // wave's tile into enc k-step 0 for the view layer
  {
    const float* vd = in2 + 3 * c.ray;
    float vv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) vv[e] = pos_enc_feature(vd[0], vd[1], vd[2], 8 * g + e, 0, 4);
    put_segb<G>(pl, 0, w, vv, ovf);
  }
  AON_WS_HALVES(L6, true, j5, j6)
  AON_WS_HALVES(L7, true, j6, j7)
  // the bottleneck's halves; the density head reads h7 of the wave's tile while it is complete
  // and not yet overwritten: tiles of half 0 during the bottleneck's half 0 (j7 writes half 1),
  // tiles of half 1 during its half 1 (its half-0 job writes half 0)
  f4 dens = {0.f, 0.f, 0.f, 0.f};
  if (first_half) dens = head_direct<Net, G, LDEN>(pl, wstream, bias_g, w, g, c.lane);
  f4 jb_a0[LG<Net, G, LBOT>::TU][LG<Net, G, LBOT>::NTh];
  half_mfma<Net, G, LBOT, 0>(ap, pl, w, jb_a0, j7, m16);
  lds_barrier();
  const auto jb_j0 = make_job<Net, G, LBOT, false, 0>(jb_a0, bias_g, w, g);
  if (!first_half) dens = head_direct<Net, G, LDEN>(pl, wstream, bias_g, w, g, c.lane);
  f4 jb_a1[LG<Net, G, LBOT>::TU][LG<Net, G, LBOT>::NTh];
  half_mfma<Net, G, LBOT, 1>(ap, pl, w, jb_a1, jb_j0, m16);
  lds_barrier();
  const auto jb = make_job<Net, G, LBOT, false, 1>(jb_a1, bias_g, w, g);
  AON_WS_HALVES(LVIEW, true, jb, jv)  // cat[bottleneck, enc_dir] + ReLU
  // the view layer's half-1 epilogue; the rgb head of half-0 tiles meanwhile (hv complete there)
  f4 rgb;
  if (first_half) rgb = head_direct<Net, G, LRGB>(pl, wstream, bias_g, w, g, c.lane);
  jv.all(pl, m16);
  lds_barrier();
  if (!first_half) rgb = head_direct<Net, G, LRGB>(pl, wstream, bias_g, w, g, c.lane);
  if (g == 0 && c.row < N) {
    const f4 o = {act_rgb(rgb[0], act), act_rgb(rgb[1], act), act_rgb(rgb[2], act), act_sigma(dens[0], act)};
    *reinterpret_cast<f4*>(raw + 4 * c.row) = o;
  }
  const bool bad = (m16 & 0x7FFFu) >= 0x7C00u || ((m16 >> 16) & 0x7FFFu) >= 0x7C00u;
  range_report(bias_g + Net::kBiasFloats, ovf | __builtin_amdgcn_ballot_w64(bad));
}
#undef AON_WS_HALVES

}  // namespace ws

// the pipelined schedule: compile with -DAON_WS_PIPE=1 (A/B), else off (measured 7% slower
// than the plain schedule: its halves stream the weights twice)
#ifndef AON_WS_PIPE
#define AON_WS_PIPE 0
#endif
static constexpr bool ws_pipe() { return AON_WS_PIPE == 1; }

// geometry of the weight-streamed kernels: -DAON_WS_WAVES=4 (A/B), else 8 (4 waves x 64 samples
// measured 2.5x slower: twice the A-fragment bytes per MFMA; the pipelined schedule is built for
// 8 waves only: at 4 its two accumulator sets and the 4-tile A fragments spill)
#ifndef AON_WS_WAVES
#define AON_WS_WAVES 8
#endif
static constexpr int ws_waves() { return AON_WS_WAVES == 4 ? 4 : 8; }

int launch_ws_f16x3(const void* packed, const float* a0, const float* a1, const float* a2,
                    const float* a3, int64_t B, int S, int act, float* raw, hipStream_t stream) {
  const int64_t N = B * S;
  const f4* wsp = static_cast<const f4*>(packed);
  const float* bias = reinterpret_cast<const float*>(static_cast<const char*>(packed) + kStreamBytesF32);
  if (ws_pipe() && ws_waves() == 8)
    hipLaunchKernelGGL(ws::k_mlp_ws_pipe_f16x3<8>, static_cast<int>((N + 127) / 128), 512, 0,
                       stream, wsp, bias, a0, a1, a2, a3, B, S, act, raw);
  else if (ws_waves() == 8)
    hipLaunchKernelGGL(ws::k_mlp_ws_f16x3<8>, static_cast<int>((N + 127) / 128), 512, 0, stream,
                       wsp, bias, a0, a1, a2, a3, B, S, act, raw);
  else
    hipLaunchKernelGGL(ws::k_mlp_ws_f16x3<4>, static_cast<int>((N + 63) / 64), 256, 0, stream,
                       wsp, bias, a0, a1, a2, a3, B, S, act, raw);
  return launch_status("aon_mlp_fwd");
}

int launch_art_ws_f16x3(const void* packed, const float* a0, const float* a1, const float* a2,
                        const float* a3, int64_t B, int S, int act, float* raw, hipStream_t stream) {
  const int64_t N = B * S;
  const f4* wsp = static_cast<const f4*>(packed);
  const float* bias = reinterpret_cast<const float*>(static_cast<const char*>(packed) + NetArtH::kStreamBytes);
  if (ws_waves() == 8)
    hipLaunchKernelGGL(ws::k_mlp_art_ws_f16x3<8>, static_cast<int>((N + 127) / 128), 512, 0, stream,
                       wsp, bias, a0, a1, a2, a3, B, S, act, raw);
  else
    hipLaunchKernelGGL(ws::k_mlp_art_ws_f16x3<4>, static_cast<int>((N + 63) / 64), 256, 0, stream,
                       wsp, bias, a0, a1, a2, a3, B, S, act, raw);
  return launch_status("aon_mlp_art_fwd");
}

}  // namespace mlp
}  // namespace aon
