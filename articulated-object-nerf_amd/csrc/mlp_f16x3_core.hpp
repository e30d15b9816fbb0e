// Building blocks of the fused fp16x3 MLP kernels (mlp_f16x3.hip: NeRFMLP of model.py;
// mlp_art.hip: the articulated NeRFMLP of model_autodecoder.py): operand split, fragment
// prefetch over the LDS weight ring, and the layer / head MFMA loops over a NetH layer table.
// Numerics and tiling are described at the top of mlp_f16x3.hip.
#pragma once

#include <type_traits>

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

// ---- bf16 numerics (the C5 training step's bf16 mode): one v_mfma_f32_16x16x32_bf16 per
// k-step and tile instead of three fp16 products; operands are plain bf16 (fp32's exponent
// range: no scaling limits, no range guard), carried in the same h8 registers as raw bits.
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f4 mfma_bf(h8 a, h8 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf8, a),
                                                 __builtin_bit_cast(bf8, b), c, 0, 0, 0);
}
__device__ __forceinline__ _Float16 bf_bits(float v) {
  return __builtin_bit_cast(_Float16, static_cast<__bf16>(v));  // round to nearest even
}

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

// Range guard.  fp16 holds |x| <= 65504: at the 2^3 activation scale a hidden activation past
// |x| = 8188 (gradients: past 65504 / their per-call scale) would become inf in the hi part --
// and the NaN it makes in the next layer is squashed to 0 by fmax's ReLU: silent garbage.
// Every value split into a hi/lo pair is range-tested (Frag::ovf: the wave's ballot of the
// test, OR-ed in SGPRs -- one v_cmp + one s_or per value pair, no VGPR held; a running fmax or
// a per-lane bool was a VGPR chain through every epilogue that made hipcc spill hundreds of
// registers), and a wave that saw one past the limit sets
// the status word behind its bias table (zeroed by the pack, read by aon_mlp_read_status): the
// caller learns the result is invalid.
constexpr float kF16Max = 65504.0f;
// ovf |= ballot(bad): the running OR is pinned to one SGPR pair per step (an empty asm on it);
// left to itself hipcc keeps every ballot live until the final OR, and the hundreds of mask
// pairs spill into VGPR lanes (1,072 v_writelane / v_readlane in the vanilla kernel, -5%)
#ifndef AON_PIN_OVF
#define AON_PIN_OVF(v) asm("" : "+s"(v))
#endif
#ifndef AON_RANGE_GUARD
#define AON_RANGE_GUARD 1  // 0: timing-only A/B build without the range test
#endif
__device__ __forceinline__ void or_ballot(uint64_t& ovf, bool bad) {
#if AON_RANGE_GUARD
  ovf |= __builtin_amdgcn_ballot_w64(bad);
  AON_PIN_OVF(ovf);
#else
  (void)ovf;
  (void)bad;
#endif
}
__device__ __forceinline__ void range_report(const float* bias_end, uint64_t ovf) {
  if (ovf && (threadIdx.x & 63) == 0) *reinterpret_cast<uint32_t*>(const_cast<float*>(bias_end)) = 1u;
}

// operand scale of a layer's input activations: 2^3 for fp16x3 (V2), 1 for bf16 layers (bf16
// has fp32's exponent range: no scaling, and their weights are packed unscaled too)
template <bool BF>
__host__ __device__ constexpr float act_scale() { return BF ? 1.0f : (AON_F16X3_V2 ? kActS : kActScale); }

// 8 fp32 values (already at activation scale) -> (hi, lo) fp16 fragments; ovf |= out of range.
// BF: bf16 values in hi, no lo, no range test.
template <bool BF = false>
__device__ __forceinline__ void split8(const float (&v)[8], h8& hi, h8& lo, uint64_t& ovf) {
  if (BF) {
#pragma unroll
    for (int j = 0; j < 8; ++j) hi[j] = bf_bits(v[j]);
    return;
  }
  float m = 0.0f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const _Float16 h = static_cast<_Float16>(v[j]);
    hi[j] = h;
    lo[j] = lo_of(v[j], h);
    m = fmaxf(m, fabsf(v[j]));
  }
  or_ballot(ovf, m > kF16Max);
}

// One-step-ahead fragment prefetch over the weight stream: blocks are consumed strictly in
// stream order (2 per (u, k-step)), so the step after block b is always b + 2.  The hi/lo pair
// of the NEXT step is read from LDS before the MFMAs of the current step are issued, hiding the
// LDS latency behind 3*NCOL MFMAs (hipcc issues ds_read -> lgkmcnt(0) -> MFMA otherwise).
#ifndef AON_SCHED_MASK
#define AON_SCHED_MASK 0
#endif

#ifndef AON_PREFETCH
#define AON_PREFETCH 3
#endif

// EOFF: the k-step at which a layer starts the pending pair's epilogue (layer_h).  Waves
// w and w + 4 of an 8-wave workgroup share a SIMD; run in lockstep they reach the epilogue VALU
// and the epilogue-free MFMA steps together, so neither wave's VALU rides beside the other's
// MFMAs.  Waves 4-7 take EOFF = 4 (a stagger: MI355X_MICROARCH.md "Two waves per SIMD" item 9).
// BF: bf16 numerics -- the compact stream (WeightPipeP) of hi blocks only.  MXL < MXH: the
// mixed stream (StreamMap mode 2): layers in the fp16x3 blocks [MXL, MXH) run fp16x3, the
// others bf16 (layer_h / head_h ask f16_block(d.blk0)).
// W1: the compact blocks of a mixed stream hold fp16 weights at the 2^6 weight scale (k_pack_h
// f16w), not bf16 -- their layers run two fp16 MFMAs per product (hi(W) x hi(x) + hi(W) x lo(x):
// the activations keep their exact hi / lo split, the weights round once to fp16) with the
// fp16x3 epilogue.
// X1F >= 0: the layers from fp16x3 block X1F on run two fp16 MFMAs per product the other way
// round, (hi(W) + lo(W)) x hi(x) -- the weights keep their exact split, the activations round
// once to fp16 (per sample, 2^-11 relative; their lo parts are never formed).
template <typename P, int D = AON_PREFETCH, int EOFF = 0, bool BF = false, int MXL = 0, int MXH = 0,
          bool W1 = false, int X1F = -1>
struct FragPipe {
  static constexpr int kEpiOff = EOFF;
  static constexpr bool kW1 = W1;
  static constexpr int kX1From = X1F;
  static constexpr int kMode = MXH > MXL ? 2 : (BF ? 1 : 0);
  __host__ __device__ static constexpr bool f16_block(int b) { return StreamMap{kMode, MXL, MXH}.f16(b); }
  __host__ __device__ static constexpr int map_block(int b) { return StreamMap{kMode, MXL, MXH}.map(b); }
  P& p;
  f4 nh[D], nl[D];  // fragments of the next D steps
  __device__ __forceinline__ explicit FragPipe(P& pp) : p(pp) {}
  __device__ __forceinline__ void fetch_into(int blk_in, f4& h, f4& l) {
    const int blk = map_block(blk_in);
    if (blk >= P::kUsedBlocks) return;
#ifdef AON_ABLATE_LDS  // timing-only build: reuse the first fragments (no LDS reads, wrong results)
    if (blk >= 2 * D) {
      if (blk % P::kChunk == 0) p.begin(blk / P::kChunk);
      return;
    }
#endif
    if (blk % P::kChunk == 0) p.begin(blk / P::kChunk);
    h = p.block(blk);
    if (f16_block(blk_in)) l = p.block(blk + 1);
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

#ifndef AON_GUARD_PK
#define AON_GUARD_PK 1  // 0: A/B build with the round-2 per-pair fp32 range test in the epilogue
#endif
template <int N, int NCOL>
struct Frag {
  h8 hi[N][NCOL], lo[N][NCOL];
  uint64_t ovf = 0;  // lanes that split a value out of fp16 range into this set (range guard)
  // AON_GUARD_PK: the layer epilogues' test, deferred -- per lane, the packed i16 max of the
  // |fp16 hi| bit patterns they produced (a value past the fp16 range rounds to inf, 0x7C00,
  // and a NaN is above it), reduced to a ballot once, by ovf_of, at the kernel's range report
  uint32_t m16 = 0;
};
template <int N, int NCOL>
__device__ __forceinline__ uint64_t ovf_of(const Frag<N, NCOL>& f) {
  const bool bad = (f.m16 & 0x7FFFu) >= 0x7C00u || ((f.m16 >> 16) & 0x7FFFu) >= 0x7C00u;
  return f.ovf | __builtin_amdgcn_ballot_w64(bad);
}

// Epilogue policies of layer_h.  begin_pair(pr) runs at the start of output pair pr (before its
// MFMAs), post() maps a finished value (after the optional ReLU), put() sees the pair's values 2
// at a time.  NoStore compiles away.  RowStore copies a layer's activations to HBM (the
// training forward keeps them for the backward): one 8-B store to y[row][16 u + 4 g + r] at
// true scale (v * s) per part; rows past the batch are not stored.  RowStoreBits also records
// the ReLU' bits; MaskBits is the backward chains' epilogue: the value is kept where the forward
// output it flows into was > 0 (torch's threshold_backward on the ReLU output) and the product
// (true scale) is stored for the weight-gradient GEMMs.
struct NoStore {
  static constexpr bool kPkEpi = true;
  static constexpr bool kPkFromF32 = false;
  __device__ __forceinline__ void begin_pair(int) const {}
  __device__ __forceinline__ float post(int, int, int, int, float v) const { return v; }
  __device__ __forceinline__ uint32_t post_pk(int, int, int, int, uint32_t pk) const { return pk; }
  __device__ __forceinline__ void put(int, int, int, int, float, float) const {}
  __device__ __forceinline__ void put_pk(int, int, int, int, uint32_t) const {}
};
// The bf16 layers' epilogue works on the PACKED pair (kPkEpi policies): the accumulator already
// holds the bias (layer_h seeds it), one v_cvt_pk_bf16_f32 makes the dword the next layer's
// fragment gets, ReLU is one v_pk_max_i16 on it (a negative bf16 is a negative i16; bf16
// rounding is sign-symmetric, so max_i16(bf16(v), 0) = bf16(max(v, 0))), post_pk masks it (the
// backward chains' ReLU'), put_pk stores it as it is and derives the ReLU' bits from it.
// Policies with kPkEpi = false (the articulated chain's enc-column stashes) see fp32 values.
typedef short s2v __attribute__((ext_vector_type(2)));
typedef unsigned short u2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_max_i16(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(s2v, a),
                                                                __builtin_bit_cast(s2v, b)));
}
// The packed bit forms are written as instructions (they only read VALU results): left to
// itself hipcc rewrites min(h, 1) into per-half compares + cndmask + v_perm (3x the VALU).
// per 16-bit half: 1 if the (non-negative) bf16 is non-zero, else 0 -- ReLU' of a ReLU output
// (op_sel_hi:[1,0]: the constant's low half feeds the high lane too; its high half is 0)
__device__ __forceinline__ uint32_t pk_nonzero(uint32_t a) {
  uint32_t r;
  asm("v_pk_min_u16 %0, %1, 1 op_sel_hi:[1,0]" : "=v"(r) : "v"(a));
  return r;
}
// (m << s) | a in one v_lshl_or_b32
__device__ __forceinline__ uint32_t lshl_or(uint32_t m, int s, uint32_t a) {
  uint32_t r;
  asm("v_lshl_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "i"(s), "v"(a));
  return r;
}
// bf16 pair at activation scale 2^3 (a ReLU output, >= 0) -> at true scale: one packed max clears
// a -0 (negative as i16), one saturating packed subtract of 3 from each exponent field divides
// by kActS -- exact for every bf16 whose exponent field is >= 4 (true scale >= 2^-126, fp32's
// normal range).  Below that it is NOT v * 2^-3: a field of exactly 3 leaves exponent 0 with the
// mantissa bits, the denormal m 2^-133 instead of (1 + m / 128) 2^-127 / 8, and a field below 3
// saturates to 0 (fp32-denormal magnitudes only: no numerical effect at these activations)
__device__ __forceinline__ uint32_t pk_bf16_unscale(uint32_t pk) {
  static_assert(kActS == 8.0f, "exponent shift of kActS");
  uint32_t r;
  asm("v_pk_sub_u16 %0, %1, %2 clamp" : "=v"(r) : "v"(pk_max_i16(pk, 0u)), "s"(0x01800180u));
  return r;
}
// (bf16(lo), bf16(hi)) round to nearest even as one v_cvt_pk_bf16_f32: the empty asm pins the
// packed dword (without it hipcc pushes the packed ReLU back through the conversion and emits
// two one-value conversions joined by a v_perm); the conversion itself stays compiler-visible,
// as it reads MFMA results (the MFMA-to-VALU wait states are the compiler's to insert)
__device__ __forceinline__ uint32_t cvt_pk_bf16(float lo, float hi) {
  const bf2 hb = {static_cast<__bf16>(lo), static_cast<__bf16>(hi)};
  uint32_t r = __builtin_bit_cast(uint32_t, hb);
  asm("" : "+v"(r));
  return r;
}

// Stores of the kept tensors (activations, ReLU' bits, the chains' gradients): read once, by a
// later kernel, long after -- AON_NT_STORE = 1 (A/B build) marks them non-temporal
#ifndef AON_NT_STORE
#define AON_NT_STORE 0
#endif
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <typename V>
__device__ __forceinline__ void kept_store(void* p, V v) {
#if AON_NT_STORE
  __builtin_nontemporal_store(v, static_cast<V*>(p));
#else
  *static_cast<V*>(p) = v;
#endif
}

// two consecutive outputs at true scale: one 8-B fp32 store, or (bf16 mode) one 4-B bf16 store
__device__ __forceinline__ void store2(float* p, float v0, float v1) {
  kept_store(p, u32x2{__float_as_uint(v0), __float_as_uint(v1)});
}
__device__ __forceinline__ void store2(__bf16* p, float v0, float v1) {
  kept_store(p, __builtin_bit_cast(uint32_t, bf2{static_cast<__bf16>(v0), static_cast<__bf16>(v1)}));
}

// four consecutive outputs: one 16-B fp32 store, or one 8-B bf16 store
__device__ __forceinline__ void store4(float* p, float v0, float v1, float v2, float v3) {
  kept_store(p, f4{v0, v1, v2, v3});
}
__device__ __forceinline__ void store4(__bf16* p, float v0, float v1, float v2, float v3) {
  const bf2 a = {static_cast<__bf16>(v0), static_cast<__bf16>(v1)};
  const bf2 b = {static_cast<__bf16>(v2), static_cast<__bf16>(v3)};
  kept_store(p, u32x2{__builtin_bit_cast(uint32_t, a), __builtin_bit_cast(uint32_t, b)});
}

#ifndef AON_TILED
#define AON_TILED 1  // 0: row-major (A/B only: the training forward's stores 15-45% slower)
#endif
// Layout of the tensors the fused training kernels keep for the backward (activations, the
// chains' pre-activation gradients, ReLU' bits): 16 x 16 tiles, each contiguous and row-major,
// element (row, f) of a width-ld tensor at (row / 16) 16 ld + 256 (f / 16) + 16 (row % 16) +
// f % 16.  A tile is one MFMA output fragment, so a wave's epilogue store (64 lanes x 2 or 4
// consecutive values) covers one contiguous 1-KB / 512-B run instead of 16 rows' scattered
// pieces (row-major stores held the bf16 training forward at 2.9 ms; tiled 1.5 ms,
// profiles/r02/ab_tiled), and the weight-gradient GEMM still reads 64-B row runs.  Buffers
// hold act_rows(N) = N rounded up to 16 rows.
__host__ __device__ constexpr int64_t act_rows(int64_t N) { return AON_TILED ? (N + 15) & ~int64_t(15) : N; }
__device__ __forceinline__ int64_t act_base(int64_t row, int ld, int g) {
  return AON_TILED ? (row & ~int64_t(15)) * ld + 16 * (row & 15) + 4 * g : row * ld + 4 * g;
}
// uint2 index of the ReLU' word (row, g): [N][4], or tiled [N/16][64 lanes]
__device__ __forceinline__ int64_t mask_index(int64_t row, int g) {
  return AON_TILED ? (row & ~int64_t(15)) * 4 + 16 * g + (row & 15) : row * 4 + g;
}
constexpr int kTileStride = AON_TILED ? 256 : 16;  // elements between output tiles of one lane
// Whether a sample's kept values are stored.  Tiled: the whole 16-row tile is stored when it
// starts below N -- the kept tensors hold act_rows(N) rows, so its rows past N land in the
// padding (never read: the weight-gradient kernels stop at row N) -- and the test is
// wave-uniform (readfirstlane of the tile's first row), so every store of the epilogues branches
// on SCC instead of masking EXEC around itself (s_and_saveexec / s_cbranch_execz / s_or per
// store).  Row-major (A/B build): row < N.
__device__ __forceinline__ bool keep_row(int64_t row, int64_t N) {
#ifdef AON_ABL_NO_KEEP  // timing-only A/B build: the training kernels store nothing they keep
  return false;
#endif
#if AON_TILED
  const uint64_t t = static_cast<uint64_t>(row & ~int64_t(15));
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(t));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(t >> 32));
  return static_cast<int64_t>((static_cast<uint64_t>(hi) << 32) | lo) < N;
#else
  return row < N;
#endif
}

// bf16 training modes: pos_enc(x) kept for the weight gradients of pts_linears.0 and the skip
// layer's enc columns, bf16 in the tiled layout (act_base) with 128 columns (63..127 zero) --
// whole 128-column tiles for the LDS-DMA dW kernel (aon_gemm n_store).  Lane group g holds
// features 32 k + 8 g .. + 7 of its sample (true scale): one 16-B run of tile 2 k + g / 2; the
// k = 2, 3 runs are the zero tiles.
__device__ __forceinline__ void store_enc_bf(__bf16* base, int64_t row, int g,
                                             const float (&fv)[2][8]) {
  __bf16* eb = base + act_base(row, 128, 0) + 8 * (g & 1) + 256 * (g >> 1);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    if (k < 2) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bf2 pr = {static_cast<__bf16>(fv[k][2 * e]), static_cast<__bf16>(fv[k][2 * e + 1])};
        w[e] = __builtin_bit_cast(uint32_t, pr);
      }
    }
    kept_store(eb + 512 * k, u32x4{w[0], w[1], w[2], w[3]});
  }
}

// The articulated training forward's fp32 pos_enc(x'), tiled (act_base) with EW columns: EW = 64
// keeps every feature (63 zero; the fp16x3 mode's enc-column weight gradients read it, and the
// chain reads x' = columns 0..2); EW = 16 keeps columns 0..15 only (the bf16 modes: their
// weight gradients read store_enc_bf's copy, so the chain's x' is all the fp32 copy serves).
// Lane group g holds features 32 k + 8 g .. + 7: two 16-B stores into tile 2 k + g / 2.
template <int EW>
__device__ __forceinline__ void store_enc_f32(float* base, int64_t row, int g,
                                              const float (&fv)[2][8]) {
  float* e = base + act_base(row, EW, 0) + 8 * (g & 1) + 256 * (g >> 1);
#pragma unroll
  for (int k = 0; k < 2; ++k)
    if (32 * k + 16 * (g >> 1) < EW) {
      kept_store(e + 512 * k, f4{fv[k][0], fv[k][1], fv[k][2], fv[k][3]});
      kept_store(e + 512 * k + 4, f4{fv[k][4], fv[k][5], fv[k][6], fv[k][7]});
    }
}
// x' (columns 0..2) of a store_enc_f32<EW> tensor
__device__ __forceinline__ int64_t enc_x_index(int64_t row, int EW) { return act_base(row, EW, 0); }

#ifndef AON_BF_ST16
#define AON_BF_ST16 1
#endif
#ifndef AON_PK_F16X3_BF
#define AON_PK_F16X3_BF 1  // 0: A/B build -- fp32 ReLU' compares and per-value scaling (RowStore::put)
#endif
template <typename S, typename = void>
struct pk_from_f32 : std::false_type {};
template <typename S>
struct pk_from_f32<S, std::void_t<decltype(S::kPkFromF32)>> : std::bool_constant<S::kPkFromF32> {};
// pairs (r0 = 0, 2) of a tile meet in one 4-value store
// fp32 kept values (the parity mode's activations and the chains' gradients): parts r0 = 0, 2 of
// a tile row meet in ONE 16-B store per lane (the wave writes a whole 1-KB tile) instead of two
// 8-B stores -- the kept stores are issue-bound (profiles/r05/vmcnt_ab/), and the 16-B form cut
// the C5 f16x3 step 14.06 -> 13.38 ms (forward -7%, chain -9%; articulated forward -10%,
// profiles/r05/st16_ab/).  0: the 8-B form (A/B).
#ifndef AON_F32_ST16
#define AON_F32_ST16 1
#endif
template <int NCOL, typename T>
struct Store4 {
  bool ok[NCOL];  // keep_row of each column's sample (wave-uniform when tiled)
  mutable float pend[NCOL][2];
  __device__ __forceinline__ void emit(T* rowp, int pr, int uu, int r0, int c, float v0,
                                       float v1) const {
    // fp32: one 16-B store per tile row (AON_F32_ST16; 0: one 8-B store per part); bf16: the
    // two parts of a tile row meet in one 8-B store (4-B stores: 1.73 -> 1.51 ms forward)
    if (std::is_same<T, float>::value && !AON_F32_ST16) {
      if (ok[c]) store2(rowp + kTileStride * (2 * pr + uu) + r0, v0, v1);
      return;
    }
    if (r0 == 0) {
      pend[c][0] = v0;
      pend[c][1] = v1;
    } else if (ok[c]) {
      store4(rowp + kTileStride * (2 * pr + uu), pend[c][0], pend[c][1], v0, v1);
    }
  }
  // bf16 layers: the packed pair as it is.  AON_BF_ST16 (tiled): the pair's two tiles meet in
  // ONE 16-B store per lane -- lane (g, j) holds 4 features of tile 2pr and 4 of tile 2pr + 1
  // (4g.., 16 + 4g.. of sample j); one v_permlane16_swap per dword trades the odd lane groups'
  // tile-2pr values for the even groups' tile-(2pr + 1) values, after which group g holds 8
  // consecutive features of one tile (g even: features 8 (g / 2).. of tile 2pr; g odd: of tile
  // 2pr + 1) -- a wave's store is the pair's whole 1-KB run, half the store instructions of the
  // 8-B form (the bf16 chain was store-issue-bound: ~6 B/cycle/CU with 8-B stores).  off16:
  // this lane group's element offset of that run from rowp (set by the makers; 0 or 252).
  // Else: parts r0 = 0, 2 of a tile row -> one 8-B store.
  static constexpr bool kPkEpi = true;
  __device__ __forceinline__ uint32_t post_pk(int, int, int, int, uint32_t pk) const { return pk; }
  mutable uint32_t pendw[NCOL];
  mutable uint2 pend0[NCOL];
  int off16 = 0;
  __device__ __forceinline__ void emit_bf(T* rowp, int pr, int uu, int r0, int c, uint32_t pk) const {
    static_assert(std::is_same<T, __bf16>::value, "bf16 layers keep bf16 activations");
    if (r0 == 0) {
      pendw[c] = pk;
      return;
    }
#if AON_BF_ST16 && AON_TILED
    if (uu == 0) {
      pend0[c] = uint2{pendw[c], pk};
      return;
    }
    // every lane takes part in the swaps (EXEC full): only the store is predicated
    const auto s0 = __builtin_amdgcn_permlane16_swap(pend0[c].x, pendw[c], false, false);
    const auto s1 = __builtin_amdgcn_permlane16_swap(pend0[c].y, pk, false, false);
    if (ok[c]) kept_store(rowp + kTileStride * 2 * pr + off16, u32x4{s0[0], s1[0], s0[1], s1[1]});
#else
    if (ok[c]) kept_store(rowp + kTileStride * (2 * pr + uu), u32x2{pendw[c], pk});
#endif
  }
};
// Store4::off16 of lane group g: 16-B run of 8 features of tile 2pr + (g & 1) at column 8 (g / 2),
// relative to act_base(row, ld, g) (which includes 4 g)
__device__ __forceinline__ int st16_off(int g) { return 256 * (g & 1) + 8 * (g >> 1) - 4 * g; }

template <int NCOL, typename T = float>
struct RowStore : Store4<NCOL, T> {
  // fp16x3 layers keeping bf16 (the articulated bf16 mode's forward): a ReLU layer's pair is
  // converted once at activation scale and stored / bit-tested packed (epi_part, put_pk)
  static constexpr bool kPkFromF32 = std::is_same<T, __bf16>::value && AON_F16X3_V2 && AON_PK_F16X3_BF;
  T* rowp[NCOL];  // act_base(row) of each column's sample (stored when ok)
  float s;        // to true scale (a power of two: exact)
  __device__ __forceinline__ void begin_pair(int) const {}
  __device__ __forceinline__ float post(int, int, int, int, float v) const { return v; }
  __device__ __forceinline__ void put(int pr, int uu, int r0, int c, float v0, float v1) const {
    this->emit(rowp[c], pr, uu, r0, c, v0 * s, v1 * s);
  }
  __device__ __forceinline__ void put_pk(int pr, int uu, int r0, int c, uint32_t pk) const {
    this->emit_bf(rowp[c], pr, uu, r0, c, pk);
  }
};

// ReLU' as bits: the training forward records, per sample and lane group g, one 64-bit word
// whose bit 4 t + r is (h[16 t + 4 g + r] > 0) for output tile t (32 B per sample and layer,
// layout [layer][N][4] of uint2), so the backward chains read 1/32 of the bytes of the fp32
// activations for their masks.  Written a byte per output pair (the pair's 2 tiles x 4 rows),
// so nothing is carried across pairs.
// bf16 kept values: a layer's ReLU' word (row, g) gathered in registers byte by byte and stored
// ONCE (8 B) at its last pair, instead of a byte store per pair (+ a zero byte per pair of a
// 128-wide layer): bf16 forward 1.239 -> 1.219 ms, articulated 2.706 -> 2.666 ms
// (profiles/r05/maskword_ab/).  fp32 forwards keep the byte stores (the gathered word spills
// them: 182-207 VGPRs).  0: byte stores everywhere (A/B).
#ifndef AON_MASK_WORD
#define AON_MASK_WORD 1
#endif
template <int NCOL, typename T = float>
struct RowStoreBits : RowStore<NCOL, T> {
  uint8_t* mrow[NCOL];  // bytes of word (row, g) (stored when ok)
  bool narrow;          // 4-pair (128-wide) layer: bytes 4..7 of the word are written as 0
  mutable uint32_t b[NCOL];  // the current pair's 8 bits (byte pr of the word)
  mutable uint32_t wlo[NCOL], whi[NCOL];  // AON_MASK_WORD: bytes 0..3 / 4..7 gathered so far
  // the finished byte of pair pr: kept and, at the layer's last pair, the whole word stored
  __device__ __forceinline__ void byte_done(int pr, int c, uint32_t byte) const {
    if constexpr (AON_MASK_WORD && std::is_same<T, __bf16>::value) {  // (fp32 forwards: spills)
    if (pr < 4) wlo[c] = pr == 0 ? byte : (wlo[c] | (byte << (8 * pr)));
    else whi[c] = pr == 4 ? byte : (whi[c] | (byte << (8 * (pr - 4))));
    if (this->ok[c]) {
      if (pr == 3 && narrow) kept_store(mrow[c], u32x2{wlo[c], 0u});
      if (pr == 7) kept_store(mrow[c], u32x2{wlo[c], whi[c]});
    }
    } else {
    if (this->ok[c]) {
      kept_store(mrow[c] + pr, static_cast<uint8_t>(byte));
      if (narrow) kept_store(mrow[c] + pr + 4, uint8_t{0});
    }
    }
  }
  // bf16 layers: the bits from the packed ReLU output -- part q = 2 uu + r0 / 2 of the pair has
  // its two values' bits at 2q (element 0) and 2q + 1 (element 1): one v_pk_min_u16 gives them at
  // 0 and 16, one v_lshl_or_b32 per part gathers them at 2q and 16 + 2q, and the byte folds the
  // upper ones down by 15 (9 VALU per pair against 25 for the fp32 compares).  A positive fp32
  // below bf16's smallest subnormal rounds to 0 here and its bit reads 0; the bf16 training mode
  // keeps that 0, so the backward masks exactly what the forward stored.
  __device__ __forceinline__ void put_pk(int pr, int uu, int r0, int c, uint32_t pk) const {
    RowStore<NCOL, T>::put_pk(pr, uu, r0, c, pk);
    const uint32_t m = pk_nonzero(pk);
    const int q = 2 * uu + (r0 >> 1);  // compile-time after unrolling
    b[c] = q == 0 ? m : lshl_or(m, 2 * q, b[c]);
    if (q == 3) byte_done(pr, c, (b[c] | (b[c] >> 15)) & 0xFFu);
  }
  __device__ __forceinline__ void put(int pr, int uu, int r0, int c, float v0, float v1) const {
    RowStore<NCOL, T>::put(pr, uu, r0, c, v0, v1);
    bits(pr, uu, r0, c, v0, v1);
  }
  __device__ __forceinline__ void bits(int pr, int uu, int r0, int c, float v0, float v1) const {
    const uint32_t m = (v0 > 0.0f ? 1u : 0u) | (v1 > 0.0f ? 2u : 0u);  // v: post-ReLU, s > 0
    const int bit = 4 * uu + r0;  // within the pair's byte (compile-time after unrolling)
    b[c] = bit == 0 ? m : (b[c] | (m << bit));
    if (uu == 1 && r0 == 2) byte_done(pr, c, b[c] & 0xFFu);
  }
};

// Backward-chain epilogue with ReLU' from those bits (no reads of the fp32
// activations): the layer's word is loaded when its first pair starts.
template <int NCOL, typename T = float>
struct MaskBits : Store4<NCOL, T> {
  const uint2* mrow[NCOL];  // masks + row * 4 + g (read and stored when ok)
  T* rowp[NCOL];            // out + row * ld + 4 g
  float s;
  mutable uint2 m[NCOL];
  __device__ __forceinline__ void begin_pair(int pr) const {
    if (pr == 0) {
#pragma unroll
      for (int c = 0; c < NCOL; ++c) m[c] = this->ok[c] ? *mrow[c] : uint2{0u, 0u};
    }
  }
  __device__ __forceinline__ float post(int pr, int uu, int r, int c, float v) const {
    const int bit = 4 * (2 * pr + uu) + r;
    const uint32_t w = bit < 32 ? m[c].x : m[c].y;
    return (w >> (bit & 31)) & 1u ? v : 0.0f;
  }
  __device__ __forceinline__ void put(int pr, int uu, int r0, int c, float v0, float v1) const {
    this->emit(rowp[c], pr, uu, r0, c, v0 * s, v1 * s);
  }
  // bf16 layers: the mask applied to the packed pair (bf16(0) = 0, so masking after the
  // conversion gives the same bits).  Part q of pair pr needs bits 2q, 2q + 1 of the pair's byte
  // as 16-bit all-ones / zero halves: the byte and its copy shifted up by 15 put them at 2q of
  // each half (once per pair: hipcc shares it between the four parts), then one packed shift
  // left moves bit 2q to the sign and one packed arithmetic shift right spreads it.
  __device__ __forceinline__ uint32_t post_pk(int pr, int uu, int r0, int c, uint32_t pk) const {
    const uint32_t w = pr < 4 ? m[c].x : m[c].y;
    const uint32_t byte = (w >> (8 * (pr & 3))) & 0xFFu;
    const uint32_t z = byte | (byte << 15);
    const short q = static_cast<short>(2 * uu + (r0 >> 1));
    const s2v sel = (__builtin_bit_cast(s2v, z) << s2v{static_cast<short>(15 - 2 * q),
                                                         static_cast<short>(15 - 2 * q)}) >>
                    s2v{15, 15};
    return pk & __builtin_bit_cast(uint32_t, sel);
  }
  __device__ __forceinline__ void put_pk(int pr, int uu, int r0, int c, uint32_t pk) const {
    this->emit_bf(rowp[c], pr, uu, r0, c, pk);
  }
};

template <int NCOL, typename T = float>
__device__ __forceinline__ MaskBits<NCOL, T> mask_bits(const uint2* mbase, T* obase, int ld,
                                                       const int64_t (&rows)[NCOL], int64_t N,
                                                       int g, float s) {
  MaskBits<NCOL, T> mb;
#pragma unroll
  for (int c = 0; c < NCOL; ++c) {
    const bool ok = keep_row(rows[c], N);
    mb.ok[c] = ok;
    mb.mrow[c] = mbase + mask_index(rows[c], g);
    mb.rowp[c] = obase + act_base(rows[c], ld, g);
  }
  mb.off16 = st16_off(g);
  mb.s = s;
  return mb;
}

// NoStore (STORE = false) or a RowStore at y + row * ld (true scale) for the training forward;
// T = the stored element type (fp32, or bf16 in the bf16 training mode)
template <bool STORE, int NCOL, typename T = float>
struct StorePick {
  __device__ __forceinline__ static NoStore make(T*, int, const int64_t (&)[NCOL], int64_t, int) {
    return {};
  }
  __device__ __forceinline__ static NoStore make(T*, int, const int64_t (&)[NCOL], int64_t, int,
                                                 uint2*) {
    return {};
  }
};
template <int NCOL, typename T>
struct StorePick<true, NCOL, T> {
  __device__ __forceinline__ static RowStore<NCOL, T> make(T* base, int ld,
                                                           const int64_t (&rows)[NCOL], int64_t N,
                                                           int g) {
    RowStore<NCOL, T> r;
#pragma unroll
    for (int c = 0; c < NCOL; ++c) {
      r.ok[c] = keep_row(rows[c], N);
      r.rowp[c] = base + act_base(rows[c], ld, g);
    }
    r.off16 = st16_off(g);
    r.s = AON_F16X3_V2 ? 1.0f / kActS : 1.0f / kActScale;
    return r;
  }
  // a ReLU layer: also its ReLU' bits at mbase ([N][4] uint2); ld / 32 output pairs
  __device__ __forceinline__ static RowStoreBits<NCOL, T> make(T* base, int ld,
                                                               const int64_t (&rows)[NCOL],
                                                               int64_t N, int g, uint2* mbase) {
    RowStoreBits<NCOL, T> r;
    static_cast<RowStore<NCOL, T>&>(r) = make(base, ld, rows, N, g);
#pragma unroll
    for (int c = 0; c < NCOL; ++c) {
      r.mrow[c] = reinterpret_cast<uint8_t*>(mbase + mask_index(rows[c], g));
      r.b[c] = 0u;
    }
    r.narrow = ld == 128;
    return r;
  }
};

// ---- backward chains (mlp_bwd.hip, mlp_art_bwd.hip): per-call gradient scale, grad_scale()
// in aon_common.hpp


// epilogue of a finished pair, in 4 parts of 2 values (so it can ride between MFMA steps):
// part q converts v[2q], v[2q+1] of the pair's 8 per-lane values (v[4uu + r] = tile uu, reg r)
// BF: a bf16 layer -- operands unscaled, the accumulator at true scale and already holding the
// bias (layer_h seeds it): one v_cvt_pk_bf16_f32, then ReLU / mask / store on the packed pair
// (kPkEpi policies, see NoStore).
// OBF: a fp16x3 layer whose consumer is a bf16 layer (the view-branch mixed stream's bottleneck):
// its output fragment is bf16 at true scale -- one v_cvt_pk_bf16_f32 of v * 2^-3 (exact), the
// same values the kept (bf16) store gets -- instead of the fp16 hi / lo split.
template <bool RELU, bool BF, int NCOL, int NO, typename Store = NoStore, bool ZB = false,
          bool OBF = false>
__device__ __forceinline__ void epi_part(int q, const f4 (&hh)[2][NCOL], const f4 (&xx)[2][NCOL],
                                         const f4 (&bias)[2], Frag<NO, NCOL>& out, int pr,
                                         const Store& st = Store{}) {
  const int uu = q >> 1, r0 = (q & 1) * 2;
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int c = 0; c < NCOL; ++c) {
    if constexpr (BF && Store::kPkEpi) {
      uint32_t pk = cvt_pk_bf16(hh[uu][c][r0], hh[uu][c][r0 + 1]);
      if (RELU) pk = pk_max_i16(pk, 0u);
      pk = st.post_pk(pr, uu, r0, c, pk);
      st.put_pk(pr, uu, r0, c, pk);
      u4 w = __builtin_bit_cast(u4, out.hi[pr][c]);
      w[q] = pk;
      out.hi[pr][c] = __builtin_bit_cast(h8, w);
      continue;
    }
    float vv[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
#if AON_F16X3_V2
      // fp16x3: one accumulator at scale 2^9 -> activation scale 2^3, plus the (pre-scaled) bias
      float v = BF ? hh[uu][c][r0 + e] : fmaf(hh[uu][c][r0 + e], 1.0f / kWS, bias[uu][r0 + e]);
      (void)xx;
#else
      float v = fmaf(xx[uu][c][r0 + e], 1.0f / kLoScale, hh[uu][c][r0 + e]);
      (void)bias;
#endif
      if (RELU) v = fmaxf(v, 0.0f);
      vv[e] = st.post(pr, uu, r0 + e, c, v);
    }
    if constexpr (BF) {  // bf16 mode: the pair as one v_cvt_pk_bf16_f32, no lo part, no range limit
      // the packed pair goes in as ONE dword of the fragment: ROCm 7.2's clang mis-lowers
      // bit_cast<_Float16>(pair[1]) of a <2 x bfloat> (it yields element 0;
      // tools/diag/bf16_pack_probe.hip), so no bf16 element is extracted
      const bf2 hb = {static_cast<__bf16>(vv[0]), static_cast<__bf16>(vv[1])};
      const uint32_t pk = __builtin_bit_cast(uint32_t, hb);
      st.put_pk(pr, uu, r0, c, pk);
      u4 w = __builtin_bit_cast(u4, out.hi[pr][c]);
      w[q] = pk;
      out.hi[pr][c] = __builtin_bit_cast(h8, w);
      continue;
    }
    if constexpr (OBF) {
      static_assert(AON_F16X3_V2 && !RELU, "OBF: a V2 layer without ReLU (the bottleneck)");
      st.put(pr, uu, r0, c, vv[0], vv[1]);
      const uint32_t pk = cvt_pk_bf16(vv[0] * (1.0f / kActS), vv[1] * (1.0f / kActS));
      u4 w = __builtin_bit_cast(u4, out.hi[pr][c]);
      w[q] = pk;
      out.hi[pr][c] = __builtin_bit_cast(h8, w);
      continue;
    }
#if !(AON_GUARD_PK && AON_F16X3_V2 && AON_FMA_MIX)
    or_ballot(out.ovf, fmaxf(fabsf(vv[0]), fabsf(vv[1])) > kF16Max);
#endif
    if constexpr (RELU && pk_from_f32<Store>::value) {
      // bf16 kept values of a fp16x3 ReLU layer: one conversion at activation scale, rescaled
      // packed, then the bf16 layers' packed store and ReLU' bits from the packed pair (bit =
      // stored value != 0: v > 0 but for fp32 denormals) -- where RowStore::put spent two
      // multiplies, two fp32 compares and their selects, and an 8-B store per tile row
      st.put_pk(pr, uu, r0, c, pk_bf16_unscale(cvt_pk_bf16(vv[0], vv[1])));
    } else {
      st.put(pr, uu, r0, c, vv[0], vv[1]);
    }
#if AON_F16X3_V2 && AON_FMA_MIX
    // hi pair by one v_cvt_pk_f16_f32; lo_e = v_e - hi_e by v_fma_mix_f32 reading the fp16 half
    // in place (exact in fp32), then one more cvt_pk
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    const h2 hp = {static_cast<_Float16>(vv[0]), static_cast<_Float16>(vv[1])};
    const uint32_t hu = __builtin_bit_cast(uint32_t, hp);
#if AON_GUARD_PK
    // range guard: one packed max per pair (ReLU outputs are >= 0: a -0 is negative as i16 and
    // drops out; otherwise the sign bits are cleared first)
    out.m16 = pk_max_i16(out.m16, RELU ? hu : (hu & 0x7FFF7FFFu));
    asm("" : "+v"(out.m16));  // pinned per step, as the ballot chain's SGPRs (or_ballot)
#endif
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
template <typename Net, int LAYER, bool RELU, bool OBF = false, typename P, int NCOL, int NA,
          int NB, int NO, typename Store = NoStore>
__device__ __forceinline__ void layer_h(P& p, const Frag<NA, NCOL>& a,
                                        const Frag<NB, NCOL>& b, Frag<NO, NCOL>& out,
                                        lds_float* bias_l, int g, const Store& st = Store{}) {
  constexpr LayerDesc d = Net::layer(LAYER);
  constexpr int K = d.ka + d.kb;
  constexpr int NP = d.u / 2;
  constexpr int EO = P::kEpiOff;  // epilogue parts of pair p-1 at k-steps EO..EO+3 of pair p
  constexpr bool CMP = !P::f16_block(d.blk0);  // a compact (hi-only) block of the stream
  constexpr bool BF = CMP && !P::kW1;  // bf16 numerics: one MFMA per k-step and tile
  constexpr bool W1 = CMP && P::kW1;   // fp16 weights: two MFMAs, the fp16x3 epilogue
  constexpr bool X1 = !CMP && P::kX1From >= 0 && d.blk0 >= P::kX1From;  // fp16 activations
  constexpr int QIN = K - EO < 0 ? 0 : (K - EO > 4 ? 4 : K - EO);  // parts done inside the loop
  static_assert(d.u % 2 == 0 && NP <= NO && d.ka <= NA && d.kb <= NB, "layer shape");
  f4 phh[2][NCOL], pxx[2][NCOL];  // accumulators of the pair whose epilogue is pending
  f4 pbias[2];                     // V2: that pair's biases, added in its epilogue
  // bf16 layers seed the accumulators with the bias (no epilogue add); each pair's bias is read
  // from LDS one pair ahead, so the first MFMA does not wait on it (zero-bias chains: nothing)
  constexpr bool kBiasC = BF && !Net::kZeroBias;
  f4 nbias[2];
  if (kBiasC) {
#pragma unroll
    for (int uu = 0; uu < 2; ++uu) nbias[uu] = *reinterpret_cast<lds_f4*>(bias_l + d.bias0 + 16 * uu);
  }
#pragma unroll
  for (int pr = 0; pr < NP; ++pr) {
    st.begin_pair(pr);
    f4 hh[2][NCOL], xx[2][NCOL], bias[2];
#pragma unroll
    for (int uu = 0; uu < 2; ++uu) {
      if (kBiasC)
        bias[uu] = nbias[uu];
      else if (!BF)
        bias[uu] = *reinterpret_cast<lds_f4*>(bias_l + d.bias0 + 16 * (2 * pr + uu));
      else
        bias[uu] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < NCOL; ++c) {
#if AON_F16X3_V2
        // fp16x3: the bias joins in the epilogue (no LDS read to wait on); bf16: in the accumulator
        hh[uu][c] = kBiasC ? bias[uu] : f4{0.f, 0.f, 0.f, 0.f};
#else
        hh[uu][c] = bias[uu];
#endif
        xx[uu][c] = f4{0.f, 0.f, 0.f, 0.f};
      }
    }
    if (kBiasC && pr + 1 < NP) {
#pragma unroll
      for (int uu = 0; uu < 2; ++uu)
        nbias[uu] = *reinterpret_cast<lds_f4*>(bias_l + d.bias0 + 16 * (2 * (pr + 1) + uu));
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
          if (BF) {
            hh[uu][c] = mfma_bf(wh, xh, hh[uu][c]);
            (void)xl;
            (void)wl;
            continue;
          }
          hh[uu][c] = mfma16(wh, xh, hh[uu][c]);
          if (X1) {
            (void)xl;
            hh[uu][c] = mfma16(wl, xh, hh[uu][c]);
            continue;
          }
          hh[uu][c] = mfma16(wh, xl, hh[uu][c]);
          if (W1) {
            (void)wl;
            continue;
          }
          hh[uu][c] = mfma16(wl, xh, hh[uu][c]);
#else
          hh[uu][c] = mfma16(wh, xh, hh[uu][c]);
          xx[uu][c] = mfma16(wh, xl, xx[uu][c]);
          xx[uu][c] = mfma16(wl, xh, xx[uu][c]);
#endif
        }
      }
      if (pr > 0 && k >= EO && k - EO < 4)
        epi_part<RELU, BF, NCOL, NO, Store, Net::kZeroBias, OBF>(k - EO, phh, pxx, pbias, out, pr - 1, st);
    }
    if (pr > 0) {
#pragma unroll
      for (int q = QIN; q < 4; ++q)
        epi_part<RELU, BF, NCOL, NO, Store, Net::kZeroBias, OBF>(q, phh, pxx, pbias, out, pr - 1, st);
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
  for (int q = 0; q < 4; ++q)
    epi_part<RELU, BF, NCOL, NO, Store, Net::kZeroBias, OBF>(q, phh, pxx, pbias, out, NP - 1, st);
}

// single-tile head (density / rgb): returns the 16-row tile at activation scale
template <typename Net, int LAYER, typename P, int NCOL, int NA>
__device__ __forceinline__ void head_h(P& p, const Frag<NA, NCOL>& a, f4 (&res)[NCOL],
                                       lds_float* bias_l, int g) {
  constexpr LayerDesc d = Net::layer(LAYER);
  constexpr bool CMP = !P::f16_block(d.blk0);
  constexpr bool BF = CMP && !P::kW1, W1 = CMP && P::kW1;
  constexpr bool X1 = !CMP && P::kX1From >= 0 && d.blk0 >= P::kX1From;
  static_assert(d.u == 1 && d.kb == 0 && d.ka <= NA, "head shape");
  f4 hh[NCOL], xx[NCOL];
  const f4 bias = *reinterpret_cast<lds_f4*>(bias_l + d.bias0);
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
      if (BF) {
        hh[c] = mfma_bf(wh, a.hi[k][c], hh[c]);
        continue;
      }
      hh[c] = mfma16(wh, a.hi[k][c], hh[c]);
      if (!X1) hh[c] = mfma16(wh, a.lo[k][c], hh[c]);
      if (!W1) hh[c] = mfma16(wl, a.hi[k][c], hh[c]);
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
      // true scale (head bias unscaled); bf16 heads: unscaled operands
      res[c][r] = BF ? __fadd_rn(hh[c][r], bias[r]) : fmaf(hh[c][r], 1.0f / (kWS * kActS), bias[r]);
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
#ifndef AON_RING_LEAD
#define AON_RING_LEAD (AON_RING - 1)
#endif
constexpr int kRingLead = AON_RING_LEAD;  // chunks in flight ahead of the one in use
// Weight pipeline: the LDS-DMA ring over the network's stream
template <typename Net, int THREADS>
using WeightPipe = DmaPipe<THREADS, kRing, kChunkH, Net::kStreamBlocks, Net::kBlocks, kRingLead>;
// The bf16 mode's stream is compact: only the hi blocks (block 2c of the fp16x3 stream is block
// c), in the first half of the stream region -- the ring moves half the bytes (the zero lo
// blocks of the fp16x3 layout were ~9% of the bf16 forward and chain, profiles/r02/ab_ring)
template <typename Net, int THREADS, bool BF>
using WeightPipeP = typename std::conditional<
    BF, DmaPipe<THREADS, kRing, kChunkH, Net::kStreamBlocks / 2, Net::kBlocks / 2, kRingLead>,
    WeightPipe<Net, THREADS>>::type;
constexpr int kLdsWeights = kRing * kChunkH * 64;  // f4

#ifndef AON_WAVES_H
#define AON_WAVES_H 8  // waves per workgroup at 16 samples per wave (2 waves per SIMD either way)
#endif

// BF: the bf16 training kernels -- at 32 samples per wave (NCOL = 2) they keep 8 waves (2 per
// SIMD): bf16 activations carry no lo part, so a wave's input and output fragments take 64 + 64
// VGPRs where fp16x3 needs 256 (its NCOL = 2 runs 4 waves, one per SIMD)
#ifndef AON_BF_NCOL_FWD
#define AON_BF_NCOL_FWD 1  // samples per wave / 16 of the bf16 training forward
#endif
#ifndef AON_BF_NCOL_BWD
#define AON_BF_NCOL_BWD 2  // ... and of the bf16 backward chain
#endif
constexpr int kBfNcolFwd = AON_BF_NCOL_FWD, kBfNcolBwd = AON_BF_NCOL_BWD;
template <int NCOL, bool BF = false>
struct GeomH {
  static constexpr int kWaves = (NCOL == 1 || BF) ? AON_WAVES_H : 4;
  static constexpr int kThreads = 64 * kWaves;
  static constexpr int kRowsPerWave = 16 * NCOL;
  static constexpr int kRowsPerBlock = kRowsPerWave * kWaves;
  static constexpr int kWavesPerSimd = kWaves / 4;  // __launch_bounds__' occupancy request
};

}  // namespace mlp
}  // namespace aon
