// Fused NeRFMLP render forward on v_mfma_f32_32x32x16_f16 (AON_PREC_F16X3_M32, ABI 12).
//
// Same numerics as mlp_f16x3.hip (the fp16x3 split: x = x_hi + x_lo, a MAC = w_hi x_hi +
// w_hi x_lo + w_lo x_hi into ONE fp32 accumulator, activations at 2^3, weights at 2^6, the
// range guard), on the 32 x 32 x 16 MFMA instead of the 16 x 16 x 32 one.  Why: an MFMA holds
// its SIMD's vector issue for 8 cycles whatever its shape (MI355X_MICROARCH.md, 'vector-
// instruction ISSUE cost'), so beside a 16-cycle 16x16x32 only 8 issue cycles remain for the
// epilogue VALU and the weight-fragment LDS reads of a step -- the 16x16 kernel's ~1.25 VALU +
// 0.75 ds_read_b128 per MFMA fill them, and it runs at 0.68 of the measured fp16 MFMA peak with
// its waves waiting 41% of their cycles.  A 32x32x16 does twice the MACs in 32 cycles with the
// same 8-cycle hold: 24 free issue cycles per MFMA, and each 1-KB weight fragment feeds twice
// the MACs (32 samples per wave), so the LDS bytes per MAC halve.
//
// Geometry: a wave owns 32 samples (the MFMA's N = lane & 31), one wave per SIMD (the wave
// holds its layer's input AND output activations as fp16 hi / lo fragments: 2 x 128 registers,
// plus the encodings, accumulators and prefetched weights -- the 512-register budget of one
// wave per SIMD), 4 waves = 128 samples per workgroup sharing one LDS-DMA weight ring
// (mlp_pipe.hpp DmaPipe, 3 x 32 KB).  Feature-major as before: D[out][sample] = W . H.  A 32 x 32
// output tile's accumulator is TWO 16-deep k-steps of the next layer's B operand with no data
// movement: lane l (s = l >> 5) holds rows 8 (r / 4) + 4 s + r % 4 (r = 0..15) of sample
// l & 31; registers 0..7 form k-step 2t, 8..15 k-step 2t + 1, and the pack orders the next
// layer's weight columns to match (feature_m32).  Tile t's epilogue (scale + bias, ReLU, the
// hi / lo split and its range test: 8 pairs of values) rides one pair per k-step on the MFMAs
// of tile t + 1.  Weight stream: one 1-KB block per (output tile, k-step, hi | lo), lane l
// holding W[32 u + (l & 31)][feature(k, 8 s .. 8 s + 7)] -- one ds_read_b128 per lane is one A
// operand.  Heads (density: 1 row, rgb: 3 rows) are one 32-row tile each (1.6% of the MACs
// issued are padding rows).
#include "mlp_f16x3_core.hpp"

namespace aon {
namespace m32 {

using mlp::h8;
using mlp::LayerDesc;
using mlp::kActS;
using mlp::kWS;
using mlp::kF16Max;
using mlp::lds_float;
using mlp::lds_f4;

typedef float f16v __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f16v mfma32(h8 a, h8 b, f16v c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// layer table: ka / kb = 16-feature k-steps of segment A (previous layer's output, fragment
// order) / B (encodings computed in-register, natural order); u = 32-row output tiles;
// blk0 = first 1-KB block (2 per (u, k)); bias0 = first bias float (32 u per layer)
enum { L0 = 0, L1, L2, L3, L4, L5, L6, L7, LDEN, LBOT, LVIEW, LRGB, kNumLayers };
constexpr LayerDesc kLayers[kNumLayers] = {
    {0, 4, 8, 0, 63, 256, 0, 0},             // pts_linears.0   256 x 63
    {16, 0, 8, 256, 0, 256, 64, 256},        // pts_linears.1
    {16, 0, 8, 256, 0, 256, 320, 512},       // pts_linears.2
    {16, 0, 8, 256, 0, 256, 576, 768},       // pts_linears.3
    {16, 0, 8, 256, 0, 256, 832, 1024},      // pts_linears.4
    {16, 4, 8, 256, 63, 256, 1088, 1280},    // pts_linears.5   256 x (256 + 63)
    {16, 0, 8, 256, 0, 256, 1408, 1536},     // pts_linears.6
    {16, 0, 8, 256, 0, 256, 1664, 1792},     // pts_linears.7
    {16, 0, 1, 256, 0, 1, 1920, 2048},       // density_layer     1 x 256
    {16, 0, 8, 256, 0, 256, 1952, 2080},     // bottleneck_layer 256 x 256
    {16, 2, 4, 256, 27, 128, 2208, 2336},    // views_linear.0  128 x (256 + 27)
    {8, 0, 1, 128, 0, 3, 2352, 2464},        // rgb_layer         3 x 128
};
constexpr int kBlocks = 2368;
constexpr int kStreamBlocks = 2368;  // 74 chunks of 32
constexpr int kBiasFloats = 2496;
constexpr size_t kStreamBytes = (size_t)kStreamBlocks * 1024;
constexpr size_t kPackedBytes = kStreamBytes + (size_t)kBiasFloats * 4 + mlp::kStatusBytes;

constexpr bool layout_ok() {
  int blk = 0, bias = 0;
  for (int i = 0; i < kNumLayers; ++i) {
    const LayerDesc d = kLayers[i];
    if (d.blk0 != blk || d.bias0 != bias) return false;
    if (d.len_a > 16 * d.ka || d.len_b > 16 * d.kb || d.out_real > 32 * d.u) return false;
    blk += (d.ka + d.kb) * d.u * 2;
    bias += d.u * 32;
  }
  return blk == kBlocks && bias == kBiasFloats && kStreamBlocks % 64 == 0;
}
static_assert(layout_ok(), "inconsistent 32x32 MLP stream layout");

// Input feature of segment-A k-step k, lane half s, element i: the previous layer's output
// row held there (D layout above: k-step 2t + h <- registers 8 h .. 8 h + 7 of tile t)
__host__ __device__ constexpr int feature_a(int k, int s, int i) {
  return 32 * (k >> 1) + 16 * (k & 1) + 8 * (i >> 2) + 4 * s + (i & 3);
}
// segment B (in-register encodings): natural order
__host__ __device__ constexpr int feature_b(int k, int s, int i) { return 16 * k + 8 * s + i; }

constexpr int kThreads = 256;  // 4 waves, one per SIMD
constexpr int kRowsPerWave = 32;
constexpr int kRowsPerBlock = kRowsPerWave * 4;
constexpr int kChunk = 32;  // 1-KB blocks per ring chunk
constexpr int kRing = 3;
using Pipe = mlp::DmaPipe<kThreads, kRing, kChunk, kStreamBlocks, kBlocks, kRing - 1>;
constexpr int kLdsWeights = kRing * kChunk * 64;  // f4

#ifndef AON_M32_PREFETCH
#define AON_M32_PREFETCH 3
#endif

// weight fragments of the next D (hi, lo) steps, in stream order (the step after block b is
// always b + 2); the chunk's ring barrier is taken at its first block
template <int D>
struct Frags {
  Pipe& p;
  f4 nh[D], nl[D];
  __device__ __forceinline__ explicit Frags(Pipe& pp) : p(pp) {}
  __device__ __forceinline__ void fetch(int blk, f4& h, f4& l) {
    if (blk >= kBlocks) return;
    if (blk % kChunk == 0) p.begin(blk / kChunk);
    h = p.block(blk);
    l = p.block(blk + 1);
  }
  __device__ __forceinline__ void start() {
#pragma unroll
    for (int i = 0; i < D; ++i) fetch(2 * i, nh[i], nl[i]);
  }
  __device__ __forceinline__ void take(int blk, h8& wh, h8& wl) {
    wh = mlp::as_h8(nh[0]);
    wl = mlp::as_h8(nl[0]);
#pragma unroll
    for (int i = 0; i + 1 < D; ++i) {
      nh[i] = nh[i + 1];
      nl[i] = nl[i + 1];
    }
    fetch(blk + 2 * D, nh[D - 1], nl[D - 1]);
    __builtin_amdgcn_sched_barrier(0);
  }
};

template <int N>
struct Frag {
  h8 hi[N], lo[N];
  uint32_t m16 = 0;  // packed i16 max of the |fp16 hi| bits split into this set (range guard)
};

// values (at activation scale, 8 of them) -> hi / lo fragment, range bits into m16
__device__ __forceinline__ void split8(const float (&v)[8], h8& hi, h8& lo, uint32_t& m16) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const _Float16 h = static_cast<_Float16>(v[j]);
    hi[j] = h;
    lo[j] = static_cast<_Float16>(__builtin_fmaf(static_cast<float>(h), -1.0f, v[j]));
    const uint32_t b = __builtin_bit_cast(uint16_t, h) & 0x7FFFu;
    m16 = b > m16 ? b : m16;
  }
}

// epilogue of pair q (registers 2q, 2q + 1) of an output tile: scale + bias, ReLU, the hi / lo
// split into the next layer's fragment (k-step 2t + q / 4, dword q % 4)
template <bool RELU, int NO>
__device__ __forceinline__ void epi_pair(int q, const f16v& acc, lds_float* bias_t,
                                         Frag<NO>& out, int t) {
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  // rows 8 (q / 2) + 4 s + 2 (q % 2) + e: bias_t already points at this lane half's 4 s
  const float b0 = bias_t[8 * (q >> 1) + 2 * (q & 1)];
  const float b1 = bias_t[8 * (q >> 1) + 2 * (q & 1) + 1];
  float v0 = fmaf(acc[2 * q], 1.0f / kWS, b0);
  float v1 = fmaf(acc[2 * q + 1], 1.0f / kWS, b1);
  if (RELU) {
    v0 = fmaxf(v0, 0.0f);
    v1 = fmaxf(v1, 0.0f);
  }
  // the packed conversions as written instructions: left to itself hipcc rebuilt the pair a
  // second time (two v_cvt_f16_f32 + v_perm) for the range test, or widened the fp16 halves
  // with separate conversions instead of v_fma_mix_f32 (each asm block costs one s_nop 0)
  uint32_t hu, lu;
  asm("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(hu) : "v"(v0), "v"(v1));
  out.m16 = mlp::pk_max_i16(out.m16, RELU ? hu : (hu & 0x7FFF7FFFu));
  asm("" : "+v"(out.m16));
  float d0, d1;
  asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mix_f32 %3, %1, -1.0, %4 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
      "v_cvt_pk_f16_f32 %5, %0, %3"
      : "=&v"(d0), "+v"(hu), "+v"(v0), "=&v"(d1), "+v"(v1), "=&v"(lu));
  const int kk = 2 * t + (q >> 2);
  u4 wh = __builtin_bit_cast(u4, out.hi[kk]);
  u4 wl = __builtin_bit_cast(u4, out.lo[kk]);
  wh[q & 3] = hu;
  wl[q & 3] = lu;
  out.hi[kk] = __builtin_bit_cast(h8, wh);
  out.lo[kk] = __builtin_bit_cast(h8, wl);
}

// one hidden layer: out = act(W [a ; b] + bias) as next-layer fragments; tile t's epilogue
// is spread over the first 8 k-steps of tile t + 1
template <int LAYER, bool RELU, typename F, int NA, int NB, int NO>
__device__ __forceinline__ void layer(F& fr, const Frag<NA>& a, const Frag<NB>& b, Frag<NO>& out,
                                      lds_float* bias_l) {
  constexpr LayerDesc d = kLayers[LAYER];
  constexpr int K = d.ka + d.kb;
  constexpr int U = d.u;
  static_assert(d.ka <= NA && d.kb <= NB && 2 * U <= NO, "layer shape");
  f16v pend;
#pragma unroll
  for (int t = 0; t < U; ++t) {
    f16v acc = {};
#pragma unroll
    for (int k = 0; k < K; ++k) {
      h8 wh, wl;
      fr.take(d.blk0 + 2 * (t * K + k), wh, wl);
      const int ia = k < NA ? k : 0, ib = (k >= d.ka && k - d.ka < NB) ? k - d.ka : 0;
      const h8 xh = k < d.ka ? a.hi[ia] : b.hi[ib];
      const h8 xl = k < d.ka ? a.lo[ia] : b.lo[ib];
      acc = mfma32(wh, xh, acc);
      acc = mfma32(wh, xl, acc);
      acc = mfma32(wl, xh, acc);
      if (t > 0 && k < 8) epi_pair<RELU>(k, pend, bias_l + d.bias0 + 32 * (t - 1), out, t - 1);
    }
    if (t > 0) {
#pragma unroll
      for (int q = K < 8 ? K : 8; q < 8; ++q)
        epi_pair<RELU>(q, pend, bias_l + d.bias0 + 32 * (t - 1), out, t - 1);
    }
    pend = acc;
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) epi_pair<RELU>(q, pend, bias_l + d.bias0 + 32 * (U - 1), out, U - 1);
}

// one-tile head (density / rgb): its accumulator at true scale plus the bias (rows 0..2 live in
// registers 0..2 of the lanes with s = 0)
template <int LAYER, typename F, int NA>
__device__ __forceinline__ void head(F& fr, const Frag<NA>& a, float (&res)[4], lds_float* bias_l) {
  constexpr LayerDesc d = kLayers[LAYER];
  static_assert(d.u == 1 && d.kb == 0 && d.ka <= NA, "head shape");
  f16v acc = {};
#pragma unroll
  for (int k = 0; k < d.ka; ++k) {
    h8 wh, wl;
    fr.take(d.blk0 + 2 * k, wh, wl);
    acc = mfma32(wh, a.hi[k], acc);
    acc = mfma32(wh, a.lo[k], acc);
    acc = mfma32(wl, a.hi[k], acc);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) res[r] = fmaf(acc[r], 1.0f / (kWS * kActS), bias_l[d.bias0 + r]);
}

// MODE 0: (rays_o, rays_d, viewdirs, t); MODE 1: encoded x (N, 63), condition (B, 27)
template <int MODE>
__global__ __launch_bounds__(kThreads, 1) void k_mlp_fwd_m32(
    const f4* __restrict__ wstream, const float* __restrict__ bias_g, const float* __restrict__ in0,
    const float* __restrict__ in1, const float* __restrict__ in2, const float* __restrict__ in3,
    int64_t B, int S, int act, float* __restrict__ raw) {
  static_assert((kLdsWeights + kBiasFloats / 4) * 16 <= 160 * 1024, "LDS");
  __shared__ f4 smem[kLdsWeights + kBiasFloats / 4];
  float* bias_s = reinterpret_cast<float*>(smem + kLdsWeights);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int s = lane >> 5, n = lane & 31;
  const int64_t N = B * S;

  Pipe p;
  p.wbuf = smem;
  p.src = wstream;
  p.tid = tid;
  p.lane = lane;
  p.start();
  for (int i = tid; i < kBiasFloats; i += kThreads) bias_s[i] = bias_g[i];

  // encodings: k-step k, lane half s, element i <-> feature 16 k + 8 s + i
  Frag<4> enc;
  Frag<2> venc;
  const int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + wave * kRowsPerWave + n;
  {
    const int64_t rr = row < N ? row : N - 1;
    const int64_t ray = rr / S;
    float ev[4][8], vv[2][8];
    if (MODE == 0) {
      const float* ro = in0 + 3 * ray;
      const float* rd = in1 + 3 * ray;
      const float* vd = in2 + 3 * ray;
      const float tt = in3[rr];
      const float x0 = __fadd_rn(ro[0], __fmul_rn(tt, rd[0]));
      const float x1 = __fadd_rn(ro[1], __fmul_rn(tt, rd[1]));
      const float x2 = __fadd_rn(ro[2], __fmul_rn(tt, rd[2]));
      const float v0 = vd[0], v1 = vd[1], v2 = vd[2];
      auto encode = [&](auto fast) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
          for (int e = 0; e < 8; ++e)
            ev[k][e] = pos_enc_feature_fast(x0, x1, x2, feature_b(k, s, e), 0, 10, fast.value);
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
          for (int e = 0; e < 8; ++e)
            vv[k][e] = pos_enc_feature_fast(v0, v1, v2, feature_b(k, s, e), 0, 4, fast.value);
      };
      // every argument of the wave inside sin_small's range (the render's points: |x| < ~10,
      // arguments < 2^13): ~20 VALU per sine instead of sinf's ~150 -- the same bits
      if (pos_enc_fast_ok(x0, x1, x2, 10) && pos_enc_fast_ok(v0, v1, v2, 4))
        encode(std::true_type{});
      else
        encode(std::false_type{});
    } else {
      const float* x = in0 + rr * 63;
      const float* cd = in1 + ray * 27;
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int f = feature_b(k, s, e);
          ev[k][e] = f < 63 ? x[f] : 0.f;
        }
#pragma unroll
      for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int f = feature_b(k, s, e);
          vv[k][e] = f < 27 ? cd[f] : 0.f;
        }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
#pragma unroll
      for (int e = 0; e < 8; ++e) ev[k][e] *= kActS;
      split8(ev[k], enc.hi[k], enc.lo[k], enc.m16);
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
#pragma unroll
      for (int e = 0; e < 8; ++e) vv[k][e] *= kActS;
      split8(vv[k], venc.hi[k], venc.lo[k], venc.m16);
    }
  }

  Frags<AON_M32_PREFETCH> fr(p);
  fr.start();  // begin(0): chunk 0 landed; its barrier also publishes bias_s
  lds_float* bias_l = mlp::opaque_lds(bias_s + 4 * s);  // this lane half's rows of the table
  Frag<1> none;
  Frag<16> x, y;
  layer<L0, true>(fr, none, enc, x, bias_l);   // model.py:95-101
  layer<L1, true>(fr, x, none, y, bias_l);
  layer<L2, true>(fr, y, none, x, bias_l);
  layer<L3, true>(fr, x, none, y, bias_l);
  layer<L4, true>(fr, y, none, x, bias_l);
  layer<L5, true>(fr, x, enc, y, bias_l);      // skip: cat[h, enc] (model.py:102-103)
  layer<L6, true>(fr, y, none, x, bias_l);
  layer<L7, true>(fr, x, none, y, bias_l);
  float dens[4], rgb[4];
  lds_float* bias_h = mlp::opaque_lds(bias_s);  // heads: rows 0..3 (lane half 0)
  head<LDEN>(fr, y, dens, bias_h);              // model.py:105-107
  layer<LBOT, false>(fr, y, none, x, bias_l);   // bottleneck, no activation (model.py:109)
  layer<LVIEW, true>(fr, x, venc, y, bias_l);   // cat[bottleneck, enc_dir] + ReLU (:110-116)
  head<LRGB>(fr, y, rgb, bias_h);               // model.py:118
  if (s == 0 && row < N) {
    const f4 o = {act_rgb(rgb[0], act), act_rgb(rgb[1], act), act_rgb(rgb[2], act),
                  act_sigma(dens[0], act)};
    *reinterpret_cast<f4*>(raw + 4 * row) = o;
  }
  // range guard: a value split past fp16's range anywhere in the wave
  const uint32_t m = x.m16 | y.m16;
  const bool bad = (m & 0x7FFFu) >= 0x7C00u || ((m >> 16) & 0x7FFFu) >= 0x7C00u ||
                   enc.m16 >= 0x7C00u || venc.m16 >= 0x7C00u;
  mlp::range_report(bias_g + kBiasFloats, __builtin_amdgcn_ballot_w64(bad));
}

// ---- pack: torch [out][in] fp32 -> the 32x32 stream (hi / lo fp16 blocks at the 2^6 weight
// scale) + biases (hidden layers at the 2^3 activation scale, heads at true scale)
struct PackArgs {
  const float* w[kNumLayers];
  const float* b[kNumLayers];
};

__global__ void k_pack_m32(PackArgs a, float* __restrict__ out_f) {
  const int64_t nhalf = (int64_t)kStreamBlocks * 512;
  _Float16* out = reinterpret_cast<_Float16*>(out_f);
  float* bias_out = out_f + (int64_t)kStreamBlocks * 256;
  const int64_t total = nhalf + kBiasFloats;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    if (e < nhalf) {
      const int blk = static_cast<int>(e >> 9);
      const int l = static_cast<int>((e >> 3) & 63), i = static_cast<int>(e & 7);
      float w = 0.f;
      bool lo_part = false;
      if (blk < kBlocks) {
        int li = 0;
        while (li + 1 < kNumLayers && kLayers[li + 1].blk0 <= blk) ++li;
        const LayerDesc d = kLayers[li];
        const int K = d.ka + d.kb;
        const int q = (blk - d.blk0) >> 1;
        lo_part = ((blk - d.blk0) & 1) != 0;
        const int u = q / K, k = q % K;
        const int o = 32 * u + (l & 31), s = l >> 5;
        int col = -1;
        if (k < d.ka) {
          const int f = feature_a(k, s, i);
          col = f < d.len_a ? f : -1;
        } else {
          const int f = feature_b(k - d.ka, s, i);
          col = f < d.len_b ? d.len_a + f : -1;
        }
        if (o < d.out_real && col >= 0) w = a.w[li][(int64_t)o * (d.len_a + d.len_b) + col];
      }
      w *= kWS;  // exact (power of two)
      const _Float16 h = static_cast<_Float16>(w);
      out[e] = lo_part ? static_cast<_Float16>(w - static_cast<float>(h)) : h;
      if (!lo_part && !(fabsf(w) <= kF16Max))  // range guard: status 2 (mlp_f16x3.hip k_pack_h)
        *reinterpret_cast<uint32_t*>(bias_out + kBiasFloats) = 2u;
    } else {
      const int i = static_cast<int>(e - nhalf);
      int li = 0;
      while (li + 1 < kNumLayers && kLayers[li + 1].bias0 <= i) ++li;
      const int o = i - kLayers[li].bias0;
      const float bs = kLayers[li].u == 1 ? 1.0f : kActS;
      bias_out[i] = o < kLayers[li].out_real ? a.b[li][o] * bs : 0.f;
    }
  }
}

}  // namespace m32

namespace mlp {

size_t packed_bytes_m32() { return m32::kPackedBytes; }

int pack_m32(const float* const* w, const float* const* b, void* packed, hipStream_t stream) {
  m32::PackArgs a;
  for (int i = 0; i < m32::kNumLayers; ++i) {
    a.w[i] = w[i];
    a.b[i] = b[i];
  }
  const hipError_t e = hipMemsetAsync(static_cast<char*>(packed) + m32::kStreamBytes +
                                          (size_t)m32::kBiasFloats * 4,
                                      0, kStatusBytes, stream);
  if (e != hipSuccess) return static_cast<int>(e);
  const int64_t total = (int64_t)m32::kStreamBlocks * 512 + m32::kBiasFloats;
  hipLaunchKernelGGL(m32::k_pack_m32, grid_for(total, 256, 4096), 256, 0, stream, a,
                     static_cast<float*>(packed));
  return launch_status("aon_mlp_pack");
}

int launch_m32(int mode, const void* packed, const float* a0, const float* a1, const float* a2,
               const float* a3, int64_t B, int S, int act, float* raw, hipStream_t stream) {
  const int64_t N = B * S;
  const f4* ws = static_cast<const f4*>(packed);
  const float* bias = reinterpret_cast<const float*>(static_cast<const char*>(packed) + m32::kStreamBytes);
  const int grid = static_cast<int>((N + m32::kRowsPerBlock - 1) / m32::kRowsPerBlock);
  if (mode == 0)
    hipLaunchKernelGGL(m32::k_mlp_fwd_m32<0>, grid, m32::kThreads, 0, stream, ws, bias, a0, a1, a2,
                       a3, B, S, act, raw);
  else
    hipLaunchKernelGGL(m32::k_mlp_fwd_m32<1>, grid, m32::kThreads, 0, stream, ws, bias, a0, a1, a2,
                       a3, B, S, act, raw);
  return launch_status("aon_mlp_fwd");
}

}  // namespace mlp
}  // namespace aon
