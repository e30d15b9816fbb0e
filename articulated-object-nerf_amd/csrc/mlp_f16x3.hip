// Fused NeRFMLP forward on fp16 MFMA with a 3-product hi/lo split ("fp16x3").
//
// Every operand x is carried as x_hi = fp16(x) and x_lo = fp16(x - x_hi) (x - x_hi is exact in
// fp32): together ~22 significant bits.  A weight-activation product is
// w_hi*x_hi + w_hi*x_lo + w_lo*x_hi (the dropped w_lo*x_lo term is 2^-22 relative), three
// v_mfma_f32_16x16x32_f16 into ONE fp32 accumulator.  That is 3 fp16 MFMAs per 32-deep k-step
// where the fp32 path needs 8 v_mfma_f32_16x16x4_f32 of twice the cycles: 16/3 = 5.3x the
// arithmetic rate at fp32-class accuracy (measured against the reference in
// tests/test_gpu_parity.py).  Scales (exact powers of two, mlp_layout.hpp AON_F16X3_V2):
// activations ride at 2^3 (kActS) and weights at 2^6 (kWS), so the unscaled lo parts stay
// normal in fp16 for |activation| >= 2^-6 and the products share the accumulator at 2^9; the
// epilogue folds 2^-6 and the bias into one fma.  fp16 then bounds a hidden activation at
// |x| < 65504 / 2^3 ~ 8188: every split value is range-tested and a wave that meets one sets
// the pack's status word (range guard, mlp_f16x3_core.hpp or_ballot; aon_mlp_read_status),
// and the callers fall back to the fp32 path or refuse the training step.
//
// Structure (mlp_layout.hpp kLayersH): feature-major tiles as in mlp.hip; a wave owns 16*NCOL
// samples; output tiles are produced in pairs (u, u+1) whose accumulators, converted in the
// epilogue, ARE the next layer's B operand for one 32-feature k-step (lane group g holds rows
// 4g..4g+3 of both tiles) -- no LDS round trip; the epilogue of pair p overlaps the MFMAs of
// pair p+1.  Weights stream through the same chunked LDS pipeline (mlp_pipe.hpp).
#include "mlp_f16x3_core.hpp"

namespace aon {
namespace mlp {

#ifndef AON_STASH_REGS
#define AON_STASH_REGS 0  // 1: keep the encodings in VGPRs instead of parking them in LDS
#endif

#ifndef AON_STAGGER
#define AON_STAGGER 0  // 1: waves 4-7 run their epilogues 4 k-steps later (A/B: no gain, profiles/r02/ab_stagger)
#endif

// The layer sequence of k_mlp_fwd_f16x3 (model.py:95-120), instantiated per FragPipe type: the
// two halves of the workgroup differ in the k-step of their epilogues (FragPipe EOFF).
// per-lane LDS stash of the encodings: enc k-steps 0, 1 and venc, hi and lo (fp16x3) or hi only
// (bf16: no lo part); slot (c, i) at stash[64 (kStashPer c + i)]
template <bool BF>
__host__ __device__ constexpr int stash_per() { return BF ? 3 : 6; }
template <bool BF>
__device__ __forceinline__ int enc_slot(int c, int k, int lo) { return BF ? 3 * c + k : 6 * c + 2 * k + lo; }
template <bool BF>
__device__ __forceinline__ int venc_slot(int c, int lo) { return BF ? 3 * c + 2 : 6 * c + 4 + lo; }

template <int NCOL, bool STORE, typename T, typename FP>
__device__ __forceinline__ void vanilla_layers(FP& fp, Frag<2, NCOL>& enc, Frag<1, NCOL>& venc,
                                               Frag<8, NCOL>& x, Frag<8, NCOL>& y, f4* stash,
                                               float* bias_s, int g, int wave,
                                               const int64_t (&rows)[NCOL], int64_t N, int act,
                                               float* __restrict__ raw, const TrainStore& ts) {
  constexpr bool BF = std::is_same<T, __bf16>::value;
  fp.start();  // begin(0): chunk 0 landed; the barrier also publishes bias_s
#if AON_PRIO_HALF
  if (wave >= GeomH<NCOL>::kWaves / 2) __builtin_amdgcn_s_setprio(AON_PRIO_HALF);
#endif
  lds_float* bias_l = opaque_lds(bias_s + 4 * g);  // this lane group's rows of the bias table

  Frag<1, NCOL> none;
  using SP = StorePick<STORE, NCOL, T>;
  // the kept activations (training forward): fp32, or bf16 in the bf16 training mode
  T* const th = reinterpret_cast<T*>(ts.h);
  T* const tbot = reinterpret_cast<T*>(ts.bot);
  T* const thv = reinterpret_cast<T*>(ts.hv);
  const int64_t hs = act_rows(N) * 256;  // one pts_linears output in ts.h
  const int64_t ms = act_rows(N) * 4;    // one layer's ReLU' bits in ts.masks
  layer_h<NetVanillaH, L0, true>(fp, none, enc, x, bias_l, g, SP::make(th, 256, rows, N, g, ts.masks));
  layer_h<NetVanillaH, L1, true>(fp, x, none, y, bias_l, g, SP::make(th + 1 * hs, 256, rows, N, g, ts.masks + 1 * ms));
  layer_h<NetVanillaH, L2, true>(fp, y, none, x, bias_l, g, SP::make(th + 2 * hs, 256, rows, N, g, ts.masks + 2 * ms));
  layer_h<NetVanillaH, L3, true>(fp, x, none, y, bias_l, g, SP::make(th + 3 * hs, 256, rows, N, g, ts.masks + 3 * ms));
  layer_h<NetVanillaH, L4, true>(fp, y, none, x, bias_l, g, SP::make(th + 4 * hs, 256, rows, N, g, ts.masks + 4 * ms));
#pragma unroll
  for (int c = 0; c < NCOL && !AON_STASH_REGS; ++c)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      enc.hi[k][c] = __builtin_bit_cast(h8, stash[64 * enc_slot<BF>(c, k, 0)]);
      if (!BF) enc.lo[k][c] = __builtin_bit_cast(h8, stash[64 * enc_slot<BF>(c, k, 1)]);
    }
  // skip: cat[h, enc] (model.py:102-103)
  layer_h<NetVanillaH, L5, true>(fp, x, enc, y, bias_l, g, SP::make(th + 5 * hs, 256, rows, N, g, ts.masks + 5 * ms));
  layer_h<NetVanillaH, L6, true>(fp, y, none, x, bias_l, g, SP::make(th + 6 * hs, 256, rows, N, g, ts.masks + 6 * ms));
  layer_h<NetVanillaH, L7, true>(fp, x, none, y, bias_l, g, SP::make(th + 7 * hs, 256, rows, N, g, ts.masks + 7 * ms));
  f4 dens[NCOL], rgb[NCOL];
  head_h<NetVanillaH, LDEN>(fp, y, dens, bias_l, g);             // model.py:105-107
  // bottleneck, no activation (model.py:109)
  layer_h<NetVanillaH, LBOT, false>(fp, y, none, x, bias_l, g, SP::make(tbot, 256, rows, N, g));
#pragma unroll
  for (int c = 0; c < NCOL && !AON_STASH_REGS; ++c) {
    venc.hi[0][c] = __builtin_bit_cast(h8, stash[64 * venc_slot<BF>(c, 0)]);
    if (!BF) venc.lo[0][c] = __builtin_bit_cast(h8, stash[64 * venc_slot<BF>(c, 1)]);
  }
  // cat[bottleneck, enc_dir] + ReLU (:110-116)
  layer_h<NetVanillaH, LVIEW, true>(fp, x, venc, y, bias_l, g, SP::make(thv, 128, rows, N, g, ts.masks + 8 * ms));
  head_h<NetVanillaH, LRGB>(fp, y, rgb, bias_l, g);              // model.py:118

  if (g == 0) {
#pragma unroll
    for (int c = 0; c < NCOL; ++c) {
      if (rows[c] < N) {
        const float s = AON_F16X3_V2 ? 1.0f : 1.0f / kActScale;  // V2 heads are at true scale
        float sig = dens[c][0] * s;
        if (STORE && ts.noise) sig = __fadd_rn(sig, ts.noise[rows[c]]);  // raw_sigma + noise
        const f4 o = {act_rgb(rgb[c][0] * s, act), act_rgb(rgb[c][1] * s, act),
                      act_rgb(rgb[c][2] * s, act), act_sigma(sig, act)};
#ifdef AON_ABL_NO_RAW_STORE  // timing-only A/B build (fused-pipeline question): no raw store
        if (__builtin_isnan(o[0] + o[1] + o[2] + o[3]))
#endif
        *reinterpret_cast<f4*>(raw + 4 * rows[c]) = o;
      }
    }
  }
}

// MODE 0: (rays_o, rays_d, viewdirs, t) inputs; MODE 1: encoded x (N, 63), condition (B, 27).
// BF: bf16 numerics (one bf16 MFMA per k-step; the kept activations stored as bf16) -- the
// bf16 training mode; the stream then carries bf16 weights in its hi blocks (k_pack_h bf16).
template <int MODE, int NCOL, bool STORE = false, bool BF = false>
__global__ __launch_bounds__((GeomH<NCOL, BF>::kThreads), (GeomH<NCOL, BF>::kWavesPerSimd)) void k_mlp_fwd_f16x3(
    const f4* __restrict__ wstream, const float* __restrict__ bias_g, const float* __restrict__ in0,
    const float* __restrict__ in1, const float* __restrict__ in2, const float* __restrict__ in3,
    int64_t B, int S, int act, float* __restrict__ raw, TrainStore ts = {}) {
  using G = GeomH<NCOL, BF>;
  // ONE __shared__ object: weight ring | bias table | per-lane stash of the encodings
  constexpr int kPer = stash_per<BF>() * NCOL;  // f4 per lane: enc 2 k-steps + venc 1, hi (& lo)
  constexpr int kStash = AON_STASH_REGS ? 0 : G::kWaves * 64 * kPer;
  static_assert((kLdsWeights + kBiasFloats / 4 + kStash) * 16 <= 160 * 1024, "LDS");
  __shared__ f4 smem[kLdsWeights + kBiasFloats / 4 + kStash];
  float* bias_s = reinterpret_cast<float*>(smem + kLdsWeights);
  f4* stash = smem + kLdsWeights + kBiasFloats / 4 + (threadIdx.x >> 6) * 64 * kPer +
              (threadIdx.x & 63);  // lane-private slots: written and read by the same lane

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, j = lane & 15;
  const int64_t N = B * S;

  WeightPipeP<NetVanillaH, G::kThreads, BF> p;
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
      const float v0 = vd[0], v1 = vd[1], v2 = vd[2];
      auto encode = [&](auto fast) {
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
          for (int e = 0; e < 8; ++e)
          {
            ev[k][e] = pos_enc_feature_fast(x0, x1, x2, 32 * k + 8 * g + e, 0, 10, fast.value);
            __builtin_amdgcn_sched_barrier(0);  // one feature's fp64 temporaries live at a time
          }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          vv[e] = pos_enc_feature_fast(v0, v1, v2, 8 * g + e, 0, 4, fast.value);
          __builtin_amdgcn_sched_barrier(0);
        }
      };
      // every argument of the wave below kSinCrMax (aon_common.hpp): no per-value range branch
      if (pos_enc_fast_ok(x0, x1, x2, 10) && pos_enc_fast_ok(v0, v1, v2, 4))
        encode(std::true_type{});
      else
        encode(std::false_type{});
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
    if (STORE && BF && ts.enc_bf && keep_row(rows[c], N)) store_enc_bf(ts.enc_bf, rows[c], g, ev);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
#pragma unroll
      for (int e = 0; e < 8; ++e) ev[k][e] *= act_scale<BF>();
      split8<BF>(ev[k], enc.hi[k][c], enc.lo[k][c], enc.ovf);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) vv[e] *= act_scale<BF>();
    split8<BF>(vv, venc.hi[0][c], venc.lo[0][c], venc.ovf);
  }

  // park the encodings in LDS until the skip / view layers need them (frees 24 VGPRs for the
  // fragment prefetch); only the owning lane ever touches its slots
#pragma unroll
  for (int c = 0; c < NCOL && !AON_STASH_REGS; ++c) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      stash[64 * enc_slot<BF>(c, k, 0)] = __builtin_bit_cast(f4, enc.hi[k][c]);
      if (!BF) stash[64 * enc_slot<BF>(c, k, 1)] = __builtin_bit_cast(f4, enc.lo[k][c]);
    }
    stash[64 * venc_slot<BF>(c, 0)] = __builtin_bit_cast(f4, venc.hi[0][c]);
    if (!BF) stash[64 * venc_slot<BF>(c, 1)] = __builtin_bit_cast(f4, venc.lo[0][c]);
  }

  Frag<8, NCOL> x, y;
  using WP = WeightPipeP<NetVanillaH, G::kThreads, BF>;
  using T = typename std::conditional<BF, __bf16, float>::type;
  // wave-uniform branch (readfirstlane): the running range masks stay in SGPRs across it
  // (not the training forward: with its row stores the second copy spills)
  if (AON_STAGGER && NCOL == 1 && !STORE && __builtin_amdgcn_readfirstlane(wave) >= G::kWaves / 2) {
    FragPipe<WP, AON_PREFETCH, 4, BF> fp(p);
    vanilla_layers<NCOL, STORE, T>(fp, enc, venc, x, y, stash, bias_s, g, wave, rows, N, act, raw, ts);
  } else {
    FragPipe<WP, AON_PREFETCH, 0, BF> fp(p);
    vanilla_layers<NCOL, STORE, T>(fp, enc, venc, x, y, stash, bias_s, g, wave, rows, N, act, raw, ts);
  }
  range_report(bias_g + kBiasFloats, ovf_of(x) | ovf_of(y) | enc.ovf | venc.ovf);
}

// ---- packing: torch [out][ldw] fp32 -> hi/lo fp16 blocks (+ biases at activation scale), for
// any NetH layer table (passed by value with each layer's weight row stride)
__global__ void k_pack_h(PackArgsH a, float* __restrict__ out_f) {
  const int64_t nhalf = (int64_t)a.stream_blocks * 512;  // fp16 elements of the stream
  _Float16* out = reinterpret_cast<_Float16*>(out_f);
  float* bias_out = out_f + (int64_t)a.stream_blocks * 256;
  const int64_t total = nhalf + a.bias_floats;
  const LayerDesc& last = a.layers[a.n_layers - 1];
  const int used_blocks = last.blk0 + (last.ka + last.kb) * last.u * 2;
  const StreamMap map{a.bf16, a.mx_lo, a.mx_hi};
  // an all-bf16 stream never reports (no weight is range-tested): the status words are cleared
  // here instead of by a memset launch ahead of the pack (pack_h)
  if (a.bf16 == 1 && !a.f16w && blockIdx.x == 0 && threadIdx.x < kStatusBytes / 4)
    reinterpret_cast<uint32_t*>(bias_out + a.bias_floats)[threadIdx.x] = 0u;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    if (e < nhalf) {
      // element e of stream block m is element e of fp16x3 block map.unmap(m) (StreamMap):
      // past the used blocks (the compact modes' tail of the stream region) it maps past the
      // weights and is zero
      const int blk = map.unmap(static_cast<int>(e >> 9));
      const bool bf = !map.f16(blk);  // a bf16 (hi-only) block
      const int l = static_cast<int>((e >> 3) & 63), jj = static_cast<int>(e & 7);
      float w = 0.f;
      bool lo_part = false;
      if (blk < used_blocks) {
        int li = 0;
        while (li + 1 < a.n_layers && a.layers[li + 1].blk0 <= blk) ++li;
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
        const float* src = a.w[li];
        int64_t ld = a.ldw[li];
        if (k < d.ka) {  // previous-layer output fragment order
          const int f = 32 * k + 16 * (jj >> 2) + 4 * gg + (jj & 3);
          col = f < d.len_a ? f : -1;
        } else {  // in-register encodings: natural order
          const int f = 32 * (k - d.ka) + 8 * gg + jj;
          col = f < d.len_b ? (a.w2[li] ? f : d.len_a + f) : -1;
          if (a.w2[li]) {
            src = a.w2[li];
            ld = a.ldw2[li];
          }
        }
        if (o < d.out_real && col >= 0)
          w = a.tr[li] ? src[(int64_t)col * ld + o] : src[(int64_t)o * ld + col];
      }
#if AON_F16X3_V2
      if (bf && !a.f16w) {  // bf16 layer: bf16(w), unscaled, in the compact (hi-only) stream
        out[e] = bf_bits(w);
        continue;
      }
      w *= kWS;  // exact (power of two)
      const _Float16 h = static_cast<_Float16>(w);
      out[e] = lo_part ? static_cast<_Float16>(w - static_cast<float>(h)) : h;
      // range guard (mlp_f16x3_core.hpp): a weight whose scaled hi part is not a finite fp16
      // makes every kernel reading this stream invalid -- status 2 (the word was cleared by
      // pack_h before this launch; many lanes may store the same value)
      if (!lo_part && !(fabsf(w) <= kF16Max))
        *reinterpret_cast<uint32_t*>(bias_out + a.bias_floats) = 2u;
#else
      const _Float16 h = static_cast<_Float16>(w);
      out[e] = lo_part ? static_cast<_Float16>((w - static_cast<float>(h)) * kLoScale) : h;
#endif
    } else {
      const int i = static_cast<int>(e - nhalf);
      int li = 0;
      while (li + 1 < a.n_layers && a.layers[li + 1].bias0 <= i) ++li;
      const int o = i - a.layers[li].bias0;
#if AON_F16X3_V2
      // hidden layers add the bias at activation scale; the 1-tile heads at true scale
      // (bf16 layers: at true scale, their activations are unscaled)
      const StreamMap map{a.bf16, a.mx_lo, a.mx_hi};
      const float bs =
          a.layers[li].u == 1 || !(map.f16(a.layers[li].blk0) || a.f16w) ? 1.0f : kActS;
#else
      const float bs = kActScale;
#endif
      bias_out[i] = (o < a.layers[li].out_real && a.b[li]) ? a.b[li][o] * bs : 0.f;
    }
  }
}

int pack_h(PackArgsH a, void* packed, hipStream_t stream) {
  const int64_t total = (int64_t)a.stream_blocks * 512 + a.bias_floats;
  // the range-status word behind the bias table: cleared (stream-ordered) before the pack, which
  // sets it for an unrepresentable weight; the kernels reading the stream set it on overflow
  // (an all-bf16 stream: k_pack_h clears it itself, one launch fewer)
  if (a.bf16 != 1 || a.f16w) {
    const hipError_t e = hipMemsetAsync(
        static_cast<char*>(packed) + (size_t)a.stream_blocks * 1024 + (size_t)a.bias_floats * 4, 0,
        kStatusBytes, stream);
    if (e != hipSuccess) return static_cast<int>(e);
  }
  hipLaunchKernelGGL(k_pack_h, grid_for(total, 256, 4096), 256, 0, stream, a,
                     static_cast<float*>(packed));
  return launch_status("aon_mlp_pack");
}

int pack_f16x3(const PackArgs& a, void* packed, hipStream_t stream, bool bf16) {
  PackArgsH h{};
  h.bf16 = bf16 ? 1 : 0;
  for (int i = 0; i < kNumLayers; ++i) {
    h.w[i] = a.w[i];
    h.b[i] = a.b[i];
    h.layers[i] = kLayersH[i];
    h.ldw[i] = kLayersH[i].len_a + kLayersH[i].len_b;
  }
  h.n_layers = kNumLayers;
  h.stream_blocks = NetVanillaH::kStreamBlocks;
  h.bias_floats = NetVanillaH::kBiasFloats;
  return pack_h(h, packed, stream);
}

int launch_f16x3(int mode, int ncol, const void* packed, const float* a0, const float* a1,
                 const float* a2, const float* a3, int64_t B, int S, int act, float* raw,
                 hipStream_t stream, const TrainStore* ts) {
  const int64_t N = B * S;
  const f4* ws = static_cast<const f4*>(packed);
  const float* bias = reinterpret_cast<const float*>(static_cast<const char*>(packed) + kStreamBytesF32);
#define AON_LAUNCH_H(M, C)                                                                       \
  hipLaunchKernelGGL((k_mlp_fwd_f16x3<M, C>),                                                    \
                     static_cast<int>((N + GeomH<C>::kRowsPerBlock - 1) / GeomH<C>::kRowsPerBlock), \
                     GeomH<C>::kThreads, 0, stream, ws, bias, a0, a1, a2, a3, B, S, act, raw)
  if (mode == 2 || mode == 3) {  // training forward: MODE 0 inputs + activation stores
    const int grid = static_cast<int>((N + GeomH<1>::kRowsPerBlock - 1) / GeomH<1>::kRowsPerBlock);
    if (mode == 3) {  // bf16 training mode: 16 kBfNcolFwd samples per wave
      using GB = GeomH<kBfNcolFwd, true>;
      hipLaunchKernelGGL((k_mlp_fwd_f16x3<0, kBfNcolFwd, true, true>),
                         static_cast<int>((N + GB::kRowsPerBlock - 1) / GB::kRowsPerBlock),
                         GB::kThreads, 0, stream, ws, bias, a0, a1, a2, a3, B, S, act, raw, *ts);
    } else
      hipLaunchKernelGGL((k_mlp_fwd_f16x3<0, 1, true>), grid, GeomH<1>::kThreads, 0, stream, ws,
                         bias, a0, a1, a2, a3, B, S, act, raw, *ts);
    return launch_status("aon_mlp_fwd_train");
  }
  if (mode == 0 && ncol == 1) AON_LAUNCH_H(0, 1);
  else if (mode == 0) AON_LAUNCH_H(0, 2);
  else if (ncol == 1) AON_LAUNCH_H(1, 1);
  else AON_LAUNCH_H(1, 2);
#undef AON_LAUNCH_H
  return launch_status("aon_mlp_fwd");
}

}  // namespace mlp
}  // namespace aon
