// Fused forward of the articulated NeRFMLP (reference models/vanilla_nerf/model_autodecoder.py:
// 168-239, default geometry: deformation_mlp, enc_after) on the fp16x3 MFMA path of
// mlp_f16x3.hip, one kernel per level:
//
//   xyz = o + t d                                     (helper.py:25-26; or given points)
//   h = relu(D3 relu(D2 relu(D1 relu(D0 [xyz | shape, art]))))          :196-203
//   x' = deformation_layer(h) + xyz;  enc = pos_enc(x', 0, 10)          :205-212
//   trunk on [enc | shape] with the skip concat, density, bottleneck    :214-225
//   view branch relu(V3 ... relu(V0 [bottleneck | enc_dir | appearance])), rgb head  :226-237
//   optional padded sigmoid / softplus(raw - 1) (model_autodecoder.py:321-323)
//
// The latent columns are folded into per-call biases by the host (NeRFMLP.folded_biases), so
// the stream (mlp_layout.hpp kLayersArt) holds only per-sample columns.  The deformation head's
// output lands in lane group 0 (rows 0..2 of its tile, column = sample); it is broadcast to the
// sample's other three lane groups with ds_bpermute, added to xyz in fp32 and encoded in
// registers, so nothing leaves the chip between the deformation and the raw outputs.
#include "mlp_f16x3_core.hpp"
#include <type_traits>
#include "param_check.hpp"

namespace aon {
namespace mlp {

// MODE 0: (rays_o, rays_d, viewdirs, t) inputs; MODE 1: points (N, 3), condition (B, 27).
// STORE: the training forward -- every layer's activations, the encodings of x' and the
// sample points are kept for the backward (TrainStoreArt), raw_sigma gets the noise.
// PREC (the training forward's numerics): 0 fp16x3, kept activations fp32; the bf16 training
// mode keeps hd / h / bot / hv as bf16 (TrainStoreArt's pointers then address bf16 arrays;
// pos_enc(x') and the points stay fp32) and computes 1: fp16x3 throughout, 2: mixed (the
// kArtMix stream, mlp_layout.hpp) -- the deformation MLP fp16x3 (x' = delta + xyz feeds
// sin(2^9 x')), the trunk, heads and view branch one bf16 MFMA per product, or 3: the view
// branch mixed (kArtMixV) -- everything through the bottleneck fp16x3, views_linear.0-3 and the
// rgb head bf16 (the bottleneck's epilogue hands them bf16 fragments, layer_h OBF), or 4: the
// kArtMix stream with fp16 weights in its compact blocks (aon_mlp_art_pack_mixed 3) -- the
// deformation MLP fp16x3, every later layer two fp16 MFMAs per product, hi(W) x (hi(x) + lo(x)),
// with the fp16x3 activations and epilogue (FragPipe W1), or 5: the fp16x3 stream
// (aon_mlp_art_pack) with every layer past the deformation MLP two fp16 MFMAs per product the
// other way round, (hi(W) + lo(W)) x hi(x): the weights exact to 22 bits, the activations
// rounded once to fp16 per sample (FragPipe X1F).
template <int MODE, int NCOL, bool STORE = false, int PREC = 0>
__global__ __launch_bounds__(GeomH<NCOL>::kThreads, NCOL == 1 ? 2 : 1) void k_mlp_art_f16x3(
    const f4* __restrict__ wstream, const float* __restrict__ bias_g, const float* __restrict__ in0,
    const float* __restrict__ in1, const float* __restrict__ in2, const float* __restrict__ in3,
    int64_t B, int S, int act, float* __restrict__ raw, TrainStoreArt ts = {}) {
  using G = GeomH<NCOL>;
  using Net = NetArtH;
  constexpr bool BFM = PREC == 2;
  constexpr bool BFV = PREC == 3;  // bf16 view branch (venc and the bottleneck's output in bf16)
  constexpr bool F16W = PREC == 4;  // fp16 weights past the deformation MLP
  constexpr int X1F = PREC == 5 ? kArtMix.hi : -1;  // fp16 activations past it
  constexpr int kStash = G::kWaves * 64 * 6 * NCOL;  // f4: enc 2 k-steps + venc 1, hi & lo
  __shared__ f4 smem[kLdsWeights + Net::kBiasFloats / 4 + kStash];
  float* bias_s = reinterpret_cast<float*>(smem + kLdsWeights);
  f4* stash = smem + kLdsWeights + Net::kBiasFloats / 4 + (threadIdx.x >> 6) * 64 * 6 * NCOL +
              (threadIdx.x & 63);  // lane-private slots

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, j = lane & 15;
  const int64_t N = B * S;

  using WP = typename std::conditional<
      BFM || F16W, DmaPipe<G::kThreads, kRing, kChunkH, kArtMixStream, kArtMixUsed, kRingLead>,
      typename std::conditional<
          BFV, DmaPipe<G::kThreads, kRing, kChunkH, kArtMixVStream, kArtMixVUsed, kRingLead>,
          WeightPipe<Net, G::kThreads>>::type>::type;
  using T = typename std::conditional<PREC != 0, __bf16, float>::type;
  WP p;
  p.wbuf = smem;
  p.src = wstream;
  p.tid = tid;
  p.lane = lane;
  p.start();
  for (int i = tid; i < Net::kBiasFloats; i += G::kThreads) bias_s[i] = bias_g[i];

  // deformation input (xyz, natural order: lane group 0 elements 0..2) and enc_dir fragments
  Frag<1, NCOL> din, venc;
  int64_t rows[NCOL];
  float px[NCOL][3];
#pragma unroll
  for (int c = 0; c < NCOL; ++c) {
    const int64_t row = (int64_t)blockIdx.x * G::kRowsPerBlock + wave * G::kRowsPerWave + 16 * c + j;
    rows[c] = row;
    const int64_t rr = row < N ? row : N - 1;
    const int64_t ray = rr / S;
    float vv[8];
    if (MODE == 0) {
      const float* ro = in0 + 3 * ray;
      const float* rd = in1 + 3 * ray;
      const float* vd = in2 + 3 * ray;
      const float tt = in3[rr];
#pragma unroll
      for (int q = 0; q < 3; ++q) px[c][q] = __fadd_rn(ro[q], __fmul_rn(tt, rd[q]));
      // (the range test hoisted out of the sines: one wave-uniform branch, aon_common.hpp)
      auto venc_fn = [&](auto fast) {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          vv[e] = pos_enc_feature_fast(vd[0], vd[1], vd[2], 8 * g + e, 0, 4, fast.value);
      };
      if (pos_enc_fast_ok(vd[0], vd[1], vd[2], 4))
        venc_fn(std::true_type{});
      else
        venc_fn(std::false_type{});
    } else {
      const float* x = in0 + rr * 3;
      const float* cd = in1 + ray * 27;
#pragma unroll
      for (int q = 0; q < 3; ++q) px[c][q] = x[q];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int f = 8 * g + e;
        vv[e] = f < 27 ? cd[f] : 0.f;
      }
    }
    if (STORE && g == 0 && row < N) {
#pragma unroll
      for (int q = 0; q < 3; ++q) ts.xyz[3 * row + q] = px[c][q];
    }
    float dv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) dv[e] = (g == 0 && e < 3) ? px[c][e < 3 ? e : 0] * kActS : 0.f;
    split8(dv, din.hi[0][c], din.lo[0][c], din.ovf);
#pragma unroll
    for (int e = 0; e < 8; ++e) vv[e] *= act_scale<BFM || BFV>();
    split8<BFM || BFV>(vv, venc.hi[0][c], venc.lo[0][c], venc.ovf);
    stash[64 * (6 * c + 4)] = __builtin_bit_cast(f4, venc.hi[0][c]);
    stash[64 * (6 * c + 5)] = __builtin_bit_cast(f4, venc.lo[0][c]);
  }

  FragPipe<WP, AON_PREFETCH, 0, false, 0, BFM || F16W ? kArtMix.hi : (BFV ? kArtMixV.hi : 0), F16W,
           X1F>
      fp(p);
  static_assert(kArtMix.lo == 0 && kArtMixV.lo == 0, "mixed streams start fp16x3");
  fp.start();  // begin(0): chunk 0 landed; the barrier also publishes bias_s
  lds_float* bias_l = opaque_lds(bias_s + 4 * g);

  Frag<8, NCOL> x, y;
  Frag<1, NCOL> none;
  using SP = StorePick<STORE, NCOL, T>;
  T* const hd_s = reinterpret_cast<T*>(ts.hd);
  T* const h_s = reinterpret_cast<T*>(ts.h);
  T* const hv_s = reinterpret_cast<T*>(ts.hv);
  const int64_t hds = act_rows(N) * 128, hs = act_rows(N) * 256;  // one deformation / pts_linears output
  const int64_t ms = act_rows(N) * 4;  // one layer's ReLU' bits: hd0..3, h0..7, hv0..3 in ts.masks
  // deformation MLP (model_autodecoder.py:196-205)
  layer_h<Net, A_D0, true>(fp, none, din, x, bias_l, g, SP::make(hd_s, 128, rows, N, g, ts.masks));
  layer_h<Net, A_D1, true>(fp, x, none, y, bias_l, g, SP::make(hd_s + hds, 128, rows, N, g, ts.masks + 1 * ms));
  layer_h<Net, A_D2, true>(fp, y, none, x, bias_l, g, SP::make(hd_s + 2 * hds, 128, rows, N, g, ts.masks + 2 * ms));
  layer_h<Net, A_D3, true>(fp, x, none, y, bias_l, g, SP::make(hd_s + 3 * hds, 128, rows, N, g, ts.masks + 3 * ms));
  f4 dlt[NCOL];
  head_h<Net, A_DOUT>(fp, y, dlt, bias_l, g);

  // x' = deformation + xyz, pos_enc(x') (enc_after, :205-212)
  Frag<2, NCOL> enc;
#pragma unroll
  for (int c = 0; c < NCOL; ++c) {
    float q3[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) q3[q] = __fadd_rn(__shfl(dlt[c][q], j, 64), px[c][q]);
    float fv[2][8], ev[2][8];
    auto enc_fn = [&](auto fast) {
#pragma unroll
      for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float f =
              pos_enc_feature_fast(q3[0], q3[1], q3[2], 32 * k + 8 * g + e, 0, 10, fast.value);
          fv[k][e] = f;
          ev[k][e] = f * act_scale<BFM>();
          __builtin_amdgcn_sched_barrier(0);  // one feature's fp64 temporaries live at a time
        }
    };
    if (pos_enc_fast_ok(q3[0], q3[1], q3[2], 10))
      enc_fn(std::true_type{});
    else
      enc_fn(std::false_type{});
    if (STORE && keep_row(rows[c], N)) {
      store_enc_f32<PREC == 0 ? 64 : 16>(ts.enc, rows[c], g, fv);
      if (PREC != 0) store_enc_bf(ts.enc_bf, rows[c], g, fv);
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      split8<BFM>(ev[k], enc.hi[k][c], enc.lo[k][c], enc.ovf);
      stash[64 * (6 * c + 2 * k)] = __builtin_bit_cast(f4, enc.hi[k][c]);
      stash[64 * (6 * c + 2 * k + 1)] = __builtin_bit_cast(f4, enc.lo[k][c]);
    }
  }

  // trunk on cat[enc, shape] (:214-220), shape folded into the pts_linears.0 / .5 biases
  layer_h<Net, A_P0, true>(fp, none, enc, x, bias_l, g, SP::make(h_s, 256, rows, N, g, ts.masks + 4 * ms));
  layer_h<Net, A_P1, true>(fp, x, none, y, bias_l, g, SP::make(h_s + hs, 256, rows, N, g, ts.masks + 5 * ms));
  layer_h<Net, A_P2, true>(fp, y, none, x, bias_l, g, SP::make(h_s + 2 * hs, 256, rows, N, g, ts.masks + 6 * ms));
  layer_h<Net, A_P3, true>(fp, x, none, y, bias_l, g, SP::make(h_s + 3 * hs, 256, rows, N, g, ts.masks + 7 * ms));
  layer_h<Net, A_P4, true>(fp, y, none, x, bias_l, g, SP::make(h_s + 4 * hs, 256, rows, N, g, ts.masks + 8 * ms));
#pragma unroll
  for (int c = 0; c < NCOL; ++c)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      enc.hi[k][c] = __builtin_bit_cast(h8, stash[64 * (6 * c + 2 * k)]);
      enc.lo[k][c] = __builtin_bit_cast(h8, stash[64 * (6 * c + 2 * k + 1)]);
    }
  // skip: cat[h, enc, shape]
  layer_h<Net, A_P5, true>(fp, x, enc, y, bias_l, g, SP::make(h_s + 5 * hs, 256, rows, N, g, ts.masks + 9 * ms));
  layer_h<Net, A_P6, true>(fp, y, none, x, bias_l, g, SP::make(h_s + 6 * hs, 256, rows, N, g, ts.masks + 10 * ms));
  layer_h<Net, A_P7, true>(fp, x, none, y, bias_l, g, SP::make(h_s + 7 * hs, 256, rows, N, g, ts.masks + 11 * ms));
  f4 dens[NCOL], rgb[NCOL];
  head_h<Net, A_DEN>(fp, y, dens, bias_l, g);  // :221-223
  // bottleneck, no activation (:225)
  layer_h<Net, A_BOT, false, BFV>(fp, y, none, x, bias_l, g, SP::make(reinterpret_cast<T*>(ts.bot), 256, rows, N, g));
#pragma unroll
  for (int c = 0; c < NCOL; ++c) {
    venc.hi[0][c] = __builtin_bit_cast(h8, stash[64 * (6 * c + 4)]);
    venc.lo[0][c] = __builtin_bit_cast(h8, stash[64 * (6 * c + 5)]);
  }
  // view branch on cat[bottleneck, enc_dir, appearance] (:226-235)
  layer_h<Net, A_V0, true>(fp, x, venc, y, bias_l, g, SP::make(hv_s, 128, rows, N, g, ts.masks + 12 * ms));
  layer_h<Net, A_V1, true>(fp, y, none, x, bias_l, g, SP::make(hv_s + hds, 128, rows, N, g, ts.masks + 13 * ms));
  layer_h<Net, A_V2, true>(fp, x, none, y, bias_l, g, SP::make(hv_s + 2 * hds, 128, rows, N, g, ts.masks + 14 * ms));
  layer_h<Net, A_V3, true>(fp, y, none, x, bias_l, g, SP::make(hv_s + 3 * hds, 128, rows, N, g, ts.masks + 15 * ms));
  head_h<Net, A_RGB>(fp, x, rgb, bias_l, g);  // :237

  if (g == 0) {
#pragma unroll
    for (int c = 0; c < NCOL; ++c) {
      if (rows[c] < N) {
        float sig = dens[c][0];
        if (STORE && ts.noise) sig = __fadd_rn(sig, ts.noise[rows[c]]);  // :318-319
        const f4 o = {act_rgb(rgb[c][0], act), act_rgb(rgb[c][1], act), act_rgb(rgb[c][2], act),
                      act_sigma(sig, act)};
        *reinterpret_cast<f4*>(raw + 4 * rows[c]) = o;
      }
    }
  }
  range_report(bias_g + Net::kBiasFloats, ovf_of(x) | ovf_of(y) | enc.ovf | venc.ovf | din.ovf);
}

}  // namespace mlp
}  // namespace aon

using namespace aon;
using namespace aon::mlp;

extern "C" size_t aon_mlp_art_packed_bytes(void) { return NetArtH::kPackedBytes; }

static int art_pack(const aon_mlp_art_params* prm, void* packed, aon_stream_t stream, int mixed) {
  AON_REQUIRE(prm && packed, "null pointer");
  AON_REQUIRE(aligned16(packed), "packed buffer must be 16-byte aligned");
  if (check_mlp_art_params(prm, mixed == 1 ? "aon_mlp_art_pack_bf16"
                                : mixed ? "aon_mlp_art_pack_mixed" : "aon_mlp_art_pack"))
    return -1;
  PackArgsH a{};
  for (int i = 0; i < 4; ++i) {
    a.w[A_D0 + i] = prm->def_w[i];
    a.b[A_D0 + i] = prm->def_b[i];
    a.w[A_V0 + i] = prm->views_w[i];
    a.b[A_V0 + i] = prm->views_b[i];
  }
  for (int i = 0; i < 8; ++i) {
    a.w[A_P0 + i] = prm->pts_w[i];
    a.b[A_P0 + i] = prm->pts_b[i];
  }
  a.w[A_DOUT] = prm->deformation_w; a.b[A_DOUT] = prm->deformation_b;
  a.w[A_DEN] = prm->density_w;      a.b[A_DEN] = prm->density_b;
  a.w[A_BOT] = prm->bottleneck_w;   a.b[A_BOT] = prm->bottleneck_b;
  a.w[A_RGB] = prm->rgb_w;          a.b[A_RGB] = prm->rgb_b;
  for (int i = 0; i < kNumLayersArt; ++i) {
    AON_REQUIRE(a.w[i] && a.b[i], "null layer parameter");
    a.layers[i] = kLayersArt[i];
    a.ldw[i] = kLayersArt[i].len_a + kLayersArt[i].len_b;
  }
  // weights whose rows carry folded latent columns after the per-sample ones
  a.ldw[A_D0] = (int)prm->w_cols[kArtDef0];
  a.ldw[A_P0] = (int)prm->w_cols[kArtPts0];
  a.ldw[A_P5] = (int)prm->w_cols[kArtPts5];
  a.ldw[A_V0] = (int)prm->w_cols[kArtView0];
  a.n_layers = kNumLayersArt;
  a.stream_blocks = NetArtH::kStreamBlocks;
  a.bias_floats = NetArtH::kBiasFloats;
  if (mixed) {
    const StreamMap m = mixed == 2 ? kArtMixV : kArtMix;
    a.bf16 = m.mode;
    a.mx_lo = m.lo;
    a.mx_hi = m.hi;
    a.f16w = mixed == 3;
  }
  return pack_h(a, packed, (hipStream_t)stream);
}

extern "C" int aon_mlp_art_pack(const aon_mlp_art_params* prm, void* packed, aon_stream_t stream) {
  return art_pack(prm, packed, stream, 0);
}

// the articulated bf16 mode's mixed streams (same buffer size and bias table): mixed = 1 the
// trunk-bf16 stream (= aon_mlp_art_pack_bf16), 2 the view-branch stream (kArtMixV), 3 the
// kArtMix map with fp16 weights in the compact blocks
extern "C" int aon_mlp_art_pack_mixed(const aon_mlp_art_params* prm, int mixed, void* packed,
                                      aon_stream_t stream) {
  AON_REQUIRE(mixed >= 1 && mixed <= 3,
              "mixed: 1 trunk bf16, 2 view branch bf16, 3 fp16 weights past the deformation MLP");
  return art_pack(prm, packed, stream, mixed);
}

// the bf16 training mode's mixed stream (kArtMix): same buffer size and bias table
extern "C" int aon_mlp_art_pack_bf16(const aon_mlp_art_params* prm, void* packed,
                                     aon_stream_t stream) {
  return art_pack(prm, packed, stream, 1);
}

static int art_launch(int mode, const void* packed, const float* a0, const float* a1,
                      const float* a2, const float* a3, int64_t B, int S, int act, float* raw,
                      aon_stream_t stream) {
  AON_REQUIRE(packed && raw && a0 && a1, "null pointer");
  AON_REQUIRE(B >= 0 && S >= 1, "bad shape");
  AON_REQUIRE(act >= AON_ACT_NONE && act <= AON_ACT_ARTIC, "bad activation");
  AON_REQUIRE(aligned16(packed) && aligned16(raw), "packed / raw must be 16-byte aligned");
  const int64_t N = B * S;
  if (N == 0) return 0;
  using G = GeomH<1>;
  const int64_t grid = (N + G::kRowsPerBlock - 1) / G::kRowsPerBlock;
  AON_REQUIRE(grid < (1ll << 31), "too many rows");
  const f4* ws = static_cast<const f4*>(packed);
  const float* bias =
      reinterpret_cast<const float*>(static_cast<const char*>(packed) + NetArtH::kStreamBytes);
#if AON_DATAFLOW_WS_BUILD
  if (mode == 0)
    return launch_art_ws_f16x3(packed, a0, a1, a2, a3, B, S, act, raw, (hipStream_t)stream);
#endif
  if (mode == 0)
    hipLaunchKernelGGL((k_mlp_art_f16x3<0, 1>), (unsigned)grid, G::kThreads, 0,
                       (hipStream_t)stream, ws, bias, a0, a1, a2, a3, B, S, act, raw);
  else
    hipLaunchKernelGGL((k_mlp_art_f16x3<1, 1>), (unsigned)grid, G::kThreads, 0,
                       (hipStream_t)stream, ws, bias, a0, a1, a2, a3, B, S, act, raw);
  return launch_status("aon_mlp_art_fwd");
}

extern "C" int aon_mlp_art_fwd(const void* packed, const float* rays_o, const float* rays_d,
                               const float* viewdirs, const float* t, int64_t B, int S, int act,
                               float* out, aon_stream_t stream) {
  AON_REQUIRE(viewdirs && t, "null pointer");
  return art_launch(0, packed, rays_o, rays_d, viewdirs, t, B, S, act, out, stream);
}

#ifndef AON_ART_X1_NCOL
#define AON_ART_X1_NCOL 1  // A/B knob (compile-time): samples per wave / 16 of the mixed-4 forward
#endif
static int art_fwd_train(const void* packed, const float* rays_o, const float* rays_d,
                         const float* viewdirs, const float* t, int64_t B, int S,
                         const float* noise, float* hd, float* h, float* bot, float* hv,
                         float* enc, float* xyz, float* raw, uint32_t* masks, aon_stream_t stream,
                         int prec, __bf16* enc_bf = nullptr) {
  AON_REQUIRE(packed && rays_o && rays_d && viewdirs && t && raw, "null pointer");
  AON_REQUIRE(hd && h && bot && hv && enc && xyz && masks, "null activation buffer");
  AON_REQUIRE(aligned16(masks) && aligned16(enc), "masks / enc must be 16-byte aligned");
  AON_REQUIRE(!prec || (enc_bf && aligned16(enc_bf)), "enc_bf: a 16-byte aligned buffer");
  AON_REQUIRE(B >= 0 && S >= 1, "bad shape");
  AON_REQUIRE(aligned16(packed) && aligned16(raw), "packed / raw must be 16-byte aligned");
  AON_REQUIRE(((reinterpret_cast<uintptr_t>(hd) | reinterpret_cast<uintptr_t>(h) |
                reinterpret_cast<uintptr_t>(bot) | reinterpret_cast<uintptr_t>(hv)) & 7) == 0,
              "activation buffers must be 8-byte aligned");
  const int64_t N = B * S;
  if (N == 0) return 0;
  using G = GeomH<1>;
  const int64_t grid = (N + G::kRowsPerBlock - 1) / G::kRowsPerBlock;
  AON_REQUIRE(grid < (1ll << 31), "too many rows");
  const f4* ws = static_cast<const f4*>(packed);
  const float* bias =
      reinterpret_cast<const float*>(static_cast<const char*>(packed) + NetArtH::kStreamBytes);
  const TrainStoreArt ts{hd, h, bot, hv, enc, xyz, noise, reinterpret_cast<uint2*>(masks), enc_bf};
  if (prec == 5) {
    using G5 = GeomH<AON_ART_X1_NCOL>;
    hipLaunchKernelGGL((k_mlp_art_f16x3<0, AON_ART_X1_NCOL, true, 5>),
                       (unsigned)((N + G5::kRowsPerBlock - 1) / G5::kRowsPerBlock), G5::kThreads, 0,
                       (hipStream_t)stream, ws, bias, rays_o, rays_d, viewdirs, t, B, S,
                       (int)AON_ACT_NONE, raw, ts);
  } else if (prec == 4)
    hipLaunchKernelGGL((k_mlp_art_f16x3<0, 1, true, 4>), (unsigned)grid, G::kThreads, 0,
                       (hipStream_t)stream, ws, bias, rays_o, rays_d, viewdirs, t, B, S,
                       (int)AON_ACT_NONE, raw, ts);
  else if (prec == 3)
    hipLaunchKernelGGL((k_mlp_art_f16x3<0, 1, true, 3>), (unsigned)grid, G::kThreads, 0,
                       (hipStream_t)stream, ws, bias, rays_o, rays_d, viewdirs, t, B, S,
                       (int)AON_ACT_NONE, raw, ts);
  else if (prec == 2)
    hipLaunchKernelGGL((k_mlp_art_f16x3<0, 1, true, 2>), (unsigned)grid, G::kThreads, 0,
                       (hipStream_t)stream, ws, bias, rays_o, rays_d, viewdirs, t, B, S,
                       (int)AON_ACT_NONE, raw, ts);
  else if (prec == 1)
    hipLaunchKernelGGL((k_mlp_art_f16x3<0, 1, true, 1>), (unsigned)grid, G::kThreads, 0,
                       (hipStream_t)stream, ws, bias, rays_o, rays_d, viewdirs, t, B, S,
                       (int)AON_ACT_NONE, raw, ts);
  else
    hipLaunchKernelGGL((k_mlp_art_f16x3<0, 1, true>), (unsigned)grid, G::kThreads, 0,
                       (hipStream_t)stream, ws, bias, rays_o, rays_d, viewdirs, t, B, S,
                       (int)AON_ACT_NONE, raw, ts);
  return launch_status(prec ? "aon_mlp_art_fwd_train_bf16" : "aon_mlp_art_fwd_train");
}

extern "C" int aon_mlp_art_fwd_train(const void* packed, const float* rays_o, const float* rays_d,
                                     const float* viewdirs, const float* t, int64_t B, int S,
                                     const float* noise, float* hd, float* h, float* bot,
                                     float* hv, float* enc, float* xyz, float* raw,
                                     uint32_t* masks, aon_stream_t stream) {
  return art_fwd_train(packed, rays_o, rays_d, viewdirs, t, B, S, noise, hd, h, bot, hv, enc, xyz,
                       raw, masks, stream, 0);
}

extern "C" int aon_mlp_art_fwd_train_bf16(const void* packed, const float* rays_o,
                                          const float* rays_d, const float* viewdirs,
                                          const float* t, int64_t B, int S, const float* noise,
                                          void* hd, void* h, void* bot, void* hv, float* enc,
                                          float* xyz, float* raw, uint32_t* masks, void* enc_bf,
                                          int mixed, aon_stream_t stream) {
  AON_REQUIRE(mixed >= 0 && mixed <= 4,
              "mixed: 0 fp16x3, 1 trunk bf16, 2 view branch bf16, 3 fp16 weights, 4 fp16 activations");
  return art_fwd_train(packed, rays_o, rays_d, viewdirs, t, B, S, noise, static_cast<float*>(hd),
                       static_cast<float*>(h), static_cast<float*>(bot), static_cast<float*>(hv),
                       enc, xyz, raw, masks, stream, mixed + 1, static_cast<__bf16*>(enc_bf));
}

extern "C" int aon_mlp_art_fwd_points(const void* packed, const float* pos,
                                      const float* condition, int64_t B, int S, int act,
                                      float* out, aon_stream_t stream) {
  return art_launch(1, packed, pos, condition, nullptr, nullptr, B, S, act, out, stream);
}
