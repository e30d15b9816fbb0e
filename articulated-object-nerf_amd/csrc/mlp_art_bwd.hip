// Fused backward chain of the articulated NeRFMLP for the training step (reference
// models/vanilla_nerf/model_autodecoder.py:168-239 under autograd, LitNeRF_AutoDecoder.training_step
// :395-477): from dL/d raw (the compositor's backward) through the view branch, the heads and
// the trunk to dL/d pos_enc(x'), through pos_enc's backward (helper.py:136-140) to dL/dx', then
// through the deformation head and the deformation MLP -- every input-gradient product
// dX = dZ W in ONE kernel, each masked by ReLU' of the forward output it flows into, every dZ
// stored for the weight-gradient GEMMs (dW = dZ^T X, train_art.py).
//
// Structure and numerics as mlp_bwd.hip (the vanilla chain): feature-major MFMA tiles, W^T
// streamed through the LDS-DMA ring (kLayersArtBwd, packed from the forward weights with tr = 1),
// each finished output pair converted in registers into the next layer's B fragments, gradients
// at a per-call power-of-two scale s from max |d raw|.  The enc columns of the skip layer give
// 64 values per sample, parked lane-private in LDS; those of pts_linears.0 join them in the
// epilogue, where pos_enc's backward runs on the fly -- sin' = cos at the forward's fp32
// arguments (x' 2^d and x' 2^d + pi/2f), summed over degrees -- and the four lane groups of a
// sample are reduced with two shuffles.  dL/dx' then re-enters fp16 at a per-sample power-of-two
// scale (it carries the 2^9 factors of pos_enc's top degree).
// the round-2 per-pair range test (AON_GUARD_PK 0): with the deferred packed test this
// 256-VGPR kernel spills
#ifndef AON_GUARD_PK
#define AON_GUARD_PK 0
#endif
#include "mlp_f16x3_core.hpp"
#include "param_check.hpp"

namespace aon {
namespace mlp {

struct ArtBwdArgs {
  const float* draw;       // (N, 4): d raw_rgb (3), d raw_sigma
  const uint2* masks;      // (16, N, 4) ReLU' bits of hd0..3, h0..7, hv0..3
  const float* enc;        // the forward's tiled fp32 pos_enc(x') (store_enc_f32): x' = columns 0..2
  float* dzv;              // (4, N, 128): dL/d pre-activation of views_linear.i
  float* dbot;             // (N, 256): dL/d bottleneck output
  float* dz;               // (8, N, 256): dL/d pre-activation of pts_linears.i
  float* dxp;              // (N, 3): dL/dx' = dL/d deformation_layer output
  float* dzd;              // (4, N, 128): dL/d pre-activation of deformations_linear.i
  const uint32_t* absmax;  // bits of max |draw|
  int64_t N;
};

// Epilogue policy of the skip layer's enc columns: park each value (scale s) in this lane's LDS
// slots [tile][reg]; nothing goes to the output fragments' consumer.
struct EncStash {
  static constexpr bool kPkEpi = false;  // sees the fp32 values (post)
  float* slot;  // lane-private: float index (t * 64) * 4 + r of the lane's f4 slot t
  __device__ __forceinline__ void begin_pair(int) const {}
  __device__ __forceinline__ float post(int pr, int uu, int r, int, float v) const {
    slot[(2 * pr + uu) * 256 + r] = v;
    return v;
  }
  __device__ __forceinline__ void put(int, int, int, int, float, float) const {}
  __device__ __forceinline__ void put_pk(int, int, int, int, uint32_t) const {}
};

// Epilogue policy of pts_linears.0's enc columns: total d enc_f = this value + the parked skip
// value, then pos_enc's backward accumulated per x' component (feature f = 16 t + 4 g + r):
// f < 3 identity; 3 <= f < 33 sin(x_c 2^d); 33 <= f < 63 sin(x_c 2^d + pi/2f), (f - 3) mod 30 =
// 3 d + c.
struct EncBwd {
  static constexpr bool kPkEpi = false;
  const float* slot;
  float x0, x1, x2;  // x' of this lane's sample
  int g;
  mutable float dx0 = 0.f, dx1 = 0.f, dx2 = 0.f;
  __device__ __forceinline__ void begin_pair(int) const {}
  __device__ __forceinline__ float post(int pr, int uu, int r, int, float v) const {
    const int t = 2 * pr + uu;
    const float tot = __fadd_rn(slot[t * 256 + r], v);
    const int f = 16 * t + 4 * g + r;
    float a = 0.f;
    int comp;
    if (f < 3) {
      a = tot;
      comp = f;
    } else if (f < 63) {
      const bool cosine = f >= 33;
      const int q = cosine ? f - 33 : f - 3;
      const int d = q / 3;
      comp = q - 3 * d;
      const float sc = __builtin_ldexpf(1.0f, d);
      const float xc = comp == 0 ? x0 : (comp == 1 ? x1 : x2);
      const float xb = __fmul_rn(xc, sc);  // exact
      a = __fmul_rn(__fmul_rn(tot, cos_cr(cosine ? __fadd_rn(xb, kHalfPi) : xb)), sc);
    } else {
      comp = 3;  // padding row
    }
    dx0 = comp == 0 ? __fadd_rn(dx0, a) : dx0;
    dx1 = comp == 1 ? __fadd_rn(dx1, a) : dx1;
    dx2 = comp == 2 ? __fadd_rn(dx2, a) : dx2;
    return v;
  }
  __device__ __forceinline__ void put(int, int, int, int, float, float) const {}
  __device__ __forceinline__ void put_pk(int, int, int, int, uint32_t) const {}
};

// The bf16 chain at 32 samples per wave (NCOL = 2): the same two policies with the skip layer's
// enc-column values parked in registers (16 floats per sample column) instead of LDS -- the
// LDS-DMA ring and the bias table leave no room for twice the lane-private slots.  Same values,
// same arithmetic per sample (bit-identical to NCOL = 1).
template <int NCOL>
struct EncStashReg {
  static constexpr bool kPkEpi = false;
  mutable float v[NCOL][4][4];  // [column][tile t = 2 pr + uu][reg r]
  __device__ __forceinline__ void begin_pair(int) const {}
  __device__ __forceinline__ float post(int pr, int uu, int r, int c, float x) const {
    v[c][2 * pr + uu][r] = x;
    return x;
  }
  __device__ __forceinline__ void put(int, int, int, int, float, float) const {}
  __device__ __forceinline__ void put_pk(int, int, int, int, uint32_t) const {}
};
template <int NCOL>
struct EncBwdReg {
  static constexpr bool kPkEpi = false;
  const EncStashReg<NCOL>* park;
  float x[NCOL][3];  // x' of each column's sample
  int g;
  mutable float dx[NCOL][3];
  __device__ __forceinline__ void begin_pair(int) const {}
  __device__ __forceinline__ float post(int pr, int uu, int r, int c, float v) const {
    const int t = 2 * pr + uu;
    const float tot = __fadd_rn(park->v[c][t][r], v);
    const int f = 16 * t + 4 * g + r;
    float a = 0.f;
    int comp;
    if (f < 3) {
      a = tot;
      comp = f;
    } else if (f < 63) {
      const bool cosine = f >= 33;
      const int q = cosine ? f - 33 : f - 3;
      const int d = q / 3;
      comp = q - 3 * d;
      const float sc = __builtin_ldexpf(1.0f, d);
      const float xc = comp == 0 ? x[c][0] : (comp == 1 ? x[c][1] : x[c][2]);
      const float xb = __fmul_rn(xc, sc);  // exact
      a = __fmul_rn(__fmul_rn(tot, cos_cr(cosine ? __fadd_rn(xb, kHalfPi) : xb)), sc);
    } else {
      comp = 3;  // padding row
    }
    dx[c][0] = comp == 0 ? __fadd_rn(dx[c][0], a) : dx[c][0];
    dx[c][1] = comp == 1 ? __fadd_rn(dx[c][1], a) : dx[c][1];
    dx[c][2] = comp == 2 ? __fadd_rn(dx[c][2], a) : dx[c][2];
    return v;
  }
  __device__ __forceinline__ void put(int, int, int, int, float, float) const {}
  __device__ __forceinline__ void put_pk(int, int, int, int, uint32_t) const {}
};

#ifndef AON_BF_NCOL_ART_BWD
#define AON_BF_NCOL_ART_BWD 2  // samples per wave / 16 of the bf16 articulated chain (1: A/B)
#endif
constexpr int kBfNcolArtBwd = AON_BF_NCOL_ART_BWD;
template <bool BF>
using ArtBwdGeom = GeomH<BF ? kBfNcolArtBwd : 1, BF>;

// BF: the bf16 training mode -- the whole chain one bf16 MFMA per product on the compact stream
// (the deformation branch too: only its forward needs fp16x3, for x'), every dZ stored as bf16
// (ArtBwdArgs' dzv / dbot / dz / dzd then address bf16 arrays); dL/dx' stays fp32.
template <bool BF = false>
__global__ __launch_bounds__(ArtBwdGeom<BF>::kThreads, 2) void k_mlp_art_bwd_f16x3(
    const f4* __restrict__ wstream, const float* __restrict__ bias_g, ArtBwdArgs a) {
  constexpr int NCOL = BF ? kBfNcolArtBwd : 1;
  constexpr bool kRegPark = NCOL > 1;  // enc-column values and d sigma kept in registers
  constexpr int kEncW = BF ? 16 : 64;  // the forward's store_enc_f32 width
  using G = ArtBwdGeom<BF>;
  using Net = NetArtBwdH;
  using T = typename std::conditional<BF, __bf16, float>::type;
  T* const dzv = reinterpret_cast<T*>(a.dzv);
  T* const dz = reinterpret_cast<T*>(a.dz);
  T* const dzd = reinterpret_cast<T*>(a.dzd);
  // per lane: d raw_sigma fragment (hi, lo) + 4 f4 of parked skip-enc gradients (NCOL = 1)
  constexpr int kSlots = kRegPark ? 0 : 6;
  __shared__ f4 smem[kLdsWeights + Net::kBiasFloats / 4 + G::kWaves * 64 * kSlots];
  float* bias_s = reinterpret_cast<float*>(smem + kLdsWeights);
  f4* stash = smem + kLdsWeights + Net::kBiasFloats / 4 + (threadIdx.x >> 6) * 64 * kSlots +
              (threadIdx.x & 63);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, j = lane & 15;
  const int64_t N = a.N;

  WeightPipeP<Net, G::kThreads, BF> p;
  p.wbuf = smem;
  p.src = wstream;
  p.tid = tid;
  p.lane = lane;
  p.start();
  for (int i = tid; i < Net::kBiasFloats; i += G::kThreads) bias_s[i] = bias_g[i];

  const float s = BF ? 1.0f : grad_scale(*a.absmax);  // bf16: unscaled (fp32's exponent range)
  const float inv = 1.0f / s;  // exact: a power of two

  Frag<1, NCOL> drgb, dsig;
  int64_t rows[NCOL], rrs[NCOL];
#pragma unroll
  for (int c = 0; c < NCOL; ++c) {
    const int64_t row = (int64_t)blockIdx.x * G::kRowsPerBlock + wave * G::kRowsPerWave + 16 * c + j;
    rows[c] = row;
    const int64_t rr = row < N ? row : N - 1;
    rrs[c] = rr;
    const f4 d = *reinterpret_cast<const f4*>(a.draw + 4 * rr);
    float dv[8], sv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      dv[e] = (g == 0 && e < 3) ? d[e < 3 ? e : 0] * s : 0.f;
      sv[e] = (g == 0 && e == 0) ? d[3] * s : 0.f;
    }
    split8<BF>(dv, drgb.hi[0][c], drgb.lo[0][c], drgb.ovf);
    split8<BF>(sv, dsig.hi[0][c], dsig.lo[0][c], dsig.ovf);
  }
  if (!kRegPark) {
    stash[0] = __builtin_bit_cast(f4, dsig.hi[0][0]);
    stash[64] = __builtin_bit_cast(f4, dsig.lo[0][0]);
  }

  FragPipe<WeightPipeP<Net, G::kThreads, BF>, AON_PREFETCH, 0, BF> fp(p);
  fp.start();
  lds_float* bias_l = opaque_lds(bias_s + 4 * g);

  const int64_t hs = act_rows(N) * 256, ws = act_rows(N) * 128, ms = act_rows(N) * 4;  // ms: one layer's ReLU' bits
  Frag<8, NCOL> x, y;
  Frag<2, NCOL> junk;  // output fragments of the enc-column layers (consumed in the epilogue)
  Frag<1, NCOL> none;
  // view branch: d hv3 = W_rgb^T d rgb, then views_linear.3 .. 1, each * ReLU'
  layer_h<Net, AB_RGB, false>(fp, none, drgb, x, bias_l, g,
                              mask_bits(a.masks + 15 * ms, dzv + 3 * ws, 128, rows, N, g, inv));
  layer_h<Net, AB_V3, false>(fp, x, none, y, bias_l, g,
                             mask_bits(a.masks + 14 * ms, dzv + 2 * ws, 128, rows, N, g, inv));
  layer_h<Net, AB_V2, false>(fp, y, none, x, bias_l, g,
                             mask_bits(a.masks + 13 * ms, dzv + 1 * ws, 128, rows, N, g, inv));
  layer_h<Net, AB_V1, false>(fp, x, none, y, bias_l, g,
                             mask_bits(a.masks + 12 * ms, dzv, 128, rows, N, g, inv));
  // d bottleneck = W_view0[:, :256]^T dZ_view0 (linear layer: no mask)
  {
    RowStore<NCOL, T> st;
#pragma unroll
    for (int c = 0; c < NCOL; ++c) {
      st.ok[c] = keep_row(rows[c], N);
      st.rowp[c] = reinterpret_cast<T*>(a.dbot) + act_base(rows[c], 256, g);
    }
    st.off16 = st16_off(g);
    st.s = inv;
    layer_h<Net, AB_V0, false>(fp, y, none, x, bias_l, g, st);
  }
  if (!kRegPark) {
    dsig.hi[0][0] = __builtin_bit_cast(h8, stash[0]);
    dsig.lo[0][0] = __builtin_bit_cast(h8, stash[64]);
  }
  // d h7 = W_bot^T d bottleneck + W_den^T d sigma, * ReLU'(h7) -> dZ_7
  layer_h<Net, AB_BOTDEN, false>(fp, x, dsig, y, bias_l, g,
                                 mask_bits(a.masks + 11 * ms, dz + 7 * hs, 256, rows, N, g, inv));
  layer_h<Net, AB_P7, false>(fp, y, none, x, bias_l, g,
                             mask_bits(a.masks + 10 * ms, dz + 6 * hs, 256, rows, N, g, inv));
  layer_h<Net, AB_P6, false>(fp, x, none, y, bias_l, g,
                             mask_bits(a.masks + 9 * ms, dz + 5 * hs, 256, rows, N, g, inv));
  // skip layer: its h4 columns continue the chain, its enc columns are parked for the encoding's
  // gradient (y = dZ_5 feeds both)
  layer_h<Net, AB_P5, false>(fp, y, none, x, bias_l, g,
                             mask_bits(a.masks + 8 * ms, dz + 4 * hs, 256, rows, N, g, inv));
  float* slot = reinterpret_cast<float*>(stash + 2 * 64);
  EncStashReg<NCOL> park;
  if constexpr (kRegPark)
    layer_h<Net, AB_P5E, false>(fp, y, none, junk, bias_l, g, park);
  else
    layer_h<Net, AB_P5E, false>(fp, y, none, junk, bias_l, g, EncStash{slot});
  layer_h<Net, AB_P4, false>(fp, x, none, y, bias_l, g,
                             mask_bits(a.masks + 7 * ms, dz + 3 * hs, 256, rows, N, g, inv));
  layer_h<Net, AB_P3, false>(fp, y, none, x, bias_l, g,
                             mask_bits(a.masks + 6 * ms, dz + 2 * hs, 256, rows, N, g, inv));
  layer_h<Net, AB_P2, false>(fp, x, none, y, bias_l, g,
                             mask_bits(a.masks + 5 * ms, dz + 1 * hs, 256, rows, N, g, inv));
  layer_h<Net, AB_P1, false>(fp, y, none, x, bias_l, g,
                             mask_bits(a.masks + 4 * ms, dz, 256, rows, N, g, inv));
  // d enc = W_0[:, :63]^T dZ_0 + the parked skip part, and pos_enc's backward (:205-212)
  float dx[NCOL][3];
  if constexpr (kRegPark) {
    EncBwdReg<NCOL> eb;
    eb.park = &park;
    eb.g = g;
#pragma unroll
    for (int c = 0; c < NCOL; ++c)
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        eb.x[c][q] = a.enc[enc_x_index(rrs[c], kEncW) + q];
        eb.dx[c][q] = 0.f;
      }
    layer_h<Net, AB_P0E, false>(fp, x, none, junk, bias_l, g, eb);
#pragma unroll
    for (int c = 0; c < NCOL; ++c)
#pragma unroll
      for (int q = 0; q < 3; ++q) dx[c][q] = eb.dx[c][q];
  } else {
    EncBwd eb;
    eb.slot = slot;
    eb.x0 = a.enc[enc_x_index(rrs[0], kEncW)];
    eb.x1 = a.enc[enc_x_index(rrs[0], kEncW) + 1];
    eb.x2 = a.enc[enc_x_index(rrs[0], kEncW) + 2];
    eb.g = g;
    layer_h<Net, AB_P0E, false>(fp, x, none, junk, bias_l, g, eb);
    dx[0][0] = eb.dx0;
    dx[0][1] = eb.dx1;
    dx[0][2] = eb.dx2;
  }
  Frag<1, NCOL> ddx;
  float invd[NCOL];
#pragma unroll
  for (int c = 0; c < NCOL; ++c) {
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      dx[c][q] = __fadd_rn(dx[c][q], __shfl_xor(dx[c][q], 16, 64));
      dx[c][q] = __fadd_rn(dx[c][q], __shfl_xor(dx[c][q], 32, 64));
      dx[c][q] *= inv;  // true dL/dx' (identical in the sample's four lane groups)
    }
    if (g == 0 && rows[c] < N) {
#pragma unroll
      for (int q = 0; q < 3; ++q) a.dxp[3 * rows[c] + q] = dx[c][q];
    }
    // dL/dx' carries pos_enc's 2^d factors: back into fp16 at this sample's own scale
    const float sd = BF ? 1.0f : grad_scale(__float_as_uint(fmaxf(fabsf(dx[c][0]), fmaxf(fabsf(dx[c][1]), fabsf(dx[c][2])))));
    invd[c] = 1.0f / sd;
    float dv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) dv[e] = (g == 0 && e < 3) ? dx[c][e < 3 ? e : 0] * sd : 0.f;
    split8<BF>(dv, ddx.hi[0][c], ddx.lo[0][c], ddx.ovf);
  }
  // (the fp16x3 chain's per-sample scale: one column; the bf16 chain runs unscaled, invd = 1)
  const float invd0 = invd[0];
  // deformation head and MLP: d hd3 = W_dl^T dL/dx', then deformations_linear.3 .. 1
  layer_h<Net, AB_DL, false>(fp, none, ddx, y, bias_l, g,
                             mask_bits(a.masks + 3 * ms, dzd + 3 * ws, 128, rows, N, g, invd0));
  layer_h<Net, AB_D3, false>(fp, y, none, x, bias_l, g,
                             mask_bits(a.masks + 2 * ms, dzd + 2 * ws, 128, rows, N, g, invd0));
  layer_h<Net, AB_D2, false>(fp, x, none, y, bias_l, g,
                             mask_bits(a.masks + 1 * ms, dzd + 1 * ws, 128, rows, N, g, invd0));
  // (the last layer's outputs are only stored, the enc-column layers' fragments are consumed in
  // their epilogues: neither fp16 split is used, so neither is range-checked)
  const uint64_t used_ovf = ovf_of(x) | ovf_of(y) | drgb.ovf | dsig.ovf | ddx.ovf;
  layer_h<Net, AB_D1, false>(fp, y, none, x, bias_l, g,
                             mask_bits(a.masks + 0 * ms, dzd, 128, rows, N, g, invd0));
  range_report(bias_g + Net::kBiasFloats, used_ovf);
}

}  // namespace mlp
}  // namespace aon

using namespace aon;
using namespace aon::mlp;

extern "C" size_t aon_mlp_art_bwd_packed_bytes(void) { return NetArtBwdH::kPackedBytes; }

static int art_bwd_pack(const aon_mlp_art_params* prm, void* packed, aon_stream_t stream,
                        bool bf16) {
  AON_REQUIRE(prm && packed, "null pointer");
  AON_REQUIRE(aligned16(packed), "packed buffer must be 16-byte aligned");
  if (check_mlp_art_params(prm, bf16 ? "aon_mlp_art_bwd_pack_bf16" : "aon_mlp_art_bwd_pack"))
    return -1;
  const int ld_view0 = (int)prm->w_cols[kArtView0], ld_pts5 = (int)prm->w_cols[kArtPts5];
  const int ld_pts0 = (int)prm->w_cols[kArtPts0];
  PackArgsH a{};
  const float* w[kNumLayersArtBwd] = {
      prm->rgb_w,     prm->views_w[3], prm->views_w[2], prm->views_w[1], prm->views_w[0],
      prm->bottleneck_w, prm->pts_w[7], prm->pts_w[6], prm->pts_w[5],
      prm->pts_w[5] ? prm->pts_w[5] + 256 : nullptr,  // enc columns of the skip layer
      prm->pts_w[4], prm->pts_w[3], prm->pts_w[2], prm->pts_w[1], prm->pts_w[0],
      prm->deformation_w, prm->def_w[3], prm->def_w[2], prm->def_w[1]};
  // row strides of the forward weights (their in-features, latent columns included)
  const int ld[kNumLayersArtBwd] = {128, 128, 128, 128, ld_view0, 256, 256, 256, ld_pts5,
                                    ld_pts5, 256, 256, 256, 256, ld_pts0, 128, 128, 128, 128};
  for (int i = 0; i < kNumLayersArtBwd; ++i) {
    AON_REQUIRE(w[i], "null layer weight");
    a.w[i] = w[i];
    a.ldw[i] = ld[i];
    a.tr[i] = 1;
    a.layers[i] = kLayersArtBwd[i];
  }
  AON_REQUIRE(prm->density_w, "null layer weight");
  a.w2[AB_BOTDEN] = prm->density_w;  // segment B of d h7: density_layer^T (1 x 256)
  a.ldw2[AB_BOTDEN] = 256;
  a.n_layers = kNumLayersArtBwd;
  a.stream_blocks = NetArtBwdH::kStreamBlocks;
  a.bias_floats = NetArtBwdH::kBiasFloats;
  a.bf16 = bf16 ? 1 : 0;
  return pack_h(a, packed, (hipStream_t)stream);
}

extern "C" int aon_mlp_art_bwd_pack(const aon_mlp_art_params* prm, void* packed,
                                    aon_stream_t stream) {
  return art_bwd_pack(prm, packed, stream, false);
}

extern "C" int aon_mlp_art_bwd_pack_bf16(const aon_mlp_art_params* prm, void* packed,
                                         aon_stream_t stream) {
  return art_bwd_pack(prm, packed, stream, true);
}

static int art_bwd(const void* packed, const float* draw, const uint32_t* masks, const float* enc,
                   int64_t N, float* dzv, float* dbot, float* dz, float* dxp, float* dzd,
                   void* work, aon_stream_t stream, bool bf16) {
  AON_REQUIRE(packed && draw && masks && enc && dzv && dbot && dz && dxp && dzd && work,
              "null pointer");
  AON_REQUIRE(N >= 0, "bad shape");
  AON_REQUIRE(aligned16(packed) && aligned16(draw) && aligned16(masks) && aligned16(enc) && aligned16(dzv) &&
                  aligned16(dbot) && aligned16(dz) && aligned16(dzd),
              "buffers must be 16-byte aligned");
  if (N == 0) return 0;
  const int64_t rpb = bf16 ? ArtBwdGeom<true>::kRowsPerBlock : ArtBwdGeom<false>::kRowsPerBlock;
  const int64_t grid = (N + rpb - 1) / rpb;
  AON_REQUIRE(grid < (1ll << 31), "too many rows");
  hipStream_t st = (hipStream_t)stream;
  uint32_t* amax = static_cast<uint32_t*>(work);
  // the fp16x3 chain's per-call gradient scale (bf16 runs unscaled: no max pass)
  const int rc = bf16 ? 0 : absmax(draw, 4 * N, amax, st);
  if (rc) return rc;
  const ArtBwdArgs args{draw, reinterpret_cast<const uint2*>(masks), enc, dzv, dbot, dz, dxp, dzd,
                        amax, N};
  const f4* wsp = static_cast<const f4*>(packed);
  const float* bias =
      reinterpret_cast<const float*>(static_cast<const char*>(packed) + NetArtBwdH::kStreamBytes);
  if (bf16)
    hipLaunchKernelGGL(k_mlp_art_bwd_f16x3<true>, (unsigned)grid, ArtBwdGeom<true>::kThreads, 0, st,
                       wsp, bias, args);
  else
    hipLaunchKernelGGL(k_mlp_art_bwd_f16x3<false>, (unsigned)grid, ArtBwdGeom<false>::kThreads, 0,
                       st, wsp, bias, args);
  return launch_status(bf16 ? "aon_mlp_art_bwd_bf16" : "aon_mlp_art_bwd");
}

extern "C" int aon_mlp_art_bwd(const void* packed, const float* draw, const uint32_t* masks,
                               const float* enc, int64_t N, float* dzv, float* dbot, float* dz,
                               float* dxp, float* dzd, void* work, aon_stream_t stream) {
  return art_bwd(packed, draw, masks, enc, N, dzv, dbot, dz, dxp, dzd, work, stream, false);
}

extern "C" int aon_mlp_art_bwd_bf16(const void* packed, const float* draw, const uint32_t* masks,
                                    const float* enc, int64_t N, void* dzv, void* dbot, void* dz,
                                    float* dxp, void* dzd, void* work, aon_stream_t stream) {
  return art_bwd(packed, draw, masks, enc, N, static_cast<float*>(dzv), static_cast<float*>(dbot),
                 static_cast<float*>(dz), dxp, static_cast<float*>(dzd), work, stream, true);
}
