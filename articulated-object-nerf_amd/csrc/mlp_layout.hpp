// Compile-time layout of the packed NeRFMLP weight stream (shared by pack and forward).
//
// The MLP runs "feature-major": a layer computes D[out][sample] = W[out][in] . H[in][sample]
// with 16x16 MFMA tiles, samples on the MFMA column (lane & 15) and features on the rows.
// The accumulator of one layer is then already the B operand of the next (no LDS round
// trip): k-step (t, r) of the next layer takes register r of feature tile t, whose lane group
// g = lane >> 4 holds input feature 16t + 4g + r.
//
// Weight stream = the A operands in consumption order.  One 1-KB "block" (t, u) holds, for lane
// l, the float4 W[16u + (l & 15)][16t + 4(l >> 4) + 0..3] -> one conflict-free ds_read_b128 per
// lane feeds 4 MFMAs.  Blocks are ordered layer by layer, t-major, u-minor, and padded to whole
// LDS chunks.  Inputs with two concatenated segments (the skip layer cat[h, enc], the view
// layer cat[bottleneck, enc_dir]; reference model.py:102-103, 113) are two K ranges of the same
// layer; padded features (63 -> 64, 27 -> 32) carry zero weights.
#pragma once

namespace aon {
namespace mlp {

struct LayerDesc {
  int ka, kb;        // 16-feature input tiles of segment A / B
  int u;             // 16-row output tiles
  int len_a, len_b;  // real columns of segment A / B in the torch weight ([out][len_a+len_b])
  int out_real;      // real output rows
  int blk0;          // first 1-KB block in the stream
  int bias0;         // first float in the bias table (u*16 floats per layer)
};

enum { L0 = 0, L1, L2, L3, L4, L5, L6, L7, LDEN, LBOT, LVIEW, LRGB, kNumLayers };

constexpr int kChunk = 16;  // 1-KB blocks per LDS pipeline stage

constexpr LayerDesc kLayers[kNumLayers] = {
    {4, 0, 16, 63, 0, 256, 0, 0},             // pts_linears.0   256 x 63
    {16, 0, 16, 256, 0, 256, 64, 256},        // pts_linears.1
    {16, 0, 16, 256, 0, 256, 320, 512},       // pts_linears.2
    {16, 0, 16, 256, 0, 256, 576, 768},       // pts_linears.3
    {16, 0, 16, 256, 0, 256, 832, 1024},      // pts_linears.4
    {16, 4, 16, 256, 63, 256, 1088, 1280},    // pts_linears.5   256 x (256 + 63)
    {16, 0, 16, 256, 0, 256, 1408, 1536},     // pts_linears.6
    {16, 0, 16, 256, 0, 256, 1664, 1792},     // pts_linears.7
    {16, 0, 1, 256, 0, 1, 1920, 2048},        // density_layer     1 x 256
    {16, 0, 16, 256, 0, 256, 1936, 2064},     // bottleneck_layer 256 x 256
    {16, 2, 8, 256, 27, 128, 2192, 2320},     // views_linear.0  128 x (256 + 27)
    {8, 0, 1, 128, 0, 3, 2336, 2448},         // rgb_layer         3 x 128
};

// The fp16x3 kernel (mlp_f16x3.hip) walks the SAME block grid with 32-feature k-steps and
// two 1-KB blocks (hi, lo) per (u, k-step): ka/kb count 32-feature k-steps, and segment B
// (enc / enc_dir, computed in-register) uses the natural feature order.
constexpr LayerDesc kLayersH[kNumLayers] = {
    {0, 2, 16, 0, 63, 256, 0, 0},             // pts_linears.0: enc only (segment B)
    {8, 0, 16, 256, 0, 256, 64, 256},
    {8, 0, 16, 256, 0, 256, 320, 512},
    {8, 0, 16, 256, 0, 256, 576, 768},
    {8, 0, 16, 256, 0, 256, 832, 1024},
    {8, 2, 16, 256, 63, 256, 1088, 1280},
    {8, 0, 16, 256, 0, 256, 1408, 1536},
    {8, 0, 16, 256, 0, 256, 1664, 1792},
    {8, 0, 1, 256, 0, 1, 1920, 2048},
    {8, 0, 16, 256, 0, 256, 1936, 2064},
    {8, 1, 8, 256, 27, 128, 2192, 2320},
    {4, 0, 1, 128, 0, 3, 2336, 2448},
};

// V1 numerics (AON_F16X3_V2 = 0, kept for A/B only): activations and biases carried at 2^-8,
// lo halves at 2^11, two accumulators
constexpr float kActScale = 1.0f / 256.0f;
constexpr float kLoScale = 2048.0f;
// V2 numerics (AON_F16X3_V2, the default): activations carried at 2^3, weights at 2^6, so the
// lo parts (x - fp16(x)) stay in fp16's normal range unscaled and hi*hi, hi*lo, lo*hi share ONE
// fp32 accumulator at scale 2^9; the epilogue folds the 2^-6 and the bias into one fma.  A
// hidden activation past 65504 / 2^3 overflows the hi part: the range guard reports it.
#ifndef AON_F16X3_V2
#define AON_F16X3_V2 1
#endif
constexpr float kActS = 8.0f;
constexpr float kWS = 64.0f;

constexpr int kBlocks = 2344;                                     // sum of (ka+kb)*u
constexpr int kStreamBlocks = (kBlocks + 63) / 64 * 64;          // 2368: whole chunks of 16/32/64
constexpr int kNumChunks = kStreamBlocks / kChunk;                // 148
constexpr int kBiasFloats = 2464;
constexpr size_t kStreamBytesF32 = (size_t)kStreamBlocks * 1024;
// every packed buffer ends in a 16-B status block (word 0: the fp16x3 range guard,
// mlp_f16x3_core.hpp range_report; zeroed by the pack, read by aon_mlp_status)
constexpr size_t kStatusBytes = 16;
constexpr size_t kPackedBytesF32 = kStreamBytesF32 + kBiasFloats * 4 + kStatusBytes;

constexpr bool layout_ok() {
  int blk = 0, bias = 0;
  for (int i = 0; i < kNumLayers; ++i) {
    const LayerDesc& d = kLayers[i];
    if (d.blk0 != blk || d.bias0 != bias) return false;
    if (d.blk0 % kChunk) return false;  // every layer starts on a chunk boundary
    if (!(d.u == 1 || d.u % 4 == 0)) return false;
    blk += (d.ka + d.kb) * d.u;
    bias += d.u * 16;
  }
  return blk == kBlocks && bias == kBiasFloats;
}
static_assert(layout_ok(), "inconsistent MLP stream layout");

constexpr bool layout_h_ok() {
  for (int i = 0; i < kNumLayers; ++i) {
    const LayerDesc& a = kLayers[i];
    const LayerDesc& h = kLayersH[i];
    if (a.blk0 != h.blk0 || a.bias0 != h.bias0 || a.u != h.u) return false;
    if ((h.ka + h.kb) * h.u * 2 != (a.ka + a.kb) * a.u) return false;
  }
  return true;
}
static_assert(layout_h_ok(), "fp16x3 layout must share the block grid");

// ---- the articulated NeRFMLP (reference model_autodecoder.py:60-239, default geometry) on the
// fp16x3 path, after latent folding: the latent columns of deformations_linear.0,
// pts_linears.0 / .5 and views_linear.0 meet the same (1, C) code on every sample, so their
// products are per-call biases (NeRFMLP.folded_biases) and the stream holds only the
// per-sample columns.  Same block grid rules as kLayersH; ka/kb in 32-feature k-steps.
enum {
  A_D0 = 0, A_D1, A_D2, A_D3, A_DOUT,
  A_P0, A_P1, A_P2, A_P3, A_P4, A_P5, A_P6, A_P7,
  A_DEN, A_BOT, A_V0, A_V1, A_V2, A_V3, A_RGB, kNumLayersArt
};

constexpr LayerDesc kLayersArt[kNumLayersArt] = {
    {0, 1, 8, 0, 3, 128, 0, 0},              // deformations_linear.0  128 x 3 (xyz columns)
    {4, 0, 8, 128, 0, 128, 16, 128},         // deformations_linear.1
    {4, 0, 8, 128, 0, 128, 80, 256},         // deformations_linear.2
    {4, 0, 8, 128, 0, 128, 144, 384},        // deformations_linear.3
    {4, 0, 1, 128, 0, 3, 208, 512},          // deformation_layer        3 x 128
    {0, 2, 16, 0, 63, 256, 216, 528},        // pts_linears.0   256 x 63 (enc columns)
    {8, 0, 16, 256, 0, 256, 280, 784},       // pts_linears.1
    {8, 0, 16, 256, 0, 256, 536, 1040},      // pts_linears.2
    {8, 0, 16, 256, 0, 256, 792, 1296},      // pts_linears.3
    {8, 0, 16, 256, 0, 256, 1048, 1552},     // pts_linears.4
    {8, 2, 16, 256, 63, 256, 1304, 1808},    // pts_linears.5   256 x (256 + 63)
    {8, 0, 16, 256, 0, 256, 1624, 2064},     // pts_linears.6
    {8, 0, 16, 256, 0, 256, 1880, 2320},     // pts_linears.7
    {8, 0, 1, 256, 0, 1, 2136, 2576},        // density_layer    1 x 256
    {8, 0, 16, 256, 0, 256, 2152, 2592},     // bottleneck_layer 256 x 256
    {8, 1, 8, 256, 27, 128, 2408, 2848},     // views_linear.0   128 x (256 + 27)
    {4, 0, 8, 128, 0, 128, 2552, 2976},      // views_linear.1
    {4, 0, 8, 128, 0, 128, 2616, 3104},      // views_linear.2
    {4, 0, 8, 128, 0, 128, 2680, 3232},      // views_linear.3
    {4, 0, 1, 128, 0, 3, 2744, 3360},        // rgb_layer        3 x 128
};

// ---- backward chain of the vanilla NeRFMLP (training, model.py:95-120 under autograd): the
// input gradients dL/dX = dZ W (W^T applied feature-major), last layer first, each masked by
// ReLU' of the forward output it flows into.  Row o of a layer = an INPUT feature of the forward
// layer, columns = its outputs; packed from the forward weights with tr = 1.
enum { B_RGB = 0, B_VIEW, B_BOTDEN, B_7, B_6, B_5, B_4, B_3, B_2, B_1, kNumLayersBwd };

constexpr LayerDesc kLayersBwd[kNumLayersBwd] = {
    {0, 1, 8, 0, 3, 128, 0, 0},             // rgb_layer^T: d hv = W_rgb^T d rgb (3 -> 128)
    {4, 0, 16, 128, 0, 256, 16, 128},       // views_linear.0^T, bottleneck columns only
    {8, 1, 16, 256, 1, 256, 144, 384},      // [bottleneck^T | density^T]: d h7
    {8, 0, 16, 256, 0, 256, 432, 640},      // pts_linears.7^T: d h6
    {8, 0, 16, 256, 0, 256, 688, 896},      // pts_linears.6^T: d h5
    {8, 0, 16, 256, 0, 256, 944, 1152},     // pts_linears.5^T, h4 columns only (not enc)
    {8, 0, 16, 256, 0, 256, 1200, 1408},    // pts_linears.4^T: d h3
    {8, 0, 16, 256, 0, 256, 1456, 1664},    // pts_linears.3^T: d h2
    {8, 0, 16, 256, 0, 256, 1712, 1920},    // pts_linears.2^T: d h1
    {8, 0, 16, 256, 0, 256, 1968, 2176},    // pts_linears.1^T: d h0
};

// ---- backward chain of the articulated NeRFMLP (training, model_autodecoder.py:168-239 under
// autograd), same conventions as kLayersBwd: the view branch, the bottleneck / density heads,
// the trunk, the enc columns of pts_linears.5 (the skip) and of pts_linears.0 (256 -> 63: the
// gradient w.r.t. pos_enc(x'), reduced in registers through pos_enc's backward to dL/dx'), the
// deformation head and the deformation MLP.  Latent columns carry no per-sample gradient (their
// codes' gradients come from the bias gradients, train_art.py).
enum {
  AB_RGB = 0, AB_V3, AB_V2, AB_V1, AB_V0, AB_BOTDEN, AB_P7, AB_P6, AB_P5, AB_P5E, AB_P4, AB_P3,
  AB_P2, AB_P1, AB_P0E, AB_DL, AB_D3, AB_D2, AB_D1, kNumLayersArtBwd
};

constexpr LayerDesc kLayersArtBwd[kNumLayersArtBwd] = {
    {0, 1, 8, 0, 3, 128, 0, 0},             // rgb_layer^T: d hv3 (3 -> 128)
    {4, 0, 8, 128, 0, 128, 16, 128},        // views_linear.3^T: d hv2
    {4, 0, 8, 128, 0, 128, 80, 256},        // views_linear.2^T: d hv1
    {4, 0, 8, 128, 0, 128, 144, 384},       // views_linear.1^T: d hv0
    {4, 0, 16, 128, 0, 256, 208, 512},      // views_linear.0^T, bottleneck columns: d bottleneck
    {8, 1, 16, 256, 1, 256, 336, 768},      // [bottleneck^T | density^T]: d h7
    {8, 0, 16, 256, 0, 256, 624, 1024},     // pts_linears.7^T: d h6
    {8, 0, 16, 256, 0, 256, 880, 1280},     // pts_linears.6^T: d h5
    {8, 0, 16, 256, 0, 256, 1136, 1536},    // pts_linears.5^T, h4 columns: d h4
    {8, 0, 4, 256, 0, 63, 1392, 1792},      // pts_linears.5^T, enc columns: d enc (skip)
    {8, 0, 16, 256, 0, 256, 1456, 1856},    // pts_linears.4^T: d h3
    {8, 0, 16, 256, 0, 256, 1712, 2112},    // pts_linears.3^T: d h2
    {8, 0, 16, 256, 0, 256, 1968, 2368},    // pts_linears.2^T: d h1
    {8, 0, 16, 256, 0, 256, 2224, 2624},    // pts_linears.1^T: d h0
    {8, 0, 4, 256, 0, 63, 2480, 2880},      // pts_linears.0^T, enc columns: d enc
    {0, 1, 8, 0, 3, 128, 2544, 2944},       // deformation_layer^T: d hd3 (3 -> 128)
    {4, 0, 8, 128, 0, 128, 2560, 3072},     // deformations_linear.3^T: d hd2
    {4, 0, 8, 128, 0, 128, 2624, 3200},     // deformations_linear.2^T: d hd1
    {4, 0, 8, 128, 0, 128, 2688, 3328},     // deformations_linear.1^T: d hd0
};

// compile-time description of one fp16x3 network: its layer table and stream geometry
template <const LayerDesc* TABLE, int NLAYERS, int BLOCKS, int STREAM_BLOCKS, int BIAS_FLOATS,
          bool ZERO_BIAS = false>
struct NetH {
  static constexpr const LayerDesc* kTable = TABLE;
  static constexpr bool kZeroBias = ZERO_BIAS;  // the backward chains: an all-zero bias table
  static constexpr int kNumLayers = NLAYERS;
  static constexpr int kBlocks = BLOCKS;               // blocks carrying weights
  static constexpr int kStreamBlocks = STREAM_BLOCKS;  // padded to whole LDS chunks
  static constexpr int kBiasFloats = BIAS_FLOATS;
  static constexpr size_t kStreamBytes = (size_t)STREAM_BLOCKS * 1024;
  static constexpr size_t kPackedBytes = kStreamBytes + (size_t)BIAS_FLOATS * 4 + kStatusBytes;
  static constexpr LayerDesc layer(int i) { return TABLE[i]; }
  static constexpr bool ok() {
    int blk = 0, bias = 0;
    for (int i = 0; i < NLAYERS; ++i) {
      const LayerDesc d = TABLE[i];
      if (d.blk0 != blk || d.bias0 != bias || d.blk0 % 2) return false;
      if (!(d.u == 1 || d.u % 2 == 0)) return false;
      if (d.len_a > 32 * d.ka || d.len_b > 32 * d.kb || d.out_real > 16 * d.u) return false;
      blk += (d.ka + d.kb) * d.u * 2;
      bias += d.u * 16;
    }
    return blk == BLOCKS && bias == BIAS_FLOATS && STREAM_BLOCKS >= BLOCKS &&
           STREAM_BLOCKS % 64 == 0;
  }
};

using NetVanillaH = NetH<kLayersH, kNumLayers, kBlocks, kStreamBlocks, kBiasFloats>;
using NetArtH = NetH<kLayersArt, kNumLayersArt, 2752, 2752, 3376>;
using NetBwdH = NetH<kLayersBwd, kNumLayersBwd, 2224, 2240, 2432, true>;
using NetArtBwdH = NetH<kLayersArtBwd, kNumLayersArtBwd, 2752, 2752, 3456, true>;
static_assert(NetVanillaH::ok(), "inconsistent vanilla fp16x3 layout");
static_assert(NetArtH::ok(), "inconsistent articulated fp16x3 layout");
static_assert(NetBwdH::ok(), "inconsistent backward-chain fp16x3 layout");
static_assert(NetArtBwdH::ok(), "inconsistent articulated backward-chain fp16x3 layout");

// pack-kernel arguments: per-layer torch parameter pointers + the layout table by value
struct PackArgs {
  const float* w[kNumLayers];
  const float* b[kNumLayers];
  LayerDesc layers[kNumLayers];
};

// fp16x3 pack: any NetH; ldw = row stride of each torch weight ([out][ldw], the real columns
// first: latent columns past len_a + len_b are folded into the biases)
constexpr int kMaxLayersH = 24;
// tr: the layer applies W^T (the backward chain): stream element (row o, column c) = w[c][o].
// w2 / ldw2: segment B from its own matrix (else columns len_a.. of w); b may be null (0).
struct PackArgsH {
  const float* w[kMaxLayersH];
  const float* w2[kMaxLayersH];
  const float* b[kMaxLayersH];
  int ldw[kMaxLayersH];
  int ldw2[kMaxLayersH];
  int tr[kMaxLayersH];
  LayerDesc layers[kMaxLayersH];
  int n_layers, stream_blocks, bias_floats;
  // 0: fp16x3; 1: bf16 (compact, StreamMap mode 1); 2: mixed -- fp16x3 pairs for the blocks
  // [mx_lo, mx_hi) of the fp16x3 numbering, compact bf16 for the rest (the articulated bf16
  // training mode keeps the deformation MLP in fp16x3, StreamMap mode 2)
  int bf16;
  int mx_lo, mx_hi;
  // compact blocks (modes 1, 2) hold fp16(w 2^6) instead of bf16(w), range-guarded like the
  // fp16x3 hi blocks, and their layers' biases are at activation scale (FragPipe W1)
  int f16w;
};

// Where the weight stream holds fp16x3 block b (even b: the hi block of a (hi, lo) pair, b + 1
// its lo block) -- shared by k_pack_h and FragPipe.  mode 0: fp16x3, in place; 1: bf16 compact,
// only hi blocks, block 2c at c; 2: mixed, [lo, hi) kept as fp16x3 pairs (lo even), every other
// hi block compact bf16, all in consumption order (the ring's chunk starts are still met: a
// chunk boundary is even, so it falls on a pair's hi block or a bf16 block).
struct StreamMap {
  int mode, lo, hi;
  __host__ __device__ constexpr bool f16(int b) const {
    return mode == 0 || (mode == 2 && b >= lo && b < hi);
  }
  __host__ __device__ constexpr int map(int b) const {
    return mode == 0 ? b
         : mode == 1 ? b >> 1
         : b < lo    ? b >> 1
         : b < hi    ? (lo >> 1) + b - lo
                     : (lo >> 1) + (hi - lo) + ((b - hi) >> 1);
  }
  // stream block m -> its fp16x3 block
  __host__ __device__ constexpr int unmap(int m) const {
    return mode == 0 ? m
         : mode == 1 ? 2 * m
         : m < (lo >> 1)            ? 2 * m
         : m < (lo >> 1) + hi - lo  ? lo + m - (lo >> 1)
                                    : hi + 2 * (m - (lo >> 1) - (hi - lo));
  }
  // stream blocks carrying the `blocks` weight blocks of the fp16x3 numbering
  __host__ __device__ constexpr int used(int blocks) const {
    return mode == 0 ? blocks : mode == 1 ? blocks / 2 : (lo >> 1) + (hi - lo) + ((blocks - hi) >> 1);
  }
};
// the articulated forward's mixed stream: the deformation MLP (kLayersArt blocks 0..215)
// fp16x3 -- x' feeds pos_enc's sin(2^9 x'), where bf16's 2^-9 would cost whole radians -- the
// trunk, heads and view branch compact bf16: 216 + 1268 = 1484 blocks, 1536 with the padding
constexpr StreamMap kArtMix{2, 0, 216};
constexpr int kArtMixUsed = kArtMix.used(2752);
constexpr int kArtMixStream = (kArtMixUsed + 63) / 64 * 64;
static_assert(kArtMixUsed == 1484 && kArtMixStream == 1536, "mixed articulated stream");
static_assert(kArtMix.unmap(kArtMix.map(2750)) == 2750 && kArtMix.unmap(kArtMix.map(214)) == 214 &&
                  kArtMix.map(216) == 216 && kArtMix.map(218) == 217,
              "stream map round trip");
// the articulated bf16 mode's view-branch stream (train_art.BF16_VIEW): the deformation MLP, the
// trunk, density and bottleneck fp16x3 (blocks 0..2407 -- everything the deformation gradients
// are ill-conditioned in), views_linear.0-3 and rgb_layer compact bf16: 2408 + 172 = 2580 blocks
constexpr StreamMap kArtMixV{2, 0, 2408};
constexpr int kArtMixVUsed = kArtMixV.used(2752);
constexpr int kArtMixVStream = (kArtMixVUsed + 63) / 64 * 64;
static_assert(kArtMixVUsed == 2580 && kArtMixVStream == 2624 && kArtMixVStream <= 2752,
              "view-branch mixed articulated stream");
static_assert(kLayersArt[A_V0].blk0 == kArtMixV.hi && kArtMixV.map(2408) == 2408 &&
                  kArtMixV.unmap(kArtMixV.map(2750)) == 2750,
              "view-branch stream map");

// Training forward of the fused kernel (launch_f16x3 mode 2): every hidden activation goes to
// HBM for the backward, as the layer-by-layer path keeps them: h (8, N, 256) post-ReLU
// pts_linears outputs, bot (N, 256), hv (N, 128) post-ReLU views_linear.0; raw_sigma gets
// + noise[row] when noise is set (model.py:183-184).
struct TrainStore {
  float* h;
  float* bot;
  float* hv;
  const float* noise;
  uint2* masks;  // (9, N, 4) ReLU' bits of h0..h7, hv (RowStoreBits)
  __bf16* enc_bf;  // bf16 mode, optional: pos_enc(x) tiled (N, 128), columns 63.. zero
};

// activations the articulated training forward keeps (aon_mlp_art_fwd_train)
struct TrainStoreArt {
  float* hd;    // (4, N, 128) deformation layers
  float* h;     // (8, N, 256) pts_linears
  float* bot;   // (N, 256)
  float* hv;    // (4, N, 128) views_linear
  float* enc;   // (N, 63) pos_enc(x'); enc[:, :3] = x'
  float* xyz;   // (N, 3) the sample points (deformation input)
  const float* noise;  // (N) added to raw_sigma, or nullptr
  uint2* masks;        // (16, N, 4) ReLU' bits of hd0..3, h0..7, hv0..3 (RowStoreBits)
  __bf16* enc_bf;      // bf16 modes, optional: pos_enc(x') tiled (N, 128), columns 63.. zero
};

// fp16x3 path (mlp_f16x3.hip)
int pack_f16x3(const PackArgs& a, void* packed, hipStream_t stream, bool bf16 = false);
int pack_h(PackArgsH a, void* packed, hipStream_t stream);
// *out = bits of max |x| over n floats (memset + k_absmax, mlp_bwd.hip): the backward chains'
// per-call gradient scale
int absmax(const float* x, int64_t n, uint32_t* out, hipStream_t stream);
int launch_f16x3(int mode, int ncol, const void* packed, const float* a0, const float* a1,
                 const float* a2, const float* a3, int64_t B, int S, int act, float* raw,
                 hipStream_t stream, const TrainStore* ts = nullptr);
// the weight-streamed fp16x3 render forward (mlp_ws.hip; MODE 0 inputs, bit-identical to
// launch_f16x3 mode 0) -- an A/B variant, not in the release library: `make variant-ws` builds
// lib/variants/libaonerf_ws.so with AON_DATAFLOW_WS_BUILD = 1, whose render forwards
// (aon_mlp_fwd, aon_mlp_art_fwd) take this dataflow; the release build has no process-global
// kernel selection and no environment knobs
#ifndef AON_DATAFLOW_WS_BUILD
#define AON_DATAFLOW_WS_BUILD 0
#endif
int launch_ws_f16x3(const void* packed, const float* a0, const float* a1, const float* a2,
                    const float* a3, int64_t B, int S, int act, float* raw, hipStream_t stream);
int launch_art_ws_f16x3(const void* packed, const float* a0, const float* a1, const float* a2,
                        const float* a3, int64_t B, int S, int act, float* raw, hipStream_t stream);

}  // namespace mlp
}  // namespace aon
