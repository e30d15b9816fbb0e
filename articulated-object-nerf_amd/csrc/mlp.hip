// Fused NeRFMLP forward (reference models/vanilla_nerf/model.py:95-120, fed as at model.py:
// 175-181) on fp32 MFMA -- the MFMA-bound kernel of the hot path.
//
// Workgroup = 8 waves x 16 samples; every wave keeps its 16 samples' activations for all 256
// features in registers (16 f4 tiles) for the whole network:
//   enc  = pos_enc(o + t*d) (64 features, 4 tiles)   venc = pos_enc(viewdir) (32, 2 tiles)
//   L0..L7 (skip cat at L5), density head, bottleneck, view layer, rgb head
// Only the weights move: the packed stream (mlp_layout.hpp) flows HBM/L2 -> registers -> LDS in
// 16-KB chunks, double-buffered with one workgroup barrier per chunk, and every lane reads its
// A operand with one ds_read_b128 per 4 MFMAs.  Biases sit in LDS and seed the accumulators.
//
// v_mfma_f32_16x16x4_f32 is exact fp32 (a k-ordered fmaf chain): the result differs from the
// reference's fp32 GEMM only by summation order.
#include "aon_common.hpp"
#include "mlp_layout.hpp"
#include "mlp_pipe.hpp"
#include "param_check.hpp"

namespace aon {
namespace mlp {

constexpr int kWaves = 8;
constexpr int kThreads = 64 * kWaves;
constexpr int kRowsPerWave = 16;
constexpr int kRowsPerBlock = kRowsPerWave * kWaves;

__device__ __forceinline__ f4 mfma(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// acc[u] (+)= W . [xa ; xb] over the layer's blocks, U output tiles (U % 4 == 0)
template <int LAYER, int NA, int NB, int NACC>
__device__ __forceinline__ void gemm(Pipe<kThreads>& p, const f4 (&xa)[NA], const f4 (&xb)[NB],
                                     f4 (&acc)[NACC]) {
  constexpr LayerDesc d = kLayers[LAYER];
  constexpr int U = d.u;
  static_assert(U % 4 == 0 && U <= NACC && d.ka <= NA && d.kb <= NB, "layer/array mismatch");
#pragma unroll
  for (int t = 0; t < d.ka + d.kb; ++t) {
    const f4 x = t < d.ka ? xa[t < NA ? t : 0] : xb[(t >= d.ka && t - d.ka < NB) ? t - d.ka : 0];
#pragma unroll
    for (int ug = 0; ug < U; ug += 4) {
      const int b = d.blk0 + t * U + ug;
      if (b % kChunk == 0 && b > 0) p.begin(b / kChunk);
      f4 a[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) a[k] = p.block(b + k);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int k = 0; k < 4; ++k) acc[ug + k] = mfma(a[k][r], x[r], acc[ug + k]);
      }
    }
  }
}

// single output tile (density / rgb heads): two interleaved accumulators over t
template <int LAYER, int NA>
__device__ __forceinline__ f4 gemm_u1(Pipe<kThreads>& p, const f4 (&xa)[NA], f4 init) {
  constexpr LayerDesc d = kLayers[LAYER];
  static_assert(d.u == 1 && d.kb == 0 && d.ka <= NA && d.ka % 2 == 0, "head layer shape");
  f4 acc0 = init, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < d.ka; t += 2) {
    const int b = d.blk0 + t;
    if (b % kChunk == 0 && b > 0) p.begin(b / kChunk);
    const f4 a0 = p.block(b), a1 = p.block(b + 1);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      acc0 = mfma(a0[r], xa[t][r], acc0);
      acc1 = mfma(a1[r], xa[t + 1][r], acc1);
    }
  }
  return acc0 + acc1;
}

template <int LAYER, int N>
__device__ __forceinline__ void init_bias(f4 (&acc)[N], const float* bias_s, int g) {
  constexpr LayerDesc d = kLayers[LAYER];
#pragma unroll
  for (int u = 0; u < d.u; ++u) acc[u] = *reinterpret_cast<const f4*>(bias_s + d.bias0 + 16 * u + 4 * g);
}

template <int N>
__device__ __forceinline__ void relu_into(f4 (&dst)[16], const f4 (&src)[N]) {
#pragma unroll
  for (int u = 0; u < N; ++u) {
#pragma unroll
    for (int r = 0; r < 4; ++r) dst[u][r] = fmaxf(src[u][r], 0.0f);
  }
}

// MODE 0: inputs (rays_o, rays_d, viewdirs, t) -> xyz + pos_enc in-kernel
// MODE 1: inputs (x = encoded points (N, 63), cond = encoded view dirs (B, 27))
template <int MODE>
__global__ __launch_bounds__(kThreads, 2) void k_mlp_fwd_f32(
    const f4* __restrict__ wstream, const float* __restrict__ bias_g, const float* __restrict__ in0,
    const float* __restrict__ in1, const float* __restrict__ in2, const float* __restrict__ in3,
    int64_t B, int S, int act, float* __restrict__ raw) {
  __shared__ f4 wbuf[2 * kChunk * 64];
  __shared__ __attribute__((aligned(16))) float bias_s[kBiasFloats];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, j = lane & 15;
  const int64_t N = B * S;
  const int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + wave * kRowsPerWave + j;
  const int64_t rr = row < N ? row : N - 1;
  const int64_t ray = rr / S;

  Pipe<kThreads> p;
  p.wbuf = wbuf;
  p.src = wstream;
  p.tid = tid;
  p.lane = lane;
  p.load(0);
  for (int i = tid; i < kBiasFloats; i += kThreads) bias_s[i] = bias_g[i];

  // ---- layer-0 / view-layer inputs in B-operand layout: tile t, reg r <-> feature 16t+4g+r
  f4 enc[4], venc[2];
  if (MODE == 0) {
    const float* ro = in0 + 3 * ray;
    const float* rd = in1 + 3 * ray;
    const float* vd = in2 + 3 * ray;
    const float tt = in3[rr];
    // cast_rays (helper.py:25-26): o + t*d, separately rounded
    const float x0 = __fadd_rn(ro[0], __fmul_rn(tt, rd[0]));
    const float x1 = __fadd_rn(ro[1], __fmul_rn(tt, rd[1]));
    const float x2 = __fadd_rn(ro[2], __fmul_rn(tt, rd[2]));
    const float v0 = vd[0], v1 = vd[1], v2 = vd[2];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) enc[t][r] = pos_enc_feature(x0, x1, x2, 16 * t + 4 * g + r, 0, 10);
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) venc[t][r] = pos_enc_feature(v0, v1, v2, 16 * t + 4 * g + r, 0, 4);
  } else {
    const float* x = in0 + rr * 63;
    const float* c = in1 + ray * 27;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int f = 16 * t + 4 * g + r;
        enc[t][r] = f < 63 ? x[f] : 0.f;
      }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int f = 16 * t + 4 * g + r;
        venc[t][r] = f < 27 ? c[f] : 0.f;
      }
  }

  p.begin(0);  // also publishes bias_s

  f4 h[16], acc[16];
  const f4 none[1] = {{0.f, 0.f, 0.f, 0.f}};

  init_bias<L0>(acc, bias_s, g);
  gemm<L0>(p, enc, none, acc);
  relu_into(h, acc);
  init_bias<L1>(acc, bias_s, g);
  gemm<L1>(p, h, none, acc);
  relu_into(h, acc);
  init_bias<L2>(acc, bias_s, g);
  gemm<L2>(p, h, none, acc);
  relu_into(h, acc);
  init_bias<L3>(acc, bias_s, g);
  gemm<L3>(p, h, none, acc);
  relu_into(h, acc);
  init_bias<L4>(acc, bias_s, g);
  gemm<L4>(p, h, none, acc);
  relu_into(h, acc);
  init_bias<L5>(acc, bias_s, g);  // skip: cat[h, enc] (model.py:102-103)
  gemm<L5>(p, h, enc, acc);
  relu_into(h, acc);
  init_bias<L6>(acc, bias_s, g);
  gemm<L6>(p, h, none, acc);
  relu_into(h, acc);
  init_bias<L7>(acc, bias_s, g);
  gemm<L7>(p, h, none, acc);
  relu_into(h, acc);

  // density head on the layer-7 features (model.py:105-107): row 0 of the tile
  const f4 dens = gemm_u1<LDEN>(p, h, *reinterpret_cast<const f4*>(bias_s + kLayers[LDEN].bias0 + 4 * g));

  // bottleneck, no activation (model.py:109)
  init_bias<LBOT>(acc, bias_s, g);
  gemm<LBOT>(p, h, none, acc);
#pragma unroll
  for (int u = 0; u < 16; ++u) h[u] = acc[u];

  // view layer on cat[bottleneck, enc_dir] + ReLU (model.py:110-116)
  f4 vacc[8];
  init_bias<LVIEW>(vacc, bias_s, g);
  gemm<LVIEW>(p, h, venc, vacc);
  relu_into(h, vacc);

  // rgb head (model.py:118): rows 0..2 of the tile
  const f4 rgb = gemm_u1<LRGB>(p, h, *reinterpret_cast<const f4*>(bias_s + kLayers[LRGB].bias0 + 4 * g));

  if (g == 0 && row < N) {
    const f4 o = {act_rgb(rgb[0], act), act_rgb(rgb[1], act), act_rgb(rgb[2], act),
                  act_sigma(dens[0], act)};
    *reinterpret_cast<f4*>(raw + 4 * row) = o;
  }
}

// ---- packing: torch [out][in] fp32 -> stream blocks (+ padded biases)
__global__ void k_pack_f32(PackArgs a, float* __restrict__ out) {
  const int64_t total = (int64_t)kStreamBlocks * 256 + kBiasFloats;
  if (blockIdx.x == 0 && threadIdx.x == 0) *reinterpret_cast<uint32_t*>(out + total) = 0u;  // status
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    float v = 0.f;
    if (e < (int64_t)kStreamBlocks * 256) {
      const int blk = static_cast<int>(e >> 8);
      const int l = static_cast<int>((e >> 2) & 63), r = static_cast<int>(e & 3);
      if (blk < kBlocks) {
        int li = 0;
        while (li + 1 < kNumLayers && a.layers[li + 1].blk0 <= blk) ++li;
        const LayerDesc d = a.layers[li];
        const int t = (blk - d.blk0) / d.u, u = (blk - d.blk0) % d.u;
        const int o = 16 * u + (l & 15);
        const int f = 16 * t + 4 * (l >> 4) + r;
        int col = -1;
        if (f < 16 * d.ka) {
          col = f < d.len_a ? f : -1;
        } else {
          const int f2 = f - 16 * d.ka;
          col = f2 < d.len_b ? d.len_a + f2 : -1;
        }
        if (o < d.out_real && col >= 0) v = a.w[li][(int64_t)o * (d.len_a + d.len_b) + col];
      }
    } else {
      const int i = static_cast<int>(e - (int64_t)kStreamBlocks * 256);
      int li = 0;
      while (li + 1 < kNumLayers && a.layers[li + 1].bias0 <= i) ++li;
      const int o = i - a.layers[li].bias0;
      if (o < a.layers[li].out_real) v = a.b[li][o];
    }
    out[e] = v;
  }
}

}  // namespace mlp
}  // namespace aon

using namespace aon;
using namespace aon::mlp;

extern "C" size_t aon_mlp_packed_bytes(int precision) {
  // every precision uses the same block grid: fp32 tiles, or hi+lo fp16 pairs of equal size
  // (bf16: bf16 weights in the hi blocks)
  if (precision == AON_PREC_FP32 || precision == AON_PREC_F16X3 || precision == AON_PREC_BF16)
    return kPackedBytesF32;
  return 0;
}

extern "C" int aon_mlp_read_status(const void* packed, size_t packed_bytes, uint32_t* status,
                                   aon_stream_t stream) {
  AON_REQUIRE(packed && status, "null pointer");
  AON_REQUIRE(packed_bytes >= kStatusBytes && packed_bytes % 16 == 0, "bad packed size");
  const char* word = static_cast<const char*>(packed) + packed_bytes - kStatusBytes;
  hipError_t e = hipMemcpyAsync(status, word, sizeof(uint32_t), hipMemcpyDeviceToHost,
                                (hipStream_t)stream);
  if (e == hipSuccess) e = hipStreamSynchronize((hipStream_t)stream);
  return static_cast<int>(e);
}

// samples per wave of the fp16x3 render kernel = 16 x AON_F16X3_NCOL (compile-time A/B knob,
// tools/build_variants.sh; 2 measured 3-5% slower: DESIGN.md §4)
#ifndef AON_F16X3_NCOL
#define AON_F16X3_NCOL 1
#endif
static_assert(AON_F16X3_NCOL == 1 || AON_F16X3_NCOL == 2, "AON_F16X3_NCOL is 1 or 2");

extern "C" int aon_mlp_pack(const aon_mlp_params* prm, int precision, void* packed,
                            aon_stream_t stream) {
  AON_REQUIRE(prm && packed, "null pointer");
  AON_REQUIRE(precision == AON_PREC_FP32 || precision == AON_PREC_F16X3 ||
                  precision == AON_PREC_BF16,
              "unsupported precision");
  AON_REQUIRE(aligned16(packed), "packed buffer must be 16-byte aligned");
  if (check_mlp_params(prm, __func__)) return -1;
  PackArgs a;
  for (int i = 0; i < 8; ++i) {
    a.w[i] = prm->pts_w[i];
    a.b[i] = prm->pts_b[i];
  }
  a.w[LDEN] = prm->density_w;    a.b[LDEN] = prm->density_b;
  a.w[LBOT] = prm->bottleneck_w; a.b[LBOT] = prm->bottleneck_b;
  a.w[LVIEW] = prm->views_w;     a.b[LVIEW] = prm->views_b;
  a.w[LRGB] = prm->rgb_w;        a.b[LRGB] = prm->rgb_b;
  for (int i = 0; i < kNumLayers; ++i) {
    AON_REQUIRE(a.w[i] && a.b[i], "null layer parameter");
    a.layers[i] = precision == AON_PREC_FP32 ? kLayers[i] : kLayersH[i];
  }
  if (precision != AON_PREC_FP32)
    return pack_f16x3(a, packed, (hipStream_t)stream, precision == AON_PREC_BF16);
  // the fp32 kernels never set the range-status word: cleared once here
  const hipError_t e = hipMemsetAsync(static_cast<char*>(packed) + kPackedBytesF32 - kStatusBytes, 0,
                                      kStatusBytes, (hipStream_t)stream);
  if (e != hipSuccess) return static_cast<int>(e);
  const int64_t total = (int64_t)kStreamBlocks * 256 + kBiasFloats;
  hipLaunchKernelGGL(k_pack_f32, grid_for(total, 256, 4096), 256, 0, (hipStream_t)stream, a,
                     static_cast<float*>(packed));
  return launch_status(__func__);
}

static int mlp_launch(int mode, const void* packed, int precision, const float* a0,
                      const float* a1, const float* a2, const float* a3, int64_t B, int S,
                      int act, float* raw, aon_stream_t stream) {
  AON_REQUIRE(packed && raw && a0 && a1, "null pointer");
  AON_REQUIRE(precision == AON_PREC_FP32 || precision == AON_PREC_F16X3,
              "unsupported precision (AON_PREC_BF16 is the training forward's: aon_mlp_fwd_train_bf16)");
  AON_REQUIRE(B >= 0 && S >= 1, "bad shape");
  AON_REQUIRE(act >= AON_ACT_NONE && act <= AON_ACT_ARTIC, "bad activation");
  AON_REQUIRE(aligned16(packed) && aligned16(raw), "packed / raw must be 16-byte aligned");
  const int64_t N = B * S;
  if (N == 0) return 0;
  AON_REQUIRE((N + kRowsPerBlock - 1) / kRowsPerBlock < (1ll << 31), "too many rows");
#if AON_DATAFLOW_WS_BUILD
  if (precision == AON_PREC_F16X3 && mode == 0)
    return launch_ws_f16x3(packed, a0, a1, a2, a3, B, S, act, raw, (hipStream_t)stream);
#endif
  if (precision == AON_PREC_F16X3)
    return launch_f16x3(mode, AON_F16X3_NCOL, packed, a0, a1, a2, a3, B, S, act, raw,
                        (hipStream_t)stream);
  const int grid = static_cast<int>((N + kRowsPerBlock - 1) / kRowsPerBlock);
  const f4* ws = static_cast<const f4*>(packed);
  const float* bias = reinterpret_cast<const float*>(static_cast<const char*>(packed) + kStreamBytesF32);
  if (mode == 0)
    hipLaunchKernelGGL(k_mlp_fwd_f32<0>, grid, kThreads, 0, (hipStream_t)stream, ws, bias, a0, a1,
                       a2, a3, B, S, act, raw);
  else
    hipLaunchKernelGGL(k_mlp_fwd_f32<1>, grid, kThreads, 0, (hipStream_t)stream, ws, bias, a0, a1,
                       a2, a3, B, S, act, raw);
  return launch_status("aon_mlp_fwd");
}

extern "C" int aon_mlp_fwd(const void* packed, int precision, const float* rays_o,
                           const float* rays_d, const float* viewdirs, const float* t, int64_t B,
                           int S, int act, float* raw, aon_stream_t stream) {
  AON_REQUIRE(viewdirs && t, "null pointer");
  return mlp_launch(0, packed, precision, rays_o, rays_d, viewdirs, t, B, S, act, raw, stream);
}

extern "C" int aon_mlp_fwd_encoded(const void* packed, int precision, const float* x,
                                   const float* condition, int64_t B, int S, int act,
                                   float* raw, aon_stream_t stream) {
  return mlp_launch(1, packed, precision, x, condition, nullptr, nullptr, B, S, act, raw, stream);
}

extern "C" int aon_mlp_fwd_train(const void* packed, const float* rays_o, const float* rays_d,
                                 const float* viewdirs, const float* t, int64_t B, int S,
                                 const float* noise, float* h, float* bot, float* hv, float* raw,
                                 uint32_t* masks, aon_stream_t stream) {
  AON_REQUIRE(packed && rays_o && rays_d && viewdirs && t && h && bot && hv && raw && masks,
              "null pointer");
  AON_REQUIRE(aligned16(masks), "masks must be 16-byte aligned");
  AON_REQUIRE(B >= 0 && S >= 1, "bad shape");
  AON_REQUIRE(aligned16(packed) && aligned16(raw) && aligned16(h) && aligned16(bot) && aligned16(hv),
              "packed / output buffers must be 16-byte aligned");
  const int64_t N = B * S;
  if (N == 0) return 0;
  AON_REQUIRE((N + 127) / 128 < (1ll << 31), "too many rows");
  const TrainStore ts{h, bot, hv, noise, reinterpret_cast<uint2*>(masks)};
  return launch_f16x3(2, 1, packed, rays_o, rays_d, viewdirs, t, B, S, AON_ACT_NONE, raw,
                      (hipStream_t)stream, &ts);
}

extern "C" int aon_mlp_fwd_train_bf16(const void* packed, const float* rays_o,
                                      const float* rays_d, const float* viewdirs, const float* t,
                                      int64_t B, int S, const float* noise, uint16_t* h,
                                      uint16_t* bot, uint16_t* hv, float* raw, uint32_t* masks,
                                      uint16_t* enc, aon_stream_t stream) {
  AON_REQUIRE(packed && rays_o && rays_d && viewdirs && t && h && bot && hv && raw && masks,
              "null pointer");
  AON_REQUIRE(B >= 0 && S >= 1, "bad shape");
  AON_REQUIRE(aligned16(packed) && aligned16(raw) && aligned16(masks) && aligned16(h) &&
                  aligned16(bot) && aligned16(hv) && aligned16(enc),
              "packed / output buffers must be 16-byte aligned");
  const int64_t N = B * S;
  if (N == 0) return 0;
  AON_REQUIRE((N + 127) / 128 < (1ll << 31), "too many rows");
  const TrainStore ts{reinterpret_cast<float*>(h), reinterpret_cast<float*>(bot),
                      reinterpret_cast<float*>(hv), noise, reinterpret_cast<uint2*>(masks),
                      reinterpret_cast<__bf16*>(enc)};
  return launch_f16x3(3, 1, packed, rays_o, rays_d, viewdirs, t, B, S, AON_ACT_NONE, raw,
                      (hipStream_t)stream, &ts);
}
