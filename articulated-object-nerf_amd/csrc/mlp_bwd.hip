// Fused backward chain of the vanilla NeRFMLP for the training step (reference model.py:95-120
// under autograd, LitNeRF.training_step model.py:256-282): from dL/d raw (the compositor's
// backward) down to dL/d pre-activation of pts_linears.0, all input-gradient products
// dX = dZ W in ONE kernel, each masked by ReLU' of the forward output it flows into, every
// layer's dZ stored for the weight-gradient GEMMs (dW = dZ^T X runs separately: a reduction
// over all samples).
//
// Same structure and numerics as the forward (mlp_f16x3.hip / mlp_f16x3_core.hpp): feature-
// major MFMA tiles, W^T streamed through the LDS-DMA ring (kLayersBwd, packed from the forward
// weights with tr = 1), each finished output pair converted in registers into the next layer's
// B fragments.  Gradients ride at a power-of-two scale s chosen per call from max|d raw|
// (|d raw * s| < 2^8: 2^8 of headroom below fp16's 65504 for growth through the chain); the
// stores undo it exactly.  The ReLU' masks come from the stored forward activations (h > 0,
// as torch's threshold_backward on the ReLU output), loaded one pair ahead.
#include "mlp_f16x3_core.hpp"
#include "param_check.hpp"

namespace aon {
namespace mlp {

struct BwdArgs {
  const float* draw;              // (N, 4): d raw_rgb (3), d raw_sigma (model.py:183-187 folded)
  const uint2* masks;             // (9, N, 4): ReLU' bits of pts_linears.0..7, views_linear.0
  float* dzv;                     // (N, 128): dL/d pre-activation of views_linear.0
  float* dzb;                     // (N, 256): dL/d bottleneck output
  float* dz;                      // (8, N, 256): dL/d pre-activation of pts_linears.i
  const uint32_t* absmax;         // bits of max |draw| (k_absmax)
  int64_t N;
};

// max |x| over n floats as uint bits (non-negative floats order like their bit patterns)
// (16-B loads over the aligned body, scalar loads for the ragged head / tail)
__global__ void k_absmax(const float* __restrict__ x, int64_t n, uint32_t* __restrict__ out) {
  float m = 0.0f;
  const int64_t tid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t nthreads = (int64_t)gridDim.x * blockDim.x;
  const int64_t head = ((16 - (reinterpret_cast<uintptr_t>(x) & 15)) & 15) / 4;  // floats to 16 B
  const int64_t h = head < n ? head : n;
  const int64_t nv = (n - h) / 4;
  const f4* xv = reinterpret_cast<const f4*>(x + h);
  for (int64_t i = tid; i < nv; i += nthreads) {
    const f4 v = xv[i];
    m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
  }
  for (int64_t i = tid; i < h; i += nthreads) m = fmaxf(m, fabsf(x[i]));
  for (int64_t i = h + 4 * nv + tid; i < n; i += nthreads) m = fmaxf(m, fabsf(x[i]));
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  // one atomic per workgroup: same-address atomics serialise in one L2 channel (one per wave
  // took 50 us on the training step's 3.2 M values)
  __shared__ float wm[4];
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0)
    atomicMax(out, __float_as_uint(fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]))));
}

int absmax(const float* x, int64_t n, uint32_t* out, hipStream_t stream) {
  if (hipMemsetAsync(out, 0, sizeof(uint32_t), stream) != hipSuccess) return launch_status("absmax");
  hipLaunchKernelGGL(k_absmax, grid_for(n / 4 + 1, 256, 512), 256, 0, stream, x, n, out);
  return launch_status("absmax");
}

// BF: the bf16 training mode -- one bf16 MFMA per product, dZ stored as bf16 (BwdArgs' output
// pointers then address bf16 arrays of the same shapes)
// (the bf16 chain runs 16 kBfNcolBwd samples per wave, 8 waves: GeomH<kBfNcolBwd, true>)
template <bool BF = false>
__global__ __launch_bounds__((GeomH<BF ? kBfNcolBwd : 1, BF>::kThreads), 2) void k_mlp_bwd_f16x3(
    const f4* __restrict__ wstream, const float* __restrict__ bias_g, BwdArgs a) {
  constexpr int NCOL = BF ? kBfNcolBwd : 1;
  using T = typename std::conditional<BF, __bf16, float>::type;
  T* const dzv = reinterpret_cast<T*>(a.dzv);
  T* const dzb = reinterpret_cast<T*>(a.dzb);
  T* const dz = reinterpret_cast<T*>(a.dz);
  using G = GeomH<NCOL, BF>;
  using Net = NetBwdH;
  constexpr int kPer = (BF ? 1 : 2) * NCOL;  // f4 per lane: d raw_sigma fragments, hi (& lo)
  constexpr int kStash = G::kWaves * 64 * kPer;
  __shared__ f4 smem[kLdsWeights + Net::kBiasFloats / 4 + kStash];
  float* bias_s = reinterpret_cast<float*>(smem + kLdsWeights);
  f4* stash = smem + kLdsWeights + Net::kBiasFloats / 4 + (threadIdx.x >> 6) * 64 * kPer +
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

  // d raw_rgb -> segment B of rgb_layer^T (lane group 0, elements 0..2); d raw_sigma ->
  // segment B of [bottleneck | density]^T (lane group 0, element 0)
  Frag<1, NCOL> drgb, dsig;
  int64_t rows[NCOL];
#pragma unroll
  for (int c = 0; c < NCOL; ++c) {
    const int64_t row = (int64_t)blockIdx.x * G::kRowsPerBlock + wave * G::kRowsPerWave + 16 * c + j;
    rows[c] = row;
    const int64_t rr = row < N ? row : N - 1;
    const f4 d = *reinterpret_cast<const f4*>(a.draw + 4 * rr);
    float dv[8], sv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      dv[e] = (g == 0 && e < 3) ? d[e < 3 ? e : 0] * s : 0.f;
      sv[e] = (g == 0 && e == 0) ? d[3] * s : 0.f;
    }
    split8<BF>(dv, drgb.hi[0][c], drgb.lo[0][c], drgb.ovf);
    split8<BF>(sv, dsig.hi[0][c], dsig.lo[0][c], dsig.ovf);
    stash[64 * (kPer / NCOL) * c] = __builtin_bit_cast(f4, dsig.hi[0][c]);
    if (!BF) stash[64 * (2 * c + 1)] = __builtin_bit_cast(f4, dsig.lo[0][c]);
  }

  FragPipe<WeightPipeP<Net, G::kThreads, BF>, AON_PREFETCH, 0, BF> fp(p);
  fp.start();
  lds_float* bias_l = opaque_lds(bias_s + 4 * g);

  const int64_t hs = act_rows(N) * 256, ms = act_rows(N) * 4;
  Frag<8, NCOL> x, y;
  Frag<1, NCOL> none;
  // d hv = W_rgb^T d rgb, * ReLU'(hv) -> dZ of views_linear.0
  layer_h<Net, B_RGB, false>(fp, none, drgb, x, bias_l, g,
                             mask_bits(a.masks + 8 * ms, dzv, 128, rows, N, g, inv));
  // d bottleneck = W_view[:, :256]^T dZ_view (linear layer: no mask)
  {
    RowStore<NCOL, T> st;
#pragma unroll
    for (int c = 0; c < NCOL; ++c) {
      st.ok[c] = keep_row(rows[c], N);
      st.rowp[c] = dzb + act_base(rows[c], 256, g);
    }
    st.off16 = st16_off(g);
    st.s = inv;
    layer_h<Net, B_VIEW, false>(fp, x, none, y, bias_l, g, st);
  }
#pragma unroll
  for (int c = 0; c < NCOL; ++c) {
    dsig.hi[0][c] = __builtin_bit_cast(h8, stash[64 * (kPer / NCOL) * c]);
    if (!BF) dsig.lo[0][c] = __builtin_bit_cast(h8, stash[64 * (2 * c + 1)]);
  }
  // d h7 = W_bot^T dZ_bot + W_den^T d sigma, * ReLU'(h7) -> dZ_7
  layer_h<Net, B_BOTDEN, false>(fp, y, dsig, x, bias_l, g,
                                mask_bits(a.masks + 7 * ms, dz + 7 * hs, 256, rows, N, g, inv));
  layer_h<Net, B_7, false>(fp, x, none, y, bias_l, g,
                           mask_bits(a.masks + 6 * ms, dz + 6 * hs, 256, rows, N, g, inv));
  layer_h<Net, B_6, false>(fp, y, none, x, bias_l, g,
                           mask_bits(a.masks + 5 * ms, dz + 5 * hs, 256, rows, N, g, inv));
  // the skip layer's enc columns carry no gradient (positions are not differentiated)
  layer_h<Net, B_5, false>(fp, x, none, y, bias_l, g,
                           mask_bits(a.masks + 4 * ms, dz + 4 * hs, 256, rows, N, g, inv));
  layer_h<Net, B_4, false>(fp, y, none, x, bias_l, g,
                           mask_bits(a.masks + 3 * ms, dz + 3 * hs, 256, rows, N, g, inv));
  layer_h<Net, B_3, false>(fp, x, none, y, bias_l, g,
                           mask_bits(a.masks + 2 * ms, dz + 2 * hs, 256, rows, N, g, inv));
  layer_h<Net, B_2, false>(fp, y, none, x, bias_l, g,
                           mask_bits(a.masks + 1 * ms, dz + 1 * hs, 256, rows, N, g, inv));
  // (the last layer's outputs are only stored: its fp16 split is unused, so not range-checked)
  const uint64_t used_ovf = ovf_of(x) | ovf_of(y) | drgb.ovf | dsig.ovf;
  layer_h<Net, B_1, false>(fp, x, none, y, bias_l, g,
                           mask_bits(a.masks + 0 * ms, dz, 256, rows, N, g, inv));
  range_report(bias_g + Net::kBiasFloats, used_ovf);
}

}  // namespace mlp
}  // namespace aon

using namespace aon;
using namespace aon::mlp;

extern "C" size_t aon_mlp_bwd_packed_bytes(void) { return NetBwdH::kPackedBytes; }

static int bwd_pack(const aon_mlp_params* prm, void* packed, aon_stream_t stream, bool bf16) {
  AON_REQUIRE(prm && packed, "null pointer");
  AON_REQUIRE(aligned16(packed), "packed buffer must be 16-byte aligned");
  if (check_mlp_params(prm, bf16 ? "aon_mlp_bwd_pack_bf16" : "aon_mlp_bwd_pack")) return -1;
  PackArgsH a{};
  const float* w[kNumLayersBwd] = {prm->rgb_w,    prm->views_w,  prm->bottleneck_w,
                                   prm->pts_w[7], prm->pts_w[6], prm->pts_w[5],
                                   prm->pts_w[4], prm->pts_w[3], prm->pts_w[2],
                                   prm->pts_w[1]};
  // row strides of the forward weights (their in-features): rgb 128, views 256 + 27, skip 256 + 63
  const int ld[kNumLayersBwd] = {128, 283, 256, 256, 256, 319, 256, 256, 256, 256};
  for (int i = 0; i < kNumLayersBwd; ++i) {
    AON_REQUIRE(w[i], "null layer weight");
    a.w[i] = w[i];
    a.ldw[i] = ld[i];
    a.tr[i] = 1;
    a.layers[i] = kLayersBwd[i];
  }
  AON_REQUIRE(prm->density_w, "null layer weight");
  a.w2[B_BOTDEN] = prm->density_w;  // segment B of d h7: density_layer^T (1 x 256)
  a.ldw2[B_BOTDEN] = 256;
  a.n_layers = kNumLayersBwd;
  a.stream_blocks = NetBwdH::kStreamBlocks;
  a.bias_floats = NetBwdH::kBiasFloats;
  a.bf16 = bf16 ? 1 : 0;
  return pack_h(a, packed, (hipStream_t)stream);
}

extern "C" int aon_mlp_bwd_pack(const aon_mlp_params* prm, void* packed, aon_stream_t stream) {
  return bwd_pack(prm, packed, stream, false);
}

extern "C" int aon_mlp_bwd_pack_bf16(const aon_mlp_params* prm, void* packed,
                                     aon_stream_t stream) {
  return bwd_pack(prm, packed, stream, true);
}

static int bwd_launch(const void* packed, const float* draw, const uint32_t* masks, int64_t N,
                      void* dzv, void* dzb, void* dz, void* work, aon_stream_t stream, bool bf16) {
  AON_REQUIRE(packed && draw && masks && dzv && dzb && dz && work, "null pointer");
  AON_REQUIRE(N >= 0, "bad shape");
  AON_REQUIRE(aligned16(packed) && aligned16(draw) && aligned16(masks) && aligned16(dzv) &&
                  aligned16(dzb) && aligned16(dz),
              "buffers must be 16-byte aligned");
  if (N == 0) return 0;
  using G1 = GeomH<1>;
  using GB = GeomH<kBfNcolBwd, true>;
  const int64_t rpb = bf16 ? GB::kRowsPerBlock : G1::kRowsPerBlock;
  const int64_t grid = (N + rpb - 1) / rpb;
  AON_REQUIRE(grid < (1ll << 31), "too many rows");
  hipStream_t st = (hipStream_t)stream;
  uint32_t* amax = static_cast<uint32_t*>(work);
  // the fp16x3 chain's per-call gradient scale (bf16 runs unscaled: no max pass)
  const int rc = bf16 ? 0 : absmax(draw, 4 * N, amax, st);
  if (rc) return rc;
  BwdArgs args{draw, reinterpret_cast<const uint2*>(masks), static_cast<float*>(dzv),
               static_cast<float*>(dzb), static_cast<float*>(dz), amax, N};
  const f4* ws = static_cast<const f4*>(packed);
  const float* bias =
      reinterpret_cast<const float*>(static_cast<const char*>(packed) + NetBwdH::kStreamBytes);
  if (bf16)
    hipLaunchKernelGGL(k_mlp_bwd_f16x3<true>, (unsigned)grid, GB::kThreads, 0, st, ws, bias, args);
  else
    hipLaunchKernelGGL(k_mlp_bwd_f16x3<false>, (unsigned)grid, G1::kThreads, 0, st, ws, bias, args);
  return launch_status(bf16 ? "aon_mlp_bwd_bf16" : "aon_mlp_bwd");
}

extern "C" int aon_absmax(const float* x, int64_t n, uint32_t* out, aon_stream_t stream) {
  AON_REQUIRE(x && out && n >= 0, "bad arguments");
  return absmax(x, n, out, (hipStream_t)stream);
}

extern "C" int aon_mlp_bwd(const void* packed, const float* draw, const uint32_t* masks,
                           int64_t N, float* dzv, float* dzb, float* dz, void* work,
                           aon_stream_t stream) {
  return bwd_launch(packed, draw, masks, N, dzv, dzb, dz, work, stream, false);
}

extern "C" int aon_mlp_bwd_bf16(const void* packed, const float* draw, const uint32_t* masks,
                                int64_t N, uint16_t* dzv, uint16_t* dzb, uint16_t* dz, void* work,
                                aon_stream_t stream) {
  return bwd_launch(packed, draw, masks, N, dzv, dzb, dz, work, stream, true);
}

// ReLU' bits of a row-major activation tensor h (N x width, width = 32 x pairs <= 256) in the
// (tiled) layout RowStoreBits writes (the layer-by-layer forward's masks for the fused chains):
// word (row, g) bit 4 t + r = h[row][16 t + 4 g + r] > 0.
__global__ void k_relu_masks(const float* __restrict__ h, int64_t N, int width,
                             uint2* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < 4 * N; i += stride) {
    const int64_t row = i >> 2;
    const int g = static_cast<int>(i & 3);
    uint32_t b[2] = {0u, 0u};
    for (int t = 0; t < width / 16; ++t)
      for (int r = 0; r < 4; ++r)
        if (h[row * width + 16 * t + 4 * g + r] > 0.0f) b[t >> 3] |= 1u << ((4 * t + r) & 31);
    out[mask_index(row, g)] = uint2{b[0], b[1]};
  }
}

extern "C" int aon_relu_masks(const float* h, int64_t N, int width, uint32_t* masks,
                              aon_stream_t stream) {
  AON_REQUIRE(h && masks, "null pointer");
  AON_REQUIRE(N >= 0 && width >= 32 && width <= 256 && width % 32 == 0, "bad shape");
  AON_REQUIRE(aligned16(masks), "masks must be 16-byte aligned");
  if (N == 0) return 0;
  hipLaunchKernelGGL(k_relu_masks, grid_for(4 * N, 256, 65536), 256, 0, (hipStream_t)stream, h, N,
                     width, reinterpret_cast<uint2*>(masks));
  return launch_status(__func__);
}
