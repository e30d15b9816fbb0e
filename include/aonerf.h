/*
 * aonerf.h -- C ABI of the MI355X (gfx950) volumetric-render hot path of
 * DJNing/articulated-object-nerf.
 *
 * Conventions (every entry point):
 *   - all tensor pointers are DEVICE pointers to contiguous row-major fp32 unless stated;
 *   - `stream` is a hipStream_t (NULL = legacy default stream); every call only enqueues work
 *     on that stream (no host synchronisation, no allocation -> graph-capturable);
 *   - return 0 on success, <0 on an invalid argument (see aon_last_error()), >0 = hipError_t;
 *   - the library never allocates: packed weights live in a caller buffer sized by
 *     aon_mlp_packed_bytes().
 *
 * Each entry point names the reference symbol it replaces (file:line in the reference tree).
 */
#ifndef AONERF_H
#define AONERF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* aon_stream_t; /* hipStream_t */

#define AON_ABI_VERSION 13 /* 13: pos_enc's sin and the alpha exp correctly rounded, sigmoid as
                            * torch's CPU kernel forms it; the 32x32x16 precision of ABI 12
                            * (value 3) withdrawn: measured slower */

/* Precision of the MLP GEMMs (see DESIGN.md "MLP precision modes"). */
#define AON_PREC_FP32 0  /* exact fp32 MFMA (v_mfma_f32_16x16x4_f32) */
#define AON_PREC_F16X3 1 /* fp16 hi/lo split, 3 products (hi*hi + hi*lo + lo*hi) per weight on
                            v_mfma_f32_16x16x32_f16, fp32 accumulate: ~22-bit operands */
#define AON_PREC_BF16 2  /* bf16 operands, 1 product per weight (v_mfma_f32_16x16x32_bf16), fp32
                         * accumulate: the training step's bf16 mode (BASELINE config C5) --
                         * aon_mlp_fwd_train_bf16 / aon_mlp_bwd_bf16 / aon_gemm with bf16 operands */

/* Output activation applied by the compositor (reference model.py:186-187,
 * model_autodecoder.py:321-323). */
#define AON_ACT_NONE 0    /* inputs are already activated (volumetric_rendering API) */
#define AON_ACT_VANILLA 1 /* rgb = sigmoid(raw), sigma = relu(raw) */
#define AON_ACT_ARTIC 2   /* rgb = sigmoid(raw)*1.002-0.001, sigma = softplus(raw-1) */

int aon_abi_version(void);
const char* aon_last_error(void); /* thread-local message of the last failing call */

/* ---------------------------------------------------------------- ray generation */
/* get_ray_directions (datasets/ray_utils.py:71-90): dirs (H*W, 3). */
int aon_ray_directions(int H, int W, float focal, float* dirs, aon_stream_t stream);

/* get_rays (datasets/ray_utils.py:118-159): rays_d = normalize(dirs @ c2w[:, :3]^T),
 * rays_o = c2w[:, 3].  c2w_host: 12 floats (3x4 row-major) in HOST memory.  viewdirs may be
 * NULL (it equals rays_d in the reference, ray_utils.py:146-147).  radii may be NULL; when
 * given, dirs must be a full (H, W, 3) grid (ray_utils.py:138-143). */
int aon_get_rays(const float* dirs, int64_t n, const float* c2w_host, float* rays_o,
                 float* rays_d, float* viewdirs, int H, int W, float* radii,
                 aon_stream_t stream);

/* get_ray_directions + get_rays fused (no dirs tensor materialised) for the n pixels
 * p0 .. p0+n-1 (row-major) of an H x W frame -- a contiguous band of an image tile shard. */
int aon_frame_rays(int H, int W, float focal, const float* c2w_host, int64_t p0, int64_t n,
                   float* rays_o, float* rays_d, float* viewdirs, aon_stream_t stream);

/* ---------------------------------------------------------------- sampling */
/* sample_along_rays + cast_rays (models/vanilla_nerf/helper.py:106-133, 25-26).
 * t_lower/t_upper: S-entry device tables built exactly as helper.py:116-125 builds them.
 * Randomized iff u != NULL: t = t_lower + (t_upper - t_lower) * u[b, s] with t_lower/t_upper
 * the strata bounds; eval (u == NULL): t = t_lower, which must then be the schedule itself.
 * xyz may be NULL. */
int aon_sample_along_rays(const float* rays_o, const float* rays_d, int64_t B, int S,
                          const float* t_lower, const float* t_upper, const float* u,
                          float* t_out, float* xyz_out, aon_stream_t stream);

/* Ray batches from a device-resident dataset (datasets/sapien.py:84-113, 131-154;
 * sapien_multi.py:196-238): poses (N, 3, 4) camera-to-world, images (N, H, W, C) uint8.
 * For each of n flat indices g = image*H*W + pixel (idx == NULL: g = 0 .. n-1) writes the
 * pixel's ray (as aon_frame_rays) and, when target != NULL, its target rgb:
 * mode 0 u8/255; mode 1 RGBA alpha-blended onto white; mode 2 channel 3 is a segmentation
 * mask, background pixels take `bg`. */
int aon_sample_rays(const float* poses, const uint8_t* images, int C, int64_t N, int H, int W,
                    float focal, const int64_t* idx, int64_t n, int mode, float bg,
                    float* rays_o, float* rays_d, float* viewdirs, float* target,
                    aon_stream_t stream);

/* cast_rays (helper.py:25-26) on per-ray sample positions t (B, S): x = o + t d, then, when
 * offset != NULL, x = offset[r] + x (the articulated deformation, model_autodecoder.py:205);
 * rays_d == NULL (t ignored): x = rays_o[r / S] (points given directly);
 * writes xyz (B*S, 3) and/or enc = pos_enc(x, min_deg, max_deg) (B*S, 3 + 6 (max - min)). */
int aon_cast_rays(const float* rays_o, const float* rays_d, const float* t, int64_t B, int S,
                  const float* offset, int64_t offset_stride, float* xyz, int min_deg,
                  int max_deg, float* enc, aon_stream_t stream);

/* cast_rays + pos_enc as above (no offset, no xyz), written in the fused training kernels'
 * tiled layout (aon_mlp_fwd_train) with `width` columns (a multiple of 16), the ones past
 * 3 + 6 (max - min) zero: enc holds B*S rounded up to 16 rows (rows past B*S not written).  The
 * parity mode's pos_enc(x) copy for the enc-column weight gradients (ABI 10). */
int aon_cast_rays_tiled(const float* rays_o, const float* rays_d, const float* t, int64_t B, int S,
                        int min_deg, int max_deg, int width, float* enc, aon_stream_t stream);

/* pos_enc (helper.py:136-140): out (n, 3 + 6*(max_deg-min_deg)). */
int aon_pos_enc(const float* x, int64_t n, int min_deg, int max_deg, float* out,
                aon_stream_t stream);

/* sorted_piecewise_constant_pdf + sample_pdf (helper.py:203-252).
 *   bins:    (B, nb) with row stride bins_stride, or NULL -> bins = 0.5*(t[k+1]+t[k]) of
 *            t_merge (the caller at models/vanilla_nerf/model.py:163);
 *   weights: (B, nb-1) with row stride w_stride (e.g. coarse weights + 1, stride Sc);
 *   u:       (B, Ns) with row stride u_stride (u_stride 0 = one shared row, eval mode);
 *   t_merge: (B, Nt) sorted, or NULL;
 *   out:     t_merge ? sorted(cat[t_merge, samples]) (B, Nt+Ns) : samples (B, Ns);
 *   xyz:     NULL or (B, Nt+Ns, 3) = o + t*d (needs rays_o/rays_d).
 * Limits: 2 <= nb <= 256, 1 <= Ns <= 512, Nt <= 512. */
int aon_sample_pdf(const float* bins, int64_t bins_stride, const float* weights,
                   int64_t w_stride, int64_t B, int nb, int Ns, const float* u,
                   int64_t u_stride, const float* t_merge, int Nt, const float* rays_o,
                   const float* rays_d, float* out, float* xyz, aon_stream_t stream);

/* The coarse level's volumetric_rendering (helper.py:157-195) fused with the resampling that
 * consumes its weights (model.py:163-172: sample_pdf on the mids of t and weights[..., 1:-1],
 * merged with t; helper.py:203-252) -- one kernel, the coarse weights stay on chip.
 *   raw:     (B*S, 4) [r, g, b, sigma], 16-byte aligned (aon_mlp_fwd's output), act as in
 *            aon_composite_fwd; t: (B, S) sorted; dirs: (B, 3) rays_d;
 *   u:       (B, Ns) with row stride u_stride (0 = one shared row, eval mode);
 *   outputs: comp_rgb (B, 3), acc, depth (B), weights (B, S) or NULL, and
 *            t_fine = sorted(cat[t, samples]) (B, S + Ns).
 * Equal, bit for bit, to aon_composite_fwd followed by aon_sample_pdf(bins = NULL, weights + 1,
 * t_merge = t).  Limits: 3 <= S <= 256, 1 <= Ns <= 256. */
int aon_composite_march(const float* raw, const float* t, const float* dirs, int64_t B, int S,
                        int white_bkgd, int act, const float* u, int64_t u_stride, int Ns,
                        float* comp_rgb, float* acc, float* weights, float* depth, float* t_fine,
                        aon_stream_t stream);

/* ---------------------------------------------------------------- MLP */
/* Device pointers to one NeRFMLP's nn.Linear parameters in torch layout ([out][in]),
 * models/vanilla_nerf/model.py:39-93 with the default geometry (min_deg_point 0,
 * max_deg_point 10, deg_view 4, netdepth 8, netwidth 256, skip 4, 1 x 128 view layer). */
typedef struct aon_mlp_params {
  const float* pts_w[8];
  const float* pts_b[8];
  const float* density_w;
  const float* density_b;
  const float* bottleneck_w;
  const float* bottleneck_b;
  const float* views_w;
  const float* views_b;
  const float* rgb_w;
  const float* rgb_b;
  /* Shapes of the tensors above (ABI 9), in layer order pts_linears.0..7, density_layer,
   * bottleneck_layer, views_linear.0, rgb_layer (the order of the fields): layer i's weight is
   * w_rows[i] x w_cols[i] ([out][in], contiguous) and its bias b_len[i] floats.  Every pack
   * (aon_mlp_pack, aon_mlp_bwd_pack[_bf16]) checks them against the default geometry --
   * 256x63, 4 x 256x256, 256x319, 2 x 256x256, 1x256, 256x256, 128x283, 3x128 -- and returns
   * < 0 before any launch on a mismatch (e.g. parameters passed in registration order), instead
   * of reading past the end of a tensor. */
  int64_t w_rows[12], w_cols[12], b_len[12];
} aon_mlp_params;

size_t aon_mlp_packed_bytes(int precision);
/* Re-lay the parameters into the MFMA-tiled weight stream consumed by aon_mlp_fwd. */
int aon_mlp_pack(const aon_mlp_params* params, int precision, void* packed,
                 aon_stream_t stream);

/* fp16x3 range guard.  Every packed buffer (aon_mlp_pack, aon_mlp_art_pack, the backward-chain
 * packs) ends in a 16-byte status block that the pack zeroes.  A fp16x3 kernel that met a value
 * its fp16 hi/lo split cannot hold (|activation| > 8188, or a gradient past 65504 at its
 * per-call scale) sets status word 0 to 1: the outputs of that launch are invalid; the pack
 * itself sets it to 2 when a weight's scaled fp16 hi part is not finite (|w| > 1023 at the
 * 2^6 weight scale, or a NaN/inf parameter): every launch reading that stream is invalid.  The
 * block stays set until the next pack (sticky across launches).  aon_mlp_read_status copies word 0
 * to *status (host) and synchronises the stream; packed_bytes is the size the *_packed_bytes
 * query returned.  (The fp32 MFMA path has no such limit and never sets it.) */
int aon_mlp_read_status(const void* packed, size_t packed_bytes, uint32_t* status,
                        aon_stream_t stream);

/* NeRFMLP.forward (model.py:95-120) fused with cast_rays + pos_enc (model.py:175-181):
 * per sample row r = b*S + s: xyz = o[b] + t[r]*d[b], enc = pos_enc(xyz, 0, 10),
 * venc = pos_enc(viewdirs[b], 0, 4); out (B*S, 4) = [rgb(3), sigma].
 * act = AON_ACT_NONE: the raw head outputs (NeRFMLP.forward);
 * act = AON_ACT_VANILLA: also rgb_activation / sigma_activation (sigmoid / relu,
 *       model.py:186-187), so the compositor can run with AON_ACT_NONE;
 * act = AON_ACT_ARTIC: the articulated model's padded sigmoid / softplus(x - 1). */
int aon_mlp_fwd(const void* packed, int precision, const float* rays_o, const float* rays_d,
                const float* viewdirs, const float* t, int64_t B, int S, int act, float* out,
                aon_stream_t stream);

/* (ABI 9: no process-global state and no environment knobs.  ABI 8's aon_mlp_set_dataflow is
 * gone: the weight-streamed render dataflow, bit-identical and measured at parity, is an A/B
 * variant library, `make -C csrc variant-ws` -> lib/variants/libaonerf_ws.so, whose aon_mlp_fwd
 * and aon_mlp_art_fwd run it.) */

/* NeRFMLP.forward on pre-encoded inputs: x (B*S, 63), condition (B, 27) -> out (B*S, 4). */
int aon_mlp_fwd_encoded(const void* packed, int precision, const float* x,
                        const float* condition, int64_t B, int S, int act, float* out,
                        aon_stream_t stream);

/* Kept tensors of the fused training kernels (activations, ReLU' bits, the backward chains'
 * pre-activation gradients) are stored TILED, in contiguous row-major 16 x 16 tiles (one MFMA
 * output fragment each): for N rows of width W (a multiple of 16), element (row, f) at
 *     (row / 16) * 16 W + 256 (f / 16) + 16 (row % 16) + f % 16,
 * and a layer's ReLU' word (row, g) (a pair of uint32) at (row / 16) * 64 + 16 g + row % 16.
 * Every buffer holds NR = N rounded up to a multiple of 16 rows, and stacked tensors such as
 * h (8, NR, 256) are NR rows apart.  aon_gemm reads them in place (a_tiled / b_tiled).
 *
 * The training forward of one level (model.py:175-184 under autograd) on the fused fp16x3
 * kernel: as aon_mlp_fwd with AON_ACT_NONE (packed = AON_PREC_F16X3 stream), plus every
 * hidden activation kept for the backward (tiled, NR = B*S rounded up to 16 rows) -- h (8, NR,
 * 256): post-ReLU pts_linears.0..7, bot (NR, 256): bottleneck_layer, hv (NR, 128): post-ReLU
 * views_linear.0 -- and raw_sigma + noise[row] when noise (B*S) is not NULL.  masks (9, NR, 4) pairs of uint32:
 * the ReLU' bits of h0..h7, hv for the backward chain (word (row, g), bit 4 t + r = output
 * feature 16 t + 4 g + r > 0; aon_relu_masks builds the same from stored activations). */
int aon_mlp_fwd_train(const void* packed, const float* rays_o, const float* rays_d,
                      const float* viewdirs, const float* t, int64_t B, int S, const float* noise,
                      float* h, float* bot, float* hv, float* raw, uint32_t* masks,
                      aon_stream_t stream);

/* The same training forward in the bf16 mode: packed = an AON_PREC_BF16 stream; one bf16
 * MFMA per weight product (fp32 accumulate, activations rounded to bf16 between layers) and
 * the kept activations h / bot / hv stored as bf16 (raw bits, same shapes): half the bytes of
 * the fp32 stores, and exactly the operands the next layer consumed.  enc (optional, NULL:
 * not kept): pos_enc(x) as bf16 in the same tiled layout, (NR, 128), columns 63..127 zero --
 * the B operand of pts_linears.0's and the skip layer's enc-column weight gradients (aon_gemm
 * with n_store = 63), so no separate encoding pass. */
int aon_mlp_fwd_train_bf16(const void* packed, const float* rays_o, const float* rays_d,
                           const float* viewdirs, const float* t, int64_t B, int S,
                           const float* noise, uint16_t* h, uint16_t* bot, uint16_t* hv,
                           float* raw, uint32_t* masks, uint16_t* enc, aon_stream_t stream);

/* ReLU' bits of a ROW-MAJOR activation tensor h (N x width, width a multiple of 32 up to 256)
 * in the tiled layout of aon_mlp_fwd_train's masks (NR, 4) pairs of uint32 -- for the fused backward chains
 * after a layer-by-layer forward (threshold_backward of model.py:95-120's ReLUs). */
int aon_relu_masks(const float* h, int64_t N, int width, uint32_t* masks, aon_stream_t stream);

/* out = the bits of max |x| over n floats (one uint32 of device memory): the per-call gradient
 * scale word aon_gemm's a_amax takes (the layer-by-layer backward scales each dY by it, as the
 * fused chains scale theirs by max |d raw|). */
int aon_absmax(const float* x, int64_t n, uint32_t* out, aon_stream_t stream);

/* Backward chain of one level's NeRFMLP for the training step (model.py:95-120 under
 * autograd): from draw (B*S, 4) = dL/d[raw_rgb, raw_sigma] (aon_composite_bwd), all input-
 * gradient products dX = dZ W down to pts_linears.0 in one fused kernel, each masked by ReLU'
 * of the forward output it flows into (masks: the ReLU' bits of aon_mlp_fwd_train), writing
 *   dzv (NR, 128): dL/d pre-activation of views_linear.0,
 *   dzb (NR, 256): dL/d bottleneck_layer output,
 *   dz  (8, NR, 256): dL/d pre-activation of pts_linears.i (all tiled, NR = N rounded up to 16),
 * the operands of the weight-gradient GEMMs dW = dZ^T X (aon_gemm).  packed: the transposed
 * weight stream of aon_mlp_bwd_pack (re-pack after every optimizer step); work: >= 4 bytes
 * of device scratch. */
size_t aon_mlp_bwd_packed_bytes(void);
int aon_mlp_bwd_pack(const aon_mlp_params* params, void* packed, aon_stream_t stream);
/* bf16 training mode: the transposed stream with bf16 weights, and the chain on bf16 MFMAs
 * writing dzv / dzb / dz as bf16 (raw bits, same shapes); draw and masks as aon_mlp_bwd. */
int aon_mlp_bwd_pack_bf16(const aon_mlp_params* params, void* packed, aon_stream_t stream);
int aon_mlp_bwd_bf16(const void* packed, const float* draw, const uint32_t* masks, int64_t N,
                     uint16_t* dzv, uint16_t* dzb, uint16_t* dz, void* work, aon_stream_t stream);
int aon_mlp_bwd(const void* packed, const float* draw, const uint32_t* masks, int64_t N,
                float* dzv, float* dzb, float* dz, void* work, aon_stream_t stream);

/* ---------------------------------------------------------------- articulated MLP */
/* Device pointers to one articulated NeRFMLP's nn.Linear parameters in torch layout
 * (models/vanilla_nerf/model_autodecoder.py:60-166, default geometry: 4 x 128 deformation
 * layers, 8 x 256 trunk with skip 4, 4 x 128 view layers).  The latent columns of
 * deformations_linear.0 (after the 3 xyz columns), pts_linears.0 (after 63 enc columns),
 * pts_linears.5 (after 256 + 63) and views_linear.0 (after 256 + 27) are NOT read: the caller
 * passes biases with the latent products folded in (b + W[:, latent] . code, the code being
 * the same for every sample), and each such weight's row stride (ld_*). */
typedef struct aon_mlp_art_params {
  const float* def_w[4];
  const float* def_b[4];
  const float* deformation_w;
  const float* deformation_b;
  const float* pts_w[8];
  const float* pts_b[8];
  const float* density_w;
  const float* density_b;
  const float* bottleneck_w;
  const float* bottleneck_b;
  const float* views_w[4];
  const float* views_b[4];
  const float* rgb_w;
  const float* rgb_b;
  /* Shapes (ABI 9; replaces ABI 8's ld_def0 / ld_pts0 / ld_pts5 / ld_view0), in layer order
   * deformations_linear.0..3, deformation_layer, pts_linears.0..7, density_layer,
   * bottleneck_layer, views_linear.0..3, rgb_layer (the order of the fields): layer i's weight
   * is w_rows[i] x w_cols[i] ([out][in], contiguous: w_cols is its row stride) and its (folded)
   * bias b_len[i] floats (b_len = w_rows).  The packs check them against the default geometry
   * and return < 0 before any launch on a mismatch: rows 4 x 128, 3, 8 x 256, 1, 256, 4 x 128,
   * 3; columns exactly 128 (deformations_linear.1-3, deformation_layer, views_linear.1-3,
   * rgb_layer) or 256 (pts_linears.1-4, 6-7, density, bottleneck) for the layers without latent
   * columns, and at least the per-sample columns -- 3 (deformations_linear.0), 63
   * (pts_linears.0), 319 (pts_linears.5), 283 (views_linear.0) -- for the four that carry them. */
  int64_t w_rows[20], w_cols[20], b_len[20];
} aon_mlp_art_params;

size_t aon_mlp_art_packed_bytes(void);
/* Re-lay the parameters (folded biases included) into the fp16x3 weight stream. */
int aon_mlp_art_pack(const aon_mlp_art_params* params, void* packed, aon_stream_t stream);

/* The articulated NeRFMLP.forward (model_autodecoder.py:168-239) fused with cast_rays and
 * both pos_encs: per sample row r = b*S + s, xyz = o[b] + t[r]*d[b]; deformation MLP;
 * enc = pos_enc(deformation + xyz, 0, 10); venc = pos_enc(viewdirs[b], 0, 4);
 * out (B*S, 4) = [rgb(3), sigma], raw (AON_ACT_NONE) or with the articulated activations
 * (AON_ACT_ARTIC: padded sigmoid, softplus(x - 1), model_autodecoder.py:321-323). */
int aon_mlp_art_fwd(const void* packed, const float* rays_o, const float* rays_d,
                    const float* viewdirs, const float* t, int64_t B, int S, int act, float* out,
                    aon_stream_t stream);
/* Training forward of one articulated level (reference model_autodecoder.py:168-239 under
 * autograd): aon_mlp_art_fwd (MODE 0 inputs, raw outputs, no activation) that also keeps what
 * the backward needs -- tiled (NR = B*S rounded up to 16): hd (4, NR, 128) deformation layers,
 * h (8, NR, 256) pts_linears, bot (NR, 256), hv (4, NR, 128) views_linear, enc (NR, 64) =
 * pos_enc(x') (column 63 zero; ABI 11 -- row-major (B*S, 63) before); row-major: xyz (B*S, 3)
 * the sample points; raw_sigma += noise[r] when noise != NULL (:318-319); masks (16, NR, 4)
 * pairs of uint32: the ReLU' bits of hd0..3, h0..7, hv0..3 (layout of aon_mlp_fwd_train's).
 * Activation buffers 8-byte aligned, raw, enc and masks 16-byte aligned. */
int aon_mlp_art_fwd_train(const void* packed, const float* rays_o, const float* rays_d,
                          const float* viewdirs, const float* t, int64_t B, int S,
                          const float* noise, float* hd, float* h, float* bot, float* hv,
                          float* enc, float* xyz, float* raw, uint32_t* masks,
                          aon_stream_t stream);
/* The articulated bf16 training mode (train_art.PRECISION = "bf16"; BASELINE config C5's
 * "bf16" on the articulated model): hd, h, bot, hv are bf16 arrays of the shapes above, xyz /
 * raw / masks as above, enc (NR, 16) fp32 tiled: pos_enc(x') columns 0..15 only (x' = columns
 * 0..2, all the chain reads; ABI 11).  mixed != 0: packed by aon_mlp_art_pack_bf16 (a mixed stream in
 * the same buffer size: the deformation MLP stays fp16x3 -- x' feeds sin(2^9 x') -- the trunk,
 * heads and view branch are bf16), one bf16 MFMA per product past the deformation head;
 * mixed == 0: packed by aon_mlp_art_pack, fp16x3 numerics throughout (only the stores bf16).
 * mixed == 2: packed by aon_mlp_art_pack_mixed(.., 2, ..) -- everything through the bottleneck
 * fp16x3, the view branch (views_linear.0-3, rgb_layer) one bf16 MFMA per product.
 * mixed == 3: packed by aon_mlp_art_pack_mixed(.., 3, ..) -- the deformation MLP fp16x3, every
 * later layer two fp16 MFMAs per product: the weights rounded once to fp16 (at 2^6), the
 * activations split exactly into fp16 hi + lo as in fp16x3 (range-guarded likewise).
 * mixed == 4: packed by aon_mlp_art_pack (the fp16x3 stream) -- the deformation MLP fp16x3,
 * every later layer two fp16 MFMAs per product, (hi(W) + lo(W)) x hi(x): the weights' exact
 * split kept, the activations rounded once to fp16 (range-guarded as the hi parts).
 * enc_bf (required since ABI 11, 16-byte aligned): pos_enc(x') as bf16, tiled (NR, 128),
 * columns 63..127 zero (as aon_mlp_fwd_train_bf16's enc) -- the enc-column weight gradients'
 * operand. */
int aon_mlp_art_pack_bf16(const aon_mlp_art_params* params, void* packed, aon_stream_t stream);
/* mixed = 1: as aon_mlp_art_pack_bf16; mixed = 2: the view-branch stream; mixed = 3: the
 * fp16-weight stream (ABI 9). */
int aon_mlp_art_pack_mixed(const aon_mlp_art_params* params, int mixed, void* packed,
                           aon_stream_t stream);
int aon_mlp_art_fwd_train_bf16(const void* packed, const float* rays_o, const float* rays_d,
                               const float* viewdirs, const float* t, int64_t B, int S,
                               const float* noise, void* hd, void* h, void* bot, void* hv,
                               float* enc, float* xyz, float* raw, uint32_t* masks,
                               void* enc_bf, int mixed, aon_stream_t stream);

/* Backward chain of one articulated level (autograd of model_autodecoder.py:168-239): from
 * dL/d raw (N, 4), the ReLU' bits (16, N, 4) of hd0..3, h0..7, hv0..3 and the tiled pos_enc(x')
 * (enc, (NR, 64); the bf16 chain: aon_mlp_art_fwd_train_bf16's (NR, 16)) kept by
 * aon_mlp_art_fwd_train, to
 * every layer's dL/d pre-activation -- tiled (NR rows): dzv (4, NR, 128) views_linear.i, dbot
 * (NR, 256) the bottleneck output, dz (8, NR, 256) pts_linears.i, dzd (4, NR, 128)
 * deformations_linear.i; row-major dxp (N, 3) = dL/dx' (the deformation head's output, through
 * pos_enc's backward) -- the operands of
 * the weight-gradient GEMMs.  packed: aon_mlp_art_bwd_pack of the forward weights (layout
 * kLayersArtBwd); work: >= 4 bytes.  Buffers 16-byte aligned (dxp: 4). */
size_t aon_mlp_art_bwd_packed_bytes(void);
int aon_mlp_art_bwd_pack(const aon_mlp_art_params* params, void* packed, aon_stream_t stream);
int aon_mlp_art_bwd(const void* packed, const float* draw, const uint32_t* masks,
                    const float* enc, int64_t N, float* dzv, float* dbot, float* dz, float* dxp,
                    float* dzd, void* work, aon_stream_t stream);
/* bf16 mode: the whole chain one bf16 MFMA per product on aon_mlp_art_bwd_pack_bf16's compact
 * stream (same buffer size); dzv, dbot, dz, dzd are bf16 arrays of the shapes above, dxp fp32. */
int aon_mlp_art_bwd_pack_bf16(const aon_mlp_art_params* params, void* packed, aon_stream_t stream);
int aon_mlp_art_bwd_bf16(const void* packed, const float* draw, const uint32_t* masks,
                         const float* enc, int64_t N, void* dzv, void* dbot, void* dz, float* dxp,
                         void* dzd, void* work, aon_stream_t stream);

/* The same on given sample points pos (B*S, 3) and encoded view directions condition (B, 27)
 * (NeRFMLP.forward(pos, condition, latents)). */
int aon_mlp_art_fwd_points(const void* packed, const float* pos, const float* condition,
                           int64_t B, int S, int act, float* out, aon_stream_t stream);

/* ---------------------------------------------------------------- compositing */
/* volumetric_rendering (helper.py:157-195) with the activations of model.py:186-187.
 * rgb: (B*S) rows of rgb_stride floats (3 = API tensor, 4 = fused raw buffer);
 * sigma: (B*S) rows of sigma_stride floats.  weights may be NULL. */
int aon_composite_fwd(const float* rgb, int64_t rgb_stride, const float* sigma,
                      int64_t sigma_stride, const float* t, const float* dirs, int64_t B,
                      int S, int white_bkgd, int act, float* comp_rgb, float* acc,
                      float* weights, float* depth, aon_stream_t stream);

/* ---------------------------------------------------------------- evaluation */
/* Per-image mean squared error of n_images images of `pixels` rgb pixels ((n, P, 3) fp32):
 * clip = 1 clips both sides to [0, 1] first (psnr_each, models/interface.py:54-62);
 * mask (n, P) uint8 != NULL restricts to the masked pixels (the object PSNR of
 * get_obj_rgbs_from_segmap, models/utils.py:102-109).  psnr (may be NULL) = -10 ln(mse)/ln 10. */
int aon_image_mse(const float* pred, const float* gt, int64_t n_images, int64_t pixels,
                  const uint8_t* mask, int clip, float* mse, float* psnr, aon_stream_t stream);

/* to8b (models/utils.py:12-13): out = uint8(255 * clip(x, 0, 1)) (truncating cast). */
int aon_to8b(const float* x, int64_t n, uint8_t* out, aon_stream_t stream);

/* ---------------------------------------------------------------- training path */
/* C (M x N) = epilogue(A (M x K) . B (K x N)): fp32 operands, fp16-MFMA hi/lo split
 * (fp32-class accuracy), the building block of the layer-by-layer training forward
 * (model.py:95-120 with activations kept) and of its autograd backward (model.py:256-282):
 *   A: a_kc = 1 -> element (m, k) = A[m*lda + k] for k < K1, and, when A2 != NULL,
 *                  A2[(m / a2_rdiv)*lda2 + (k - K1)] for k >= K1 (cat[h, enc] of model.py:102,
 *                  cat[bottleneck, enc_dir tiled over samples] of model.py:110-112);
 *      a_kc = 0 -> element (m, k) = A[k*lda + m] (dY^T of a weight gradient).
 *   B: b_kc = 1 -> element (k, n) = B[n*ldb + k] (nn.Linear weight [out][in]: x . W^T);
 *      b_kc = 0 -> element (k, n) = B[(k / b_rdiv)*ldb + n] (W for dX = dY . W; X for
 *                  dW = dY^T . X; b_rdiv = S broadcasts a per-ray row over its S samples).
 *   epilogue per element, in this order: v = sum / (a_scale * b_scale); v += C[m*ldc+n] when
 *   accumulate; v += bias[n]; relu; v *= (mask[m*ldm+n] > 0).  a_scale / b_scale are
 *   power-of-two operand prescales that keep |x * scale| < 65504 (fp16 range of the hi part).
 *   rowsum (optional, a_kc = 0 only): rowsum[m] = sum_k A(m, k) -- the bias gradient
 *   sum_rows dY that accompanies the weight gradient dY^T . X, from the same operand pass.
 *   Long reductions (K of a weight gradient = rows) are split over workgroups into
 *   `work` (aon_gemm_workspace_bytes) and summed in a fixed order (deterministic).
 *   k_splits = 0 chooses the split automatically. */
typedef struct aon_gemm_args {
  int64_t M, N, K;
  const float* A;
  int64_t lda;
  int a_kc;
  const float* A2;
  int64_t lda2, K1, a2_rdiv;
  const float* B;
  int64_t ldb;
  int b_kc;
  int64_t b_rdiv;
  float* C;
  int64_t ldc;
  const float* bias;
  const float* mask;
  int64_t ldm;
  int relu, accumulate;
  float a_scale, b_scale;
  int64_t k_splits;
  float* rowsum;
  /* optional (device): bits of max |A| (the word aon_mlp_bwd / aon_mlp_art_bwd leave in their
   * work buffer, or any k_absmax result); A is then also scaled by 2^(8 - e) for max = m 2^e,
   * m in [0.5, 1) -- the backward chains' own per-call gradient scale, so small gradients keep
   * full fp16 hi/lo precision.  NULL: a_scale alone. */
  const uint32_t* a_amax;
  /* bf16 mode (AON_PREC_BF16 training): mma_bf16 = 1 computes on one bf16 MFMA per product
   * (operands rounded to bf16 while staged, fp32 accumulate) -- reduction-major operands only
   * (a_kc = b_kc = 0: the weight gradients dW = dY^T X), no A2 / bias / mask / relu; a_bf16 /
   * b_bf16 = 1: that operand's elements are bf16 (raw 16-bit), else fp32. */
  int mma_bf16, a_bf16, b_bf16;
  /* a reduction-major operand stored in the fused training kernels' tiled layout (see
   * aon_mlp_fwd_train): a_tiled needs lda == M, b_tiled ldb == N and b_rdiv 1, both widths
   * multiples of 16 */
  int a_tiled, b_tiled;
  /* columns of C written (0: all N): a B zero-padded to whole 128-column tiles (the bf16 mode's
   * pos_enc copy, 63 -> 128 columns) updates only the real columns of dW; n_store < N on the
   * bf16 LDS-DMA path (both operands bf16, M and N multiples of 128) and on fp32 products
   * (the parity mode's 64-column pos_enc copy, aon_cast_rays_tiled; ABI 10) */
  int64_t n_store;
  /* exact_fp32 = 1: compute in exact fp32 fmaf instead of the fp16x3 MFMA split, in a fixed
   * (deterministic) order: K <= 16 one fma chain in k order per output; K > 16 one wave per
   * output, lane-strided partial chains (lane l sums k = l, l + 64, ...) combined by a fixed
   * xor-butterfly -- not k order -- tiny products only (M N <= 65536, K <= 1024, no A2 / mask / relu / rowsum /
   * a_amax / tiled operands): the bf16 training mode's latent-code terms, which the 128 x 128
   * tiled kernel ran at 17-27 us each */
  int exact_fp32;
  /* c_trans = 1: C is written transposed -- element (m, n) of the product at C[n * ldc + m] --
   * and rowsum receives the column sums of B (N entries, in B's element type rounded as staged)
   * instead of the row sums of A: dW of a layer whose input has <= 4 columns, computed as the
   * skinny product (input)^T dZ.  The skinny path only (M <= 4, below). */
  int c_trans;
  /* f16_single = 1 (ABI 10): licence for the single-accumulator fp16x3 kernel -- hi*hi + hi*lo +
   * lo*hi in ONE fp32 accumulator, the lo parts unscaled (normal fp16 for |x s| >= 2^-3, an
   * absolute 2^-25 at scale below) -- where the caller guarantees |A a_scale| (times a_amax's
   * scale) and |B b_scale| below 65504: the parity-mode weight gradients dW = dY^T X of the fused
   * kernels' tiled tensors, dY at the backward chain's own scale (a_amax) and X at b_scale 8 (the
   * forward's activation scale: both kernels range-guard their splits at exactly these scales).
   * Used for 256 x 256 products with both operands tiled, fp32, K >= 8192 (k_gemm_f1_256, one
   * 256 x 256 tile per workgroup); any other product computes as with f16_single = 0. */
  int f16_single;
} aon_gemm_args;

/* Weight gradients (a_kc = b_kc = 0, no A2 / bias / mask / relu) with M <= 4 rows (B of <= 256
 * columns, 16-B aligned, a row-major A), or against a per-ray B (b_rdiv > 1, M a multiple of 8
 * up to 256), compute without the fp16x3 split when mma_bf16 = 0: fp32 products and sums in a
 * fixed order (the streaming skinny / segment-sum kernels; a_scale, b_scale and a_amax then
 * only cancel). */
size_t aon_gemm_workspace_bytes(const aon_gemm_args* args);
int aon_gemm(const aon_gemm_args* args, void* work, size_t work_bytes, aon_stream_t stream);

/* `count` (<= AON_GEMM_BATCH_MAX) independent aon_gemm products (no product reads what another
 * writes), stream-ordered, with one workspace: one level's bf16 weight gradients, the loop of
 * LitNeRF.training_step's backward (model.py:256-282).  The bf16 256 x 256 products (mma_bf16,
 * both operands bf16, M = N = 256, k_splits 0, equal K >= 8192: pts_linears / bottleneck) run
 * as ONE launch of count x (256 / count) K chunks and one split-K reduce -- count times fewer
 * fp32 partials than count launches; the other bf16 products in whole 128 x 128 tiles
 * (views_linear.0, the enc columns) likewise as one launch, the fp16x3 weight gradients (fp32
 * reduction-major operands in whole 128 x 128 tiles, no A2 / bias / mask / relu) as one more;
 * the rest one by one as aon_gemm.
 * Deterministic; the chunking, and so the fp32 summation order, differs from aon_gemm's. */
#define AON_GEMM_BATCH_MAX 12
size_t aon_gemm_batch_workspace_bytes(const aon_gemm_args* args, int count);
int aon_gemm_batch(const aon_gemm_args* args, int count, void* work, size_t work_bytes,
                   aon_stream_t stream);

/* `count` (<= AON_GEMM_SMALL_BATCH_MAX) exact_fp32 tiny products (each valid for aon_gemm's
 * exact_fp32 path) in ONE launch, bit for bit what the launches in argument order give: products
 * writing the same C (same M, N, ldc, and accumulate = 1 after the first) are applied in argument
 * order; any other two products must not touch each other's output (checked, < 0 otherwise).
 * The articulated training step's latent-code terms (model_autodecoder.py:186-194: dW of the
 * latent columns = db l^T, dl = db^T W_l, three terms summed into the shape code's gradient) and
 * the per-call folded biases of its forward.  No workspace. */
#define AON_GEMM_SMALL_BATCH_MAX 16
int aon_gemm_small_batch(const aon_gemm_args* args, int count, aon_stream_t stream);

/* Backward of volumetric_rendering (helper.py:157-195) and of the activations `act` applied to
 * the raw MLP outputs (model.py:186-187): given dL/dcomp_rgb (B,3) and optionally dL/dacc,
 * dL/ddepth (B,), writes dL/draw_rgb (3 floats at d_rgb + r*d_stride) and dL/draw_sigma
 * (d_sigma + r*d_stride) for every sample row r.  Inputs as aon_composite_fwd (raw values). */
int aon_composite_bwd(const float* rgb, int64_t rgb_stride, const float* sigma,
                      int64_t sigma_stride, const float* t, const float* dirs, int64_t B, int S,
                      int white_bkgd, int act, const float* g_rgb, const float* g_acc,
                      const float* g_depth, float* d_rgb, float* d_sigma, int64_t d_stride,
                      aon_stream_t stream);

/* img2mse (helper.py:17-18): *loss = mean((pred - target)^2) over n values and
 * grad = grad_scale * 2 (pred - target) / n (either output may be NULL). */
int aon_mse(const float* pred, const float* target, int64_t n, float grad_scale, float* loss,
            float* grad, aon_stream_t stream);

/* The training step's loss terms in one launch (LitNeRF.training_step, model.py:265-270;
 * LitNeRF_AutoDecoder.training_step, model_autodecoder.py:455-470): the coarse (pred0) and fine
 * (pred1) img2mse against one target, each with aon_mse's arithmetic; out[0] = loss1 + loss0
 * (+ *extra when extra != NULL: the latent regulariser), out[1] = loss0, out[2] = loss1;
 * grad0 / grad1 (may be NULL) = 2 (pred - target) / n. */
int aon_loss_pair(const float* pred0, const float* pred1, const float* target, int64_t n,
                  const float* extra, float* out, float* grad0, float* grad1, aon_stream_t stream);
/* Its backward: d0 = grad0 * (g_loss + g_loss0), d1 = grad1 * (g_loss + g_loss1) for device
 * scalars g_* (NULL = absent, taken as 0). */
int aon_loss_pair_bwd(const float* grad0, const float* grad1, int64_t n, const float* g_loss,
                      const float* g_loss0, const float* g_loss1, float* d0, float* d1,
                      aon_stream_t stream);

/* out[n] (+)= sum_m X[m*ldx + n] (bias gradients), deterministic order. */
size_t aon_colsum_workspace_bytes(int64_t M, int64_t N);
int aon_colsum(const float* X, int64_t ldx, int64_t M, int64_t N, int accumulate, float* out,
               void* work, size_t work_bytes, aon_stream_t stream);

/* torch.optim.Adam step (model.py:386-389; no weight decay / amsgrad) over up to
 * AON_ADAM_MAX_TENSORS parameter tensors; `step` counts from 1; lr from optimizer_step's
 * schedule (model.py:399-416).  The hyperparameters are doubles (Python floats): 1 - beta1,
 * 1 - beta2, lr / (1 - beta1^step) and sqrt(1 - beta2^step) are formed in double and rounded
 * to fp32 once, as torch.optim.Adam forms them. */
#define AON_ADAM_MAX_TENSORS 64
typedef struct aon_adam_tensor {
  float* param;
  const float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  int64_t numel;
} aon_adam_tensor;
int aon_adam_step(const aon_adam_tensor* tensors, int count, double lr, double beta1,
                  double beta2, double eps, int64_t step, aon_stream_t stream);

/* ---------------------------------------------------------------- articulated training */
/* Autograd of pos_enc (helper.py:136-140) on the deformed points of the articulated MLP
 * (model_autodecoder.py:205-212): dx (n x 3, row stride lddx) (+)= dL/dx given the points x
 * (row stride ldx; the encodings' identity channels serve, ldx = 3 + 6L) and dL/denc (n x
 * (3 + 6L), row stride ldg), L = max_deg - min_deg.  Replaces torch autograd through
 * model_autodecoder.py:205-212 (SinBackward / CatBackward / MulBackward). */
int aon_pos_enc_bwd(const float* x, int64_t ldx, const float* g_enc, int64_t ldg, int64_t n,
                    int min_deg, int max_deg, int accumulate, float* dx, int64_t lddx,
                    aon_stream_t stream);

/* One term of the latent-code regulariser of LitNeRF_AutoDecoder.training_step
 * (model_autodecoder.py:456-466, weight 1e-4): *loss (+)= weight * mean_c ||code[:, c]||_2 over
 * an (n x c) code; grad (n x c) = weight / c * code / ||code[:, c]|| (0 on a zero column). */
int aon_latent_reg(const float* code, int64_t n, int64_t c, float weight, int accumulate,
                   float* loss, float* grad, aon_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* AONERF_H */
