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

#define AON_ABI_VERSION 2

/* Precision of the MLP GEMMs (see DESIGN.md "MLP precision modes"). */
#define AON_PREC_FP32 0  /* exact fp32 MFMA (v_mfma_f32_16x16x4_f32) */
#define AON_PREC_F16X3 1 /* fp16 hi/lo split, 3 products (hi*hi + hi*lo + lo*hi) per weight on
                            v_mfma_f32_16x16x32_f16, fp32 accumulate: ~22-bit operands */

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
} aon_mlp_params;

size_t aon_mlp_packed_bytes(int precision);
/* Re-lay the parameters into the MFMA-tiled weight stream consumed by aon_mlp_fwd. */
int aon_mlp_pack(const aon_mlp_params* params, int precision, void* packed,
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

/* NeRFMLP.forward on pre-encoded inputs: x (B*S, 63), condition (B, 27) -> out (B*S, 4). */
int aon_mlp_fwd_encoded(const void* packed, int precision, const float* x,
                        const float* condition, int64_t B, int S, int act, float* out,
                        aon_stream_t stream);

/* ---------------------------------------------------------------- compositing */
/* volumetric_rendering (helper.py:157-195) with the activations of model.py:186-187.
 * rgb: (B*S) rows of rgb_stride floats (3 = API tensor, 4 = fused raw buffer);
 * sigma: (B*S) rows of sigma_stride floats.  weights may be NULL. */
int aon_composite_fwd(const float* rgb, int64_t rgb_stride, const float* sigma,
                      int64_t sigma_stride, const float* t, const float* dirs, int64_t B,
                      int S, int white_bkgd, int act, float* comp_rgb, float* acc,
                      float* weights, float* depth, aon_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* AONERF_H */
