// Ray generation, stratified sampling and positional encoding (HBM-bound, one lane per
// element, coalesced).  Rounding follows the reference's torch CPU ops: the (n,3)@(3,3)
// product and the row norm are forward fma chains (measured bit-exact against torch 2.10).
#include "aon_common.hpp"

namespace aon {

struct Mat34 {
  float m[12];
};

// rays_d = dirs @ R^T (fma chain over k = 0, 1, 2), then / ||rays_d||
__device__ __forceinline__ void rotate_normalize(float x, float y, float z, const Mat34& c,
                                                 float& ox, float& oy, float& oz, float& rx,
                                                 float& ry, float& rz, bool normalize) {
  rx = fmaf(z, c.m[2], fmaf(y, c.m[1], __fmul_rn(x, c.m[0])));
  ry = fmaf(z, c.m[6], fmaf(y, c.m[5], __fmul_rn(x, c.m[4])));
  rz = fmaf(z, c.m[10], fmaf(y, c.m[9], __fmul_rn(x, c.m[8])));
  if (normalize) {
    const float n = sqrtf(fmaf(rz, rz, fmaf(ry, ry, __fmul_rn(rx, rx))));
    rx = __fdiv_rn(rx, n);
    ry = __fdiv_rn(ry, n);
    rz = __fdiv_rn(rz, n);
  }
  ox = c.m[3];
  oy = c.m[7];
  oz = c.m[11];
}

// reference datasets/ray_utils.py:84-88 (kornia grid: i = column, j = row; no +0.5)
__device__ __forceinline__ void pixel_dir(int64_t p, int H, int W, float focal, float& x,
                                          float& y) {
  const int row = static_cast<int>(p / W), col = static_cast<int>(p - static_cast<int64_t>(row) * W);
  x = __fdiv_rn(__fsub_rn(static_cast<float>(col), 0.5f * static_cast<float>(W)), focal);
  y = __fdiv_rn(-__fsub_rn(static_cast<float>(row), 0.5f * static_cast<float>(H)), focal);
}

__global__ void k_ray_directions(int H, int W, float focal, float* __restrict__ dirs) {
  const int64_t n = static_cast<int64_t>(H) * W;
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < n;
       p += (int64_t)gridDim.x * blockDim.x) {
    float x, y;
    pixel_dir(p, H, W, focal, x, y);
    dirs[3 * p + 0] = x;
    dirs[3 * p + 1] = y;
    dirs[3 * p + 2] = -1.0f;
  }
}

__global__ void k_get_rays(const float* __restrict__ dirs, int64_t n, Mat34 c2w,
                           float* __restrict__ ro, float* __restrict__ rd,
                           float* __restrict__ vd) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < n;
       p += (int64_t)gridDim.x * blockDim.x) {
    float ox, oy, oz, rx, ry, rz;
    rotate_normalize(dirs[3 * p], dirs[3 * p + 1], dirs[3 * p + 2], c2w, ox, oy, oz, rx, ry, rz,
                     true);
    ro[3 * p] = ox; ro[3 * p + 1] = oy; ro[3 * p + 2] = oz;
    rd[3 * p] = rx; rd[3 * p + 1] = ry; rd[3 * p + 2] = rz;
    if (vd) { vd[3 * p] = rx; vd[3 * p + 1] = ry; vd[3 * p + 2] = rz; }
  }
}

// radii (ray_utils.py:138-143): || rd[y] - rd[y+1] || * 2 / sqrt(12) on UNnormalised world
// directions; the last row repeats dx[-2:-1], the SECOND-to-last of dx's H-1 rows (row H-3).
__global__ void k_radii(const float* __restrict__ dirs, int H, int W, Mat34 c2w,
                        float* __restrict__ radii) {
  const int64_t n = static_cast<int64_t>(H) * W;
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < n;
       p += (int64_t)gridDim.x * blockDim.x) {
    int64_t row = p / W;
    const int64_t col = p - row * W;
    if (row == H - 1) row = H - 3;  // torch.cat([dx, dx[-2:-1, :]])
    const int64_t a = row * W + col, b = (row + 1) * W + col;
    float o0, o1, o2, ax, ay, az, bx, by, bz;
    rotate_normalize(dirs[3 * a], dirs[3 * a + 1], dirs[3 * a + 2], c2w, o0, o1, o2, ax, ay, az,
                     false);
    rotate_normalize(dirs[3 * b], dirs[3 * b + 1], dirs[3 * b + 2], c2w, o0, o1, o2, bx, by, bz,
                     false);
    const float dx = __fsub_rn(ax, bx), dy = __fsub_rn(ay, by), dz = __fsub_rn(az, bz);
    // torch.sum over 3 squared terms (a 3-wide reduction adds (x+y)+z)
    const float s = __fadd_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)), __fmul_rn(dz, dz));
    radii[p] = __fdiv_rn(__fmul_rn(sqrtf(s), 2.0f), 3.46410155f);
  }
}

__global__ void k_frame_rays(int H, int W, float focal, Mat34 c2w, int64_t p0, int64_t n,
                             float* __restrict__ ro, float* __restrict__ rd,
                             float* __restrict__ vd) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < n;
       p += (int64_t)gridDim.x * blockDim.x) {
    float x, y, ox, oy, oz, rx, ry, rz;
    pixel_dir(p0 + p, H, W, focal, x, y);
    rotate_normalize(x, y, -1.0f, c2w, ox, oy, oz, rx, ry, rz, true);
    ro[3 * p] = ox; ro[3 * p + 1] = oy; ro[3 * p + 2] = oz;
    rd[3 * p] = rx; rd[3 * p + 1] = ry; rd[3 * p + 2] = rz;
    if (vd) { vd[3 * p] = rx; vd[3 * p + 1] = ry; vd[3 * p + 2] = rz; }
  }
}

// helper.py:122-131: t = lower + (upper - lower) * u (randomized) or the schedule; xyz = o + t*d
__global__ void k_sample_along_rays(const float* __restrict__ ro, const float* __restrict__ rd,
                                    int64_t B, int S, const float* __restrict__ lower,
                                    const float* __restrict__ upper, const float* __restrict__ u,
                                    float* __restrict__ t_out, float* __restrict__ xyz) {
  const int64_t n = B * S;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / S;
    const int s = static_cast<int>(i - b * S);
    float t = lower[s];
    if (u) t = __fadd_rn(t, __fmul_rn(__fsub_rn(upper[s], lower[s]), u[i]));
    t_out[i] = t;
    if (xyz) {
#pragma unroll
      for (int c = 0; c < 3; ++c) xyz[3 * i + c] = __fadd_rn(ro[3 * b + c], __fmul_rn(t, rd[3 * b + c]));
    }
  }
}

__global__ void k_pos_enc(const float* __restrict__ x, int64_t n, int min_deg, int L,
                          float* __restrict__ out) {
  const int C = 3 + 6 * L;
  const int64_t total = n * C;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / C;
    const int f = static_cast<int>(i - r * C);
    out[i] = pos_enc_feature(x[3 * r], x[3 * r + 1], x[3 * r + 2], f, min_deg, L);
  }
}

// cast_rays (helper.py:25-26) on per-ray t (B, S), optionally displaced by a per-sample offset
// (the articulated deformation, model_autodecoder.py:205: deformation_layer(x) + pos) and
// optionally straight into pos_enc (helper.py:136-140): one thread per (sample, feature)
// Idx: the element index type -- 32-bit when the launch has < 2^31 elements (the training
// step's 50 M), so the two index divisions per element are 32-bit, not 64-bit, sequences.
template <typename Idx>
__global__ void k_cast_rays(const float* __restrict__ ro, const float* __restrict__ rd,
                            const float* __restrict__ t, int64_t B, int S,
                            const float* __restrict__ off, int64_t off_stride,
                            float* __restrict__ xyz, int min_deg, int L, float* __restrict__ enc) {
  const int C = enc ? 3 + 6 * L : 3;
  const Idx total = static_cast<Idx>(B * S * C);
  for (Idx i = blockIdx.x * (Idx)blockDim.x + threadIdx.x; i < total;
       i += (Idx)gridDim.x * blockDim.x) {
    const Idx r = i / static_cast<Idx>(C);
    const int f = static_cast<int>(i - r * static_cast<Idx>(C));
    const Idx b = r / static_cast<Idx>(S);
    float x0 = ro[3 * b], x1 = ro[3 * b + 1], x2 = ro[3 * b + 2];
    if (rd) {  // rays_d == NULL: the points are given directly (rays_o rows)
      const float tv = t[r];
      x0 = __fadd_rn(x0, __fmul_rn(tv, rd[3 * b]));
      x1 = __fadd_rn(x1, __fmul_rn(tv, rd[3 * b + 1]));
      x2 = __fadd_rn(x2, __fmul_rn(tv, rd[3 * b + 2]));
    }
    if (off) {
      const float* o = off + r * off_stride;
      x0 = __fadd_rn(o[0], x0);
      x1 = __fadd_rn(o[1], x1);
      x2 = __fadd_rn(o[2], x2);
    }
    if (xyz && f < 3) xyz[3 * r + f] = f == 0 ? x0 : (f == 1 ? x1 : x2);
    if (enc) enc[i] = pos_enc_feature(x0, x1, x2, f, min_deg, L);
  }
}

// The same encodings in the fused training kernels' 16-row tiled layout (mlp_f16x3_core.hpp
// act_base) with `width` columns, the ones past 3 + 6 L zero: the parity mode's copy of
// pos_enc(x) for the enc-column weight gradients (aon_gemm's 256 x 64 f16_single kernel reads
// whole 16-column tiles).  One thread per (sample, column).
template <typename Idx>
__global__ void k_cast_rays_tiled(const float* __restrict__ ro, const float* __restrict__ rd,
                                  const float* __restrict__ t, int64_t B, int S, int min_deg,
                                  int L, int width, float* __restrict__ enc) {
  const int C = 3 + 6 * L;
  const Idx total = static_cast<Idx>(B * S * width);
  for (Idx i = blockIdx.x * (Idx)blockDim.x + threadIdx.x; i < total;
       i += (Idx)gridDim.x * blockDim.x) {
    const Idx r = i / static_cast<Idx>(width);
    const int f = static_cast<int>(i - r * static_cast<Idx>(width));
    float v = 0.0f;
    if (f < C) {
      const Idx b = r / static_cast<Idx>(S);
      const float tv = t[r];
      const float x0 = __fadd_rn(ro[3 * b], __fmul_rn(tv, rd[3 * b]));
      const float x1 = __fadd_rn(ro[3 * b + 1], __fmul_rn(tv, rd[3 * b + 1]));
      const float x2 = __fadd_rn(ro[3 * b + 2], __fmul_rn(tv, rd[3 * b + 2]));
      v = pos_enc_feature(x0, x1, x2, f, min_deg, L);
    }
    const int64_t rr = static_cast<int64_t>(r);
    enc[(rr & ~int64_t(15)) * width + 256 * (f >> 4) + 16 * (rr & 15) + (f & 15)] = v;
  }
}

// Training-ray batches straight from the device-resident dataset (reference
// datasets/sapien.py:84-113 / :131-154 and sapien_multi.py:196-238): for flat index
// g = image * H * W + pixel, the camera ray of that pixel (as k_frame_rays) and its target:
//   mode 0: rgb = u8 / 255                          (C >= 3)
//   mode 1: rgb * a + (1 - a), a = alpha / 255      (RGBA onto white, sapien.py:98-99)
//   mode 2: channel 3 is a segmentation mask: rgb where mask > 0, else bg (sapien_multi.py:186-194)
__global__ void k_sample_rays(const float* __restrict__ poses, const uint8_t* __restrict__ img,
                              int C, int64_t N, int H, int W, float focal,
                              const int64_t* __restrict__ idx, int64_t n, int mode, float bg,
                              float* __restrict__ ro, float* __restrict__ rd,
                              float* __restrict__ vd, float* __restrict__ target) {
  const int64_t hw = static_cast<int64_t>(H) * W;
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t g = idx ? idx[q] : q;
    const int64_t k = g / hw, p = g - k * hw;
    Mat34 c;
#pragma unroll
    for (int e = 0; e < 12; ++e) c.m[e] = poses[12 * k + e];
    float x, y, ox, oy, oz, rx, ry, rz;
    pixel_dir(p, H, W, focal, x, y);
    rotate_normalize(x, y, -1.0f, c, ox, oy, oz, rx, ry, rz, true);
    ro[3 * q] = ox; ro[3 * q + 1] = oy; ro[3 * q + 2] = oz;
    rd[3 * q] = rx; rd[3 * q + 1] = ry; rd[3 * q + 2] = rz;
    if (vd) { vd[3 * q] = rx; vd[3 * q + 1] = ry; vd[3 * q + 2] = rz; }
    if (target) {
      const uint8_t* px = img + g * C;
      float v[3];
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) v[ch] = __fdiv_rn(static_cast<float>(px[ch]), 255.0f);
      if (mode == 1) {
        const float a = __fdiv_rn(static_cast<float>(px[3]), 255.0f);
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) v[ch] = __fadd_rn(__fmul_rn(v[ch], a), __fsub_rn(1.0f, a));
      } else if (mode == 2 && px[3] == 0) {
        v[0] = v[1] = v[2] = bg;
      }
      target[3 * q] = v[0]; target[3 * q + 1] = v[1]; target[3 * q + 2] = v[2];
    }
  }
}

static Mat34 load_c2w(const float* h) {
  Mat34 m;
  for (int i = 0; i < 12; ++i) m.m[i] = h[i];
  return m;
}

}  // namespace aon

using namespace aon;

extern "C" int aon_ray_directions(int H, int W, float focal, float* dirs, aon_stream_t stream) {
  AON_REQUIRE(H > 0 && W > 0 && dirs, "bad arguments");
  hipLaunchKernelGGL(k_ray_directions, grid_for((int64_t)H * W, 256, 65536), 256, 0,
                     (hipStream_t)stream, H, W, focal, dirs);
  return launch_status(__func__);
}

extern "C" int aon_get_rays(const float* dirs, int64_t n, const float* c2w_host, float* rays_o,
                            float* rays_d, float* viewdirs, int H, int W, float* radii,
                            aon_stream_t stream) {
  AON_REQUIRE(dirs && c2w_host && rays_o && rays_d && n >= 0, "null pointer or negative n");
  if (n == 0) return 0;
  const Mat34 c = load_c2w(c2w_host);
  hipLaunchKernelGGL(k_get_rays, grid_for(n, 256, 65536), 256, 0, (hipStream_t)stream, dirs, n, c,
                     rays_o, rays_d, viewdirs);
  if (radii) {
    // dx has H-1 rows and the reference appends dx[-2:-1]: H = 2 leaves it a row short
    AON_REQUIRE(H >= 3 && (int64_t)H * W == n, "radii need a full (H>=3, W) direction grid");
    hipLaunchKernelGGL(k_radii, grid_for(n, 256, 65536), 256, 0, (hipStream_t)stream, dirs, H, W,
                       c, radii);
  }
  return launch_status(__func__);
}

extern "C" int aon_frame_rays(int H, int W, float focal, const float* c2w_host, int64_t p0,
                              int64_t n, float* rays_o, float* rays_d, float* viewdirs,
                              aon_stream_t stream) {
  AON_REQUIRE(H > 0 && W > 0 && c2w_host && rays_o && rays_d, "bad arguments");
  AON_REQUIRE(p0 >= 0 && n >= 0 && p0 + n <= (int64_t)H * W, "pixel range outside the frame");
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_frame_rays, grid_for(n, 256, 65536), 256, 0, (hipStream_t)stream, H, W,
                     focal, load_c2w(c2w_host), p0, n, rays_o, rays_d, viewdirs);
  return launch_status(__func__);
}

extern "C" int aon_sample_along_rays(const float* rays_o, const float* rays_d, int64_t B, int S,
                                     const float* t_lower, const float* t_upper, const float* u,
                                     float* t_out, float* xyz_out, aon_stream_t stream) {
  AON_REQUIRE(B >= 0 && S > 0 && t_lower && t_out, "bad arguments");
  AON_REQUIRE(!u || t_upper, "randomized sampling needs t_upper");
  AON_REQUIRE(!xyz_out || (rays_o && rays_d), "xyz needs rays_o/rays_d");
  if (B == 0) return 0;
  hipLaunchKernelGGL(k_sample_along_rays, grid_for(B * S, 256, 65536), 256, 0, (hipStream_t)stream,
                     rays_o, rays_d, B, S, t_lower, t_upper, u, t_out, xyz_out);
  return launch_status(__func__);
}

extern "C" int aon_pos_enc(const float* x, int64_t n, int min_deg, int max_deg, float* out,
                           aon_stream_t stream) {
  AON_REQUIRE(x && out && n >= 0 && max_deg >= min_deg && min_deg >= -126 && max_deg <= 127,
              "bad arguments");
  if (n == 0) return 0;
  const int L = max_deg - min_deg;
  hipLaunchKernelGGL(k_pos_enc, grid_for(n * (3 + 6 * L), 256, 65536), 256, 0, (hipStream_t)stream,
                     x, n, min_deg, L, out);
  return launch_status(__func__);
}

extern "C" int aon_cast_rays(const float* rays_o, const float* rays_d, const float* t, int64_t B,
                             int S, const float* offset, int64_t offset_stride, float* xyz,
                             int min_deg, int max_deg, float* enc, aon_stream_t stream) {
  AON_REQUIRE(rays_o && (!rays_d || t) && (xyz || enc) && B >= 0 && S >= 1, "bad arguments");
  AON_REQUIRE(!offset || offset_stride >= 3, "offset rows need >= 3 floats");
  AON_REQUIRE(!enc || (max_deg >= min_deg && min_deg >= -126 && max_deg <= 127), "bad degrees");
  if (B == 0) return 0;
  const int L = max_deg - min_deg;
  const int C = enc ? 3 + 6 * L : 3;
  if (B * S * C < (int64_t(1) << 31))
    hipLaunchKernelGGL(k_cast_rays<uint32_t>, grid_for(B * S * C, 256, 65536), 256, 0,
                       (hipStream_t)stream, rays_o, rays_d, t, B, S, offset, offset_stride, xyz,
                       min_deg, L, enc);
  else
    hipLaunchKernelGGL(k_cast_rays<int64_t>, grid_for(B * S * C, 256, 65536), 256, 0,
                       (hipStream_t)stream, rays_o, rays_d, t, B, S, offset, offset_stride, xyz,
                       min_deg, L, enc);
  return launch_status(__func__);
}

extern "C" int aon_cast_rays_tiled(const float* rays_o, const float* rays_d, const float* t,
                                   int64_t B, int S, int min_deg, int max_deg, int width,
                                   float* enc, aon_stream_t stream) {
  AON_REQUIRE(rays_o && rays_d && t && enc && B >= 0 && S >= 1, "bad arguments");
  AON_REQUIRE(max_deg >= min_deg && min_deg >= -126 && max_deg <= 127, "bad degrees");
  AON_REQUIRE(width % 16 == 0 && width >= 3 + 6 * (max_deg - min_deg),
              "width: a multiple of 16 holding every encoding");
  if (B == 0) return 0;
  const int L = max_deg - min_deg;
  if (B * S * width < (int64_t(1) << 31))
    hipLaunchKernelGGL(k_cast_rays_tiled<uint32_t>, grid_for(B * S * width, 256, 65536), 256, 0,
                       (hipStream_t)stream, rays_o, rays_d, t, B, S, min_deg, L, width, enc);
  else
    hipLaunchKernelGGL(k_cast_rays_tiled<int64_t>, grid_for(B * S * width, 256, 65536), 256, 0,
                       (hipStream_t)stream, rays_o, rays_d, t, B, S, min_deg, L, width, enc);
  return launch_status(__func__);
}

extern "C" int aon_sample_rays(const float* poses, const uint8_t* images, int C, int64_t N, int H,
                               int W, float focal, const int64_t* idx, int64_t n, int mode,
                               float bg, float* rays_o, float* rays_d, float* viewdirs,
                               float* target, aon_stream_t stream) {
  AON_REQUIRE(poses && rays_o && rays_d && N >= 1 && H > 0 && W > 0 && n >= 0, "bad arguments");
  AON_REQUIRE(!target || (images && C >= 3 && (mode == 0 || C >= 4)), "bad image layout");
  AON_REQUIRE(mode >= 0 && mode <= 2, "bad mode");
  AON_REQUIRE(idx || n <= N * (int64_t)H * W, "n exceeds the dataset");
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_sample_rays, grid_for(n, 256, 65536), 256, 0, (hipStream_t)stream, poses,
                     images, C, N, H, W, focal, idx, n, mode, bg, rays_o, rays_d, viewdirs, target);
  return launch_status(__func__);
}
