// Shared helpers of the aonerf HIP library (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <string>
#include <unordered_map>

#include "aonerf.h"

namespace aon {

typedef float f4 __attribute__((ext_vector_type(4)));

// thread-local error message behind aon_last_error()
void set_error(const std::string& msg);

#define AON_REQUIRE(cond, msg)                                   \
  do {                                                           \
    if (!(cond)) {                                               \
      ::aon::set_error(std::string(__func__) + ": " + (msg));    \
      return -1;                                                 \
    }                                                            \
  } while (0)

inline int launch_status(const char* fn) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(std::string(fn) + ": " + hipGetErrorString(e));
    return static_cast<int>(e);
  }
  return 0;
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

inline int grid_for(int64_t work, int per_block, int cap = 1 << 20) {
  int64_t g = (work + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return static_cast<int>(g);
}

// Workgroups of `kernel` the device keeps resident at once (occupancy x CUs), queried once per
// kernel.  A grid-stride kernel that software-pipelines over its items launches at most this
// many: a second, partial round of workgroups would add a tail of one workgroup's duration.
inline int64_t resident_blocks(const void* kernel, int threads) {
  static std::mutex mu;
  static std::unordered_map<const void*, int64_t> cache;
  std::lock_guard<std::mutex> lock(mu);
  auto it = cache.find(kernel);
  if (it != cache.end()) return it->second;
  int dev = 0, cus = 0, per_cu = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, 0);
  const int64_t r = static_cast<int64_t>(cus > 0 ? cus : 256) * (per_cu > 0 ? per_cu : 1);
  cache.emplace(kernel, r);
  return r;
}

template <typename Kernel>
inline int resident_grid(Kernel kernel, int threads, int64_t work_blocks) {
  const int64_t r = resident_blocks(reinterpret_cast<const void*>(kernel), threads);
  return grid_for(work_blocks, 1, static_cast<int>(r));
}

// torch.nan_to_num(x, nan=nan_val) with default posinf/neginf (float max / lowest)
__device__ __forceinline__ float nan_to_num(float x, float nan_val) {
  if (x != x) return nan_val;
  if (x == __builtin_inff()) return 3.40282347e+38f;
  if (x == -__builtin_inff()) return -3.40282347e+38f;
  return x;
}

// exp as torch's vectorised CPU kernels evaluate it inside sigmoid and softplus: SLEEF
// 3.x xexpf (the u10 variant; ATen's Vectorized<float>::exp), restated from its published
// algorithm -- round(d/ln2) with a two-part Cody-Waite reduction, a degree-6 Horner
// polynomial and a split 2^q scaling.  With it, 1/(1 + exp_sleef(-x)) reproduces
// torch.sigmoid bit for bit (checked on 4M values, tests/test_transcendentals.py).
__host__ __device__ inline float exp_sleef(float d) {  // (built with -ffp-contract=off)
  const int q = (int)__builtin_rintf(d * 1.442695040888963407359924681f);
  float s = __builtin_fmaf((float)q, -0.693145751953125f, d);
  s = __builtin_fmaf((float)q, -1.428606765330187045e-06f, s);
  float u = 0.000198527617612853646278381f;
  u = __builtin_fmaf(u, s, 0.00139304355252534151077271f);
  u = __builtin_fmaf(u, s, 0.00833336077630519866943359f);
  u = __builtin_fmaf(u, s, 0.0416664853692054748535156f);
  u = __builtin_fmaf(u, s, 0.166666671633720397949219f);
  u = __builtin_fmaf(u, s, 0.5f);
  u = 1.0f + __builtin_fmaf(s * s, u, s);
  const int q1 = q >> 1, q2 = q - q1;  // 2^q as two factors so q = 128 does not overflow
  u = (u * __builtin_bit_cast(float, (q1 + 127) << 23)) * __builtin_bit_cast(float, (q2 + 127) << 23);
  if (d < -104.0f) u = 0.0f;
  if (d > 100.0f) u = __builtin_inff();
  return d != d ? d : u;
}

// exp as torch.exp evaluates it on CPU for the alpha of volumetric_rendering (MKL's
// high-accuracy vsExp: correctly rounded in ~99% of elements): the correctly rounded fp32
// exp, evaluated in fp64 and rounded once.  Every alpha argument is -sigma * delta <= 0: k =
// round(x / ln2) and r = x - k ln2 (fdlibm's two-part ln2, fmas; |r| <= 0.347), then the degree-12
// Taylor polynomial (remainder < 2^-52) and 2^k by v_ldexp_f64 -- fewer live fp64 temporaries
// than the general fp64 exp (the fine compositor runs at 80 VGPRs).  Arguments below -120 (fp32
// result 0) are clamped; NaN propagates; x > 0 is outside the domain the callers use (correct
// to x = 88, where fp32 overflows anyway only through the polynomial's accuracy at |r| <= 0.347).
#ifndef AON_ALPHA_EXP_DEVICE
#define AON_ALPHA_EXP_DEVICE 0  // 1: timing-only A/B build -- the device's own expf (not the torch value)
#endif
__host__ __device__ inline float exp_cr(float xf) {
#if AON_ALPHA_EXP_DEVICE
  return expf(xf);
#endif
  const double x = xf < -120.0f ? -120.0 : (double)xf;
  const double k = __builtin_rint(x * 1.44269504088896338700e+00);
  double r = __builtin_fma(-k, 6.93147180369123816490e-01, x);
  r = __builtin_fma(-k, 1.90821492927058770002e-10, r);
  double p = 1.0 / 479001600.0;
  p = __builtin_fma(r, p, 1.0 / 39916800.0);
  p = __builtin_fma(r, p, 1.0 / 3628800.0);
  p = __builtin_fma(r, p, 1.0 / 362880.0);
  p = __builtin_fma(r, p, 1.0 / 40320.0);
  p = __builtin_fma(r, p, 1.0 / 5040.0);
  p = __builtin_fma(r, p, 1.0 / 720.0);
  p = __builtin_fma(r, p, 1.0 / 120.0);
  p = __builtin_fma(r, p, 1.0 / 24.0);
  p = __builtin_fma(r, p, 1.0 / 6.0);
  p = __builtin_fma(r, p, 0.5);
  p = __builtin_fma(r, p, 1.0);
  p = __builtin_fma(r, p, 1.0);
  return (float)__builtin_ldexp(p, (int)k);
}

// rgb_activation / sigma_activation (reference model.py:142-143, 186-187; articulated:
// model_autodecoder.py:265, 323), shared by the MLP epilogue and the compositor.
// torch.sigmoid on CPU is 1/(1 + exp(-x)) with SLEEF's exp; F.softplus is
// log1p(exp(x)) with SLEEF's exp and log1p (here the device log1pf).
__device__ __forceinline__ float act_rgb(float x, int act) {
  if (act == AON_ACT_NONE) return x;
  const float s = __fdiv_rn(1.0f, __fadd_rn(1.0f, exp_sleef(-x)));
  return act == AON_ACT_ARTIC ? __fsub_rn(__fmul_rn(s, 1.002f), 0.001f) : s;
}

__device__ __forceinline__ float act_sigma(float x, int act) {
  if (act == AON_ACT_NONE) return x;
  if (act == AON_ACT_VANILLA) return fmaxf(x, 0.0f);
  // softplus(x - 1) with torch's threshold 20 (model_autodecoder.py:323)
  const float z = __fsub_rn(x, 1.0f);
  return z > 20.0f ? z : log1pf(exp_sleef(z));
}

// sin / cos of an fp32 argument, correctly rounded: evaluated in fp64 and rounded once.  torch's
// CPU sin / cos (the reference's pos_enc, helper.py:139, and its autograd's cos) are correctly
// rounded in ~95% of elements; the device sinf (OCML) in ~79% -- measured on 12M arguments, and
// this evaluation equals float(sin(double(x))) on all of them (tests/test_transcendentals.py
// runs the same arithmetic on the host, tests/test_gpu_transcendentals.py on the device).
// Cody-Waite reduction by pi/2 in three fmas (fdlibm's pio2_1 / pio2_2 are 33-bit: r * part is
// exact while |r| < 2^20, i.e. |x| < kSinCrMax), then fdlibm's __kernel_sin / __kernel_cos
// minimax polynomials on [-pi/4, pi/4] (~2^-55 relative; the single rounding to fp32 is
// then off only within 2^-30 of a rounding midpoint).  qoff = 1 gives cos (sin(x + pi/2)).
constexpr float kSinCrMax = 1048576.0f;
__host__ __device__ inline float sincos_cr(float xf, int qoff) {
  const double x = xf;
  const double r = __builtin_rint(x * 6.36619772367581382433e-01);
  double t = __builtin_fma(-r, 1.57079632673412561417e+00, x);
  t = __builtin_fma(-r, 6.07710050630396597660e-11, t);
  t = __builtin_fma(-r, 2.02226624879595063154e-21, t);
  const int q = (static_cast<int>(r) + qoff) & 3;
  // one Horner chain for both: sin(t) = t (1 + z (S1 + .. + z S6)), cos(t) = 1 + z (-1/2 + z (C1
  // + .. + z C6)), z = t^2 -- the coefficients selected per lane (the two chains' registers
  // would both stay live across the unrolled features)
  const bool odd = q & 1;
  const double z = t * t;
  double p = odd ? -1.13596475577881948265e-11 : 0.0;
  p = __builtin_fma(z, p, odd ? 2.08757232129817482790e-09 : 1.58969099521155010221e-10);
  p = __builtin_fma(z, p, odd ? -2.75573143513906633035e-07 : -2.50507602534068634195e-08);
  p = __builtin_fma(z, p, odd ? 2.48015872894767294178e-05 : 2.75573137070700676789e-06);
  p = __builtin_fma(z, p, odd ? -1.38888888888741095749e-03 : -1.98412698298579493134e-04);
  p = __builtin_fma(z, p, odd ? 4.16666666666666019037e-02 : 8.33333333332248946124e-03);
  p = __builtin_fma(z, p, odd ? -0.5 : -1.66666666666666324348e-01);
  p = __builtin_fma(z, p, 1.0);
  const double v = odd ? p : t * p;
  return static_cast<float>((q & 2) ? -v : v);
}
// any argument (past kSinCrMax: OCML's fp64 sin / cos, also rounded once)
__device__ __forceinline__ float sin_cr(float x) {
  if (__builtin_expect(fabsf(x) < kSinCrMax, 1)) return sincos_cr(x, 0);
  return static_cast<float>(__ocml_sin_f64(static_cast<double>(x)));
}
__device__ __forceinline__ float cos_cr(float x) {
  if (__builtin_expect(fabsf(x) < kSinCrMax, 1)) return sincos_cr(x, 1);
  return static_cast<float>(__ocml_cos_f64(static_cast<double>(x)));
}

#ifndef AON_POS_ENC_NOSIN
#define AON_POS_ENC_NOSIN 0
#endif
// fp32(0.5 * pi) as torch adds it to an fp32 tensor (reference helper.py:139)
constexpr float kHalfPi = 1.57079637050628662109375f;

// One pos_enc feature f of a 3-vector (reference helper.py:136-140):
//   f < 3            -> x[f]
//   3 <= f < 3+3L    -> sin(x[c] * 2^d),          (f-3) = 3d + c
//   3+3L <= f < 3+6L -> sin(x[c] * 2^d + pi/2f),  (f-3-3L) = 3d + c
//   otherwise        -> 0 (K padding)
__device__ __forceinline__ float pos_enc_feature(float x0, float x1, float x2, int f, int min_deg,
                                                 int L) {
  if (f < 3) return f == 0 ? x0 : (f == 1 ? x1 : x2);
  int q = f - 3;
  bool cosine = false;
  if (q >= 3 * L) {
    q -= 3 * L;
    cosine = true;
  }
  if (q >= 3 * L) return 0.f;
  const int d = q / 3, c = q - 3 * d;
  const float xc = c == 0 ? x0 : (c == 1 ? x1 : x2);
  const float xb = xc * __builtin_ldexpf(1.0f, min_deg + d);  // exact power-of-two scaling
  return sin_cr(cosine ? __fadd_rn(xb, kHalfPi) : xb);
}

// pos_enc_feature with the range test hoisted (fast = every |argument| of the caller's wave
// below kSinCrMax: no per-value branch): the same value bit for bit
__device__ __forceinline__ float pos_enc_feature_fast(float x0, float x1, float x2, int f,
                                                      int min_deg, int L, bool fast) {
  if (f < 3) return f == 0 ? x0 : (f == 1 ? x1 : x2);
  int q = f - 3;
  bool cosine = false;
  if (q >= 3 * L) {
    q -= 3 * L;
    cosine = true;
  }
  if (q >= 3 * L) return 0.f;
  const int d = q / 3, c = q - 3 * d;
  const float xc = c == 0 ? x0 : (c == 1 ? x1 : x2);
  const float xb = xc * __builtin_ldexpf(1.0f, min_deg + d);
  const float arg = cosine ? __fadd_rn(xb, kHalfPi) : xb;
#if AON_POS_ENC_NOSIN  // timing-only A/B build: no sine at all (wrong values; bounds its cost)
  (void)fast;
  return arg;
#else
  return fast ? sincos_cr(arg, 0) : sin_cr(arg);
#endif
}
// wave-uniform: every pos_enc argument of this wave's points (|x| 2^(max_deg - 1) + pi/2) is
// below kSinCrMax
__device__ __forceinline__ bool pos_enc_fast_ok(float x0, float x1, float x2, int max_deg) {
  const float m = fmaxf(fabsf(x0), fmaxf(fabsf(x1), fabsf(x2)));
  const bool ok = m * __builtin_ldexpf(1.0f, max_deg - 1) + 2.0f < kSinCrMax;  // (NaN: false)
  return __builtin_amdgcn_ballot_w64(!ok) == 0;
}

// Per-call power-of-two scale of a gradient operand from the bits of its max |x| (k_absmax):
// |x * s| < 2^8 for the largest |x|: s = 2^(8 - e) with max = m 2^e, m in [0.5, 1).  The fp16
// hi/lo splits of the backward chains and the weight-gradient GEMMs carry gradients at s, so
// their hi parts stay normal however small the loss gradient gets (a mean over 4096 rays).
__device__ __forceinline__ float grad_scale(uint32_t bits) {
  const float m = __uint_as_float(bits);
  if (!(m > 0.0f) || !isfinite(m)) return 1.0f;
  int e;
  (void)frexpf(m, &e);
  e = e < -100 ? -100 : (e > 100 ? 100 : e);
  return __builtin_ldexpf(1.0f, 8 - e);
}

// ---- DPP lane moves (gfx9 controls).  Lanes whose source is outside the pattern keep `old`.
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ double dpp_f64(double src, double old) {
  const long long s = __builtin_bit_cast(long long, src), o = __builtin_bit_cast(long long, old);
  const int lo = __builtin_amdgcn_update_dpp((int)o, (int)s, CTRL, ROW_MASK, 0xF, false);
  const int hi =
      __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(s >> 32), CTRL, ROW_MASK, 0xF, false);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
}

__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const long long s = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_readlane((int)s, lane);
  const int hi = __builtin_amdgcn_readlane((int)(s >> 32), lane);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
}

// inclusive prefix product over the 64 lanes: row_shr 1/2/4/8 inside 16-lane rows, then
// row_bcast:15 (rows 1, 3) and row_bcast:31 (rows 2, 3) -- VALU lane moves, no LDS
__device__ __forceinline__ double wave_incl_prod(double x) {
  x *= dpp_f64<0x111>(x, 1.0);
  x *= dpp_f64<0x112>(x, 1.0);
  x *= dpp_f64<0x114>(x, 1.0);
  x *= dpp_f64<0x118>(x, 1.0);
  x *= dpp_f64<0x142, 0xA>(x, 1.0);
  x *= dpp_f64<0x143, 0xC>(x, 1.0);
  return x;
}

// inclusive prefix sum over the 64 lanes, same lane moves as wave_incl_prod
__device__ __forceinline__ double wave_incl_sum(double x) {
  x += dpp_f64<0x111>(x, 0.0);
  x += dpp_f64<0x112>(x, 0.0);
  x += dpp_f64<0x114>(x, 0.0);
  x += dpp_f64<0x118>(x, 0.0);
  x += dpp_f64<0x142, 0xA>(x, 0.0);
  x += dpp_f64<0x143, 0xC>(x, 0.0);
  return x;
}

}  // namespace aon
