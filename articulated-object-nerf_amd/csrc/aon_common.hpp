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

// rgb_activation / sigma_activation (reference model.py:142-143, 186-187; articulated:
// model_autodecoder.py:265, 323), shared by the MLP epilogue and the compositor
__device__ __forceinline__ float act_rgb(float x, int act) {
  if (act == AON_ACT_NONE) return x;
  const float s = __fdiv_rn(1.0f, __fadd_rn(1.0f, expf(-x)));
  return act == AON_ACT_ARTIC ? __fsub_rn(__fmul_rn(s, 1.002f), 0.001f) : s;
}

__device__ __forceinline__ float act_sigma(float x, int act) {
  if (act == AON_ACT_NONE) return x;
  if (act == AON_ACT_VANILLA) return fmaxf(x, 0.0f);
  // softplus(x - 1) with torch's threshold 20 (model_autodecoder.py:323)
  const float z = __fsub_rn(x, 1.0f);
  return z > 20.0f ? z : log1pf(expf(z));
}

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
  return sinf(cosine ? __fadd_rn(xb, kHalfPi) : xb);
}

// sinf for |x| < 2^17, bit for bit: OCML's __ocml_sin_f32 takes this path there on gfx9.5
// (__ocmlpriv_trigredsmall_f32: a 3-part Cody-Waite reduction by pi/2 in fmas, then
// __ocmlpriv_sincosred_f32's two minimax polynomials and the quadrant's sign / swap).  Called
// directly it costs ~20 VALU; sinf itself compiles both reductions (the Payne-Hanek one for
// |x| >= 2^17 too) and selects, ~150.  Callers guarantee the range (a wave-uniform test, falling
// back to sinf) -- tools/sin_small_check.hip compares the two on every float below 2^17.
__device__ __forceinline__ float sin_small(float x) {
  const float ax = fabsf(x);
  const float r = __builtin_rintf(__fmul_rn(ax, 0x1.45f306p-1f));  // 2/pi
  float t = __builtin_fmaf(r, -0x1.921fb4p+0f, ax);
  t = __builtin_fmaf(r, -0x1.4442d0p-24f, t);
  t = __builtin_fmaf(r, -0x1.846988p-48f, t);
  const int q = static_cast<int>(r) & 3;
  const float t2 = __fmul_rn(t, t);
  float ps = __builtin_fmaf(t2, -0x1.983304p-13f, 0x1.110388p-7f);
  ps = __builtin_fmaf(t2, ps, -0x1.55553ap-3f);
  const float sn = __builtin_fmaf(t, __fmul_rn(t2, ps), t);
  float pc = __builtin_fmaf(t2, 0x1.aea668p-16f, -0x1.6c9e76p-10f);
  pc = __builtin_fmaf(t2, pc, 0x1.5557eep-5f);
  pc = __builtin_fmaf(t2, pc, -0x1.000008p-1f);
  const float cs = __builtin_fmaf(t2, pc, 1.0f);
  const uint32_t v = __float_as_uint((q & 1) == 0 ? sn : cs);
  const uint32_t sgn = (q > 1 ? 0x80000000u : 0u) ^ (__float_as_uint(ax) ^ __float_as_uint(x));
  return __uint_as_float(v ^ sgn);
}
constexpr float kSinSmallMax = 131072.0f;

// pos_enc_feature with sin_small (fast = every |argument| of the caller's wave < 2^17): the
// same value bit for bit
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
  return fast ? sin_small(arg) : sinf(arg);
}
// wave-uniform: every pos_enc argument of this wave's points (|x| 2^(max_deg - 1) + pi/2) is
// below sin_small's range
__device__ __forceinline__ bool pos_enc_fast_ok(float x0, float x1, float x2, int max_deg) {
  const float m = fmaxf(fabsf(x0), fmaxf(fabsf(x1), fabsf(x2)));
  const bool ok = m * __builtin_ldexpf(1.0f, max_deg - 1) + 2.0f < kSinSmallMax;  // (NaN: false)
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
