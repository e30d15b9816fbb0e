// MFMA peak microbenchmark ("peaks ... must be confirmed by a measured MFMA
// microbenchmark").  Back-to-back MFMAs with operands in registers on random data (the chip's
// held clock depends on operand toggling: MI355X_MICROARCH.md 'DVFS give-back'), 8 independent
// accumulators per wave, every CU filled.  kind 0: v_mfma_f32_16x16x32_f16 (the f16x3 MLP's
// instruction); kind 1: v_mfma_f32_16x16x4_f32 (the fp32 path's); kind 2: the f16x3 pattern,
// three dependent MFMAs into one accumulator per step.  Returns TFLOP/s of the issued MFMAs.
#include <hip/hip_runtime.h>
#include <cstdint>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ float rnd(uint32_t s) { return (mix(s) >> 8) * (1.0f / 16777216.0f) - 0.5f; }

template <int KIND>
__global__ __launch_bounds__(256) void k_mfma_loop(int iters, float* out, uint64_t* stamps) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  // in-kernel clock (MI355X_MICROARCH.md DVFS item 6): s_memtime / s_memrealtime (100 MHz)
  // around the loop, one workgroup; stamps go to their own buffer only
  uint64_t c0 = 0, r0 = 0;
  if (blockIdx.x == gridDim.x / 2 && threadIdx.x == 0) {
    c0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  f4 acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = f4{rnd(t * 8 + i), 0.f, 0.f, 0.f};  // distinct chains
  if (KIND == 1) {
    float a[8], b[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      a[i] = rnd(t * 16 + i);
      b[i] = rnd(t * 16 + 8 + i);
    }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[i], acc[i], 0, 0, 0);
    }
  } else {
    h8 a[2], b[2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        a[i][e] = static_cast<_Float16>(rnd(t * 64 + 16 * i + e));
        b[i][e] = static_cast<_Float16>(rnd(t * 64 + 32 + 16 * i + e));
      }
    for (int it = 0; it < iters; ++it) {
      if (KIND == 0) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
          acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[0], b[0], acc[i], 0, 0, 0);
      } else {  // f16x3: hi*hi, hi*lo, lo*hi into one accumulator, 8 accumulators interleaved
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[0], b[0], acc[i], 0, 0, 0);
          acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[0], b[1], acc[i], 0, 0, 0);
          acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[1], b[0], acc[i], 0, 0, 0);
        }
      }
    }
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[t] = s;
  if (blockIdx.x == gridDim.x / 2 && threadIdx.x == 0) {
    stamps[0] = __builtin_amdgcn_s_memtime() - c0;
    stamps[1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}

// returns issued TFLOP/s; *clock_ghz = the in-kernel clock of the last launch
extern "C" double aon_mfma_peak(int kind, int iters, int blocks, float* out, uint64_t* stamps,
                                double* clock_ghz) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  auto launch = [&]() {
    if (kind == 0) hipLaunchKernelGGL(k_mfma_loop<0>, blocks, 256, 0, 0, iters, out, stamps);
    else if (kind == 1) hipLaunchKernelGGL(k_mfma_loop<1>, blocks, 256, 0, 0, iters, out, stamps);
    else hipLaunchKernelGGL(k_mfma_loop<2>, blocks, 256, 0, 0, iters, out, stamps);
  };
  for (int w = 0; w < 3; ++w) launch();  // warm-up (and let the clock settle)
  (void)hipEventRecord(e0, 0);
  const int reps = 10;
  for (int r = 0; r < reps; ++r) launch();
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  if (hipGetLastError() != hipSuccess || ms <= 0.f) return -1.0;
  uint64_t st[2] = {0, 0};
  (void)hipMemcpy(st, stamps, sizeof(st), hipMemcpyDeviceToHost);
  *clock_ghz = st[1] ? (double)st[0] / (double)st[1] * 0.1 : 0.0;
  const double per_mfma = kind == 1 ? 2.0 * 16 * 16 * 4 : 2.0 * 16 * 16 * 32;
  const double mfmas = (double)blocks * 4 /* waves */ * iters * (kind == 2 ? 24 : 8) * reps;
  return mfmas * per_mfma / (ms * 1e-3) / 1e12;
}
