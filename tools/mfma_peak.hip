// MFMA peak microbenchmark ("peaks ... must be confirmed by a measured MFMA
// microbenchmark").  Back-to-back MFMAs with operands in registers on random data (the chip's
// held clock depends on operand toggling: MI355X_MICROARCH.md 'DVFS give-back'), 8 independent
// accumulators per wave, every CU filled.  kind 0: v_mfma_f32_16x16x32_f16 (the f16x3 MLP's
// instruction); kind 1: v_mfma_f32_16x16x4_f32 (the fp32 path's); kind 2: the f16x3 pattern,
// three dependent MFMAs into one accumulator per step; kind 3: v_mfma_f32_32x32x16_f16 (the
// withdrawn 32x32 render MLP's, git e46498b); kind 4: its f16x3 triple.  Returns TFLOP/s of the issued
// MFMAs.
#include <hip/hip_runtime.h>
#include <cstdint>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ float rnd(uint32_t s) { return (mix(s) >> 8) * (1.0f / 16777216.0f) - 0.5f; }

// 32x32x16: 4 independent 16-register accumulators per wave
template <int KIND>
__global__ __launch_bounds__(256) void k_mfma_loop32(int iters, float* out, uint64_t* stamps) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  uint64_t c0 = 0, r0 = 0;
  if (blockIdx.x == gridDim.x / 2 && threadIdx.x == 0) {
    c0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  f16v acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    acc[i] = f16v{};
    acc[i][0] = rnd(t * 8 + i);
  }
  h8 a[2], b[2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      a[i][e] = static_cast<_Float16>(rnd(t * 64 + 16 * i + e));
      b[i][e] = static_cast<_Float16>(rnd(t * 64 + 32 + 16 * i + e));
    }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], b[0], acc[i], 0, 0, 0);
      if (KIND == 4) {
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], b[1], acc[i], 0, 0, 0);
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[1], b[0], acc[i], 0, 0, 0);
      }
    }
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) s += acc[i][r];
  out[t] = s;
  if (blockIdx.x == gridDim.x / 2 && threadIdx.x == 0) {
    stamps[0] = __builtin_amdgcn_s_memtime() - c0;
    stamps[1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}

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
    else if (kind == 2) hipLaunchKernelGGL(k_mfma_loop<2>, blocks, 256, 0, 0, iters, out, stamps);
    else if (kind == 3) hipLaunchKernelGGL(k_mfma_loop32<3>, blocks, 256, 0, 0, iters, out, stamps);
    else hipLaunchKernelGGL(k_mfma_loop32<4>, blocks, 256, 0, 0, iters, out, stamps);
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
  const double per_mfma = kind == 1 ? 2.0 * 16 * 16 * 4 : kind >= 3 ? 2.0 * 32 * 32 * 16 : 2.0 * 16 * 16 * 32;
  const double per_iter = kind == 2 ? 24 : kind == 3 ? 4 : kind == 4 ? 12 : 8;
  const double mfmas = (double)blocks * 4 /* waves */ * iters * per_iter * reps;
  return mfmas * per_mfma / (ms * 1e-3) / 1e12;
}

// ---- the fine MLP's per-wave instruction mix without its dependencies (verdict r04 #5): does the
// chip sustain more than the streamed kernel's ~1.3 GHz-equivalent MFMA rate (MFMA busy x held
// clock) when the same mix -- per MFMA ~1.2 other VALU and ~0.72 ds_read_b128 (the streamed
// kernel's counters: 3,516 MFMA, 4,216 VALU, 2,515 LDS reads per wave) -- has no true
// dependencies?  One 512-thread workgroup per CU (2 waves per SIMD, as k_mlp_fwd_f16x3), random
// fp16 operands, 8 independent accumulators; per iteration 8 MFMAs plus
//   MIX & 1: 10 independent v_fma_f32 (the epilogue's VALU, not fed by the MFMAs),
//   MIX & 2: 6 ds_read_b128 of lane-linear 16-B fragments (the A-fragment reads) whose values
//            become the NEXT iteration's MFMA A operands (a one-iteration prefetch),
//   MIX & 4: 1 ds_write_b128 (the weight ring's refill, 1 write per ~8 reads).
constexpr int kMixLds = 96 * 1024;  // > 80 KB: one workgroup per CU

template <int MIX>
__global__ __launch_bounds__(512) void k_mfma_mix(int iters, float* out, uint64_t* stamps) {
  __shared__ __align__(16) char lds[kMixLds];
  const uint32_t t = blockIdx.x * 512 + threadIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint64_t c0 = 0, r0 = 0;
  if (blockIdx.x == gridDim.x / 2 && threadIdx.x == 0) {
    c0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  for (int i = threadIdx.x; i < kMixLds / 4; i += 512)
    reinterpret_cast<float*>(lds)[i] = rnd(blockIdx.x * kMixLds + i) * 0.25f;
  __syncthreads();
  f4 acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = f4{rnd(t * 8 + i), 0.f, 0.f, 0.f};
  // A fragments in a ring of three register sets: the loads of phase p fill set (p + 2) % 3,
  // read by the MFMAs two phases (16 MFMAs of this wave) later -- a prefetch depth like the
  // streamed kernel's, so the reads are not waited on
  h8 a[3][6], b;
#pragma unroll
  for (int e = 0; e < 8; ++e) b[e] = static_cast<_Float16>(rnd(t * 64 + 48 + e));
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
      for (int e = 0; e < 8; ++e) a[r][i][e] = static_cast<_Float16>(rnd(t * 256 + 48 * r + 8 * i + e));
  float x[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) x[i] = rnd(t * 16 + 100 + i);
  const float cm = 0.999f, ca = 1e-3f;
  // 6 fragments of 1 KB per wave and phase from the wave's own 6 KB (the first 48 KB read, the
  // upper 48 KB written); the base is laundered every phase (an empty asm: no instruction) so
  // the loads stay in the loop with their offsets in the instruction's field
  uint32_t roff = (uint32_t)(wave * 6 * 1024 + lane * 16);
  const uint32_t woff = 48 * 1024 + (uint32_t)(wave * 1024 + lane * 16);
  for (int it = 0; it < iters; it += 3) {
#pragma unroll
    for (int ph = 0; ph < 3; ++ph) {
      if (MIX & 2) {
        asm volatile("" : "+v"(roff));
#pragma unroll
        for (int j = 0; j < 6; ++j)
          a[(ph + 2) % 3][j] = *reinterpret_cast<const h8*>(lds + roff + j * 1024);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i)
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[ph][i % 6], b, acc[i], 0, 0, 0);
      if (MIX & 1) {  // one v_fma_f32 each (asm: hipcc would pair them into v_pk_fma_f32)
#pragma unroll
        for (int i = 0; i < 10; ++i)
          asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(cm), "v"(ca));
      }
      if (MIX & 4)  // a volatile LDS store (address space 3: ds_write_b128) stays in the loop
        *reinterpret_cast<volatile __attribute__((address_space(3))) h8*>(
            static_cast<uint32_t>(reinterpret_cast<uintptr_t>(lds + woff))) = b;
    }
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
#pragma unroll
  for (int i = 0; i < 10; ++i) s += x[i];
  out[t] = s;
  if (blockIdx.x == gridDim.x / 2 && threadIdx.x == 0) {
    stamps[0] = __builtin_amdgcn_s_memtime() - c0;
    stamps[1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}

// issued fp16 MFMA TFLOP/s of k_mfma_mix<mix> over `blocks` workgroups; *clock_ghz = the
// in-kernel clock of the last launch
extern "C" double aon_mfma_mix(int mix, int iters, int blocks, float* out, uint64_t* stamps,
                               double* clock_ghz) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  auto launch = [&]() {
    switch (mix) {
      case 0: hipLaunchKernelGGL(k_mfma_mix<0>, blocks, 512, 0, 0, iters, out, stamps); break;
      case 1: hipLaunchKernelGGL(k_mfma_mix<1>, blocks, 512, 0, 0, iters, out, stamps); break;
      case 2: hipLaunchKernelGGL(k_mfma_mix<2>, blocks, 512, 0, 0, iters, out, stamps); break;
      case 3: hipLaunchKernelGGL(k_mfma_mix<3>, blocks, 512, 0, 0, iters, out, stamps); break;
      default: hipLaunchKernelGGL(k_mfma_mix<7>, blocks, 512, 0, 0, iters, out, stamps); break;
    }
  };
  for (int w = 0; w < 3; ++w) launch();
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
  const double mfmas = (double)blocks * 8 /* waves */ * iters * 8 * reps;
  return mfmas * (2.0 * 16 * 16 * 32) / (ms * 1e-3) / 1e12;
}
