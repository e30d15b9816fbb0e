// Probe: bf16 pair conversion into h8 fragment slots, as mlp_f16x3_core.hpp's bf16 epilogue does.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
struct Frag { h8 hi[2]; };
__device__ __noinline__ void epi(Frag& out, int pr, int q, float v0, float v1) {
  const bf2 hb = {static_cast<__bf16>(v0), static_cast<__bf16>(v1)};
  out.hi[pr][2 * q] = __builtin_bit_cast(_Float16, hb[0]);
  out.hi[pr][2 * q + 1] = __builtin_bit_cast(_Float16, hb[1]);
}
typedef uint32_t u4 __attribute__((ext_vector_type(4)));
// MODE 0: element extraction (hb[0], hb[1]) bit_cast to _Float16; 1: the pair bit_cast to one
// dword inserted into the h8 viewed as 4 dwords
template <int MODE>
__global__ void k(const float* in, uint16_t* out) {
  Frag f;
  const int t = threadIdx.x;
#pragma unroll
  for (int pr = 0; pr < 2; ++pr)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float a = in[t * 16 + pr * 8 + 2 * q], b = in[t * 16 + pr * 8 + 2 * q + 1];
      const bf2 hb = {static_cast<__bf16>(a), static_cast<__bf16>(b)};
      if (MODE == 0) {
        f.hi[pr][2 * q] = __builtin_bit_cast(_Float16, hb[0]);
        f.hi[pr][2 * q + 1] = __builtin_bit_cast(_Float16, hb[1]);
      } else {
        u4 w = __builtin_bit_cast(u4, f.hi[pr]);
        w[q] = __builtin_bit_cast(uint32_t, hb);
        f.hi[pr] = __builtin_bit_cast(h8, w);
      }
    }
  for (int pr = 0; pr < 2; ++pr) *reinterpret_cast<h8*>(out + t * 16 + pr * 8) = f.hi[pr];
}
static uint16_t bf16_rne(float x) {
  uint32_t u; memcpy(&u, &x, 4);
  u += 0x7fff + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}
int main() {
  const int n = 64 * 16;
  float h[n]; uint16_t r[n];
  for (int i = 0; i < n; ++i) h[i] = 0.37f * i - 11.0f;
  float* din; uint16_t* dout;
  hipMalloc(&din, n * 4); hipMalloc(&dout, n * 2);
  hipMemcpy(din, h, n * 4, hipMemcpyHostToDevice);
  int total = 0;
  for (int mode = 0; mode < 2; ++mode) {
    if (mode == 0) k<0><<<1, 64>>>(din, dout); else k<1><<<1, 64>>>(din, dout);
    hipMemcpy(r, dout, n * 2, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < n; ++i) if (r[i] != bf16_rne(h[i])) { if (bad < 3) printf("mode %d i=%d got %04x want %04x\n", mode, i, r[i], bf16_rne(h[i])); ++bad; }
    printf("bf16 pack probe mode %d: %d mismatches of %d\n", mode, bad, n);
    total += mode == 1 ? bad : 0;
  }
  return total != 0;
}
