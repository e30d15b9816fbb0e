// Exhaustive check of aon::sin_small (aon_common.hpp) against the device sinf on every float
// with |x| < 2^17 (both signs): mismatching bit patterns are counted and the first few printed.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I include -I articulated-object-nerf_amd/csrc \
//     tools/sin_small_check.hip -o tools/sin_small_check && tools/sin_small_check
#include "aon_common.hpp"

namespace aon {
void set_error(const std::string&) {}
}

__global__ void k_check(uint32_t lo, uint32_t hi, unsigned long long* bad, uint32_t* first) {
  for (uint32_t b = lo + blockIdx.x * blockDim.x + threadIdx.x; b < hi; b += gridDim.x * blockDim.x) {
#pragma unroll
    for (int sgn = 0; sgn < 2; ++sgn) {
      const float x = __uint_as_float(b | (sgn ? 0x80000000u : 0u));
      const float a = sinf(x), c = aon::sin_small(x);
      if (__float_as_uint(a) != __float_as_uint(c)) {
        const unsigned long long n = atomicAdd(bad, 1ull);
        if (n < 8) first[n] = __float_as_uint(x);
      }
    }
  }
}

int main() {
  unsigned long long* bad;
  uint32_t* first;
  hipMalloc(&bad, 8);
  hipMalloc(&first, 32);
  hipMemset(bad, 0, 8);
  const uint32_t hi = 0x48000000u;  // 2^17
  hipLaunchKernelGGL(k_check, 65536, 256, 0, 0, 0u, hi, bad, first);
  unsigned long long nb = 0;
  uint32_t f[8] = {};
  hipMemcpy(&nb, bad, 8, hipMemcpyDeviceToHost);
  hipMemcpy(f, first, 32, hipMemcpyDeviceToHost);
  printf("sin_small vs sinf on %llu floats (|x| < 2^17): %llu mismatches\n",
         2ull * hi, nb);
  for (int i = 0; i < 8 && i < (int)nb; ++i) printf("  x bits %08x\n", f[i]);
  return nb == 0 ? 0 : 1;
}
