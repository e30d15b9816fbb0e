// Summation orders of torch's CPU fp32 sum kernel (aten/src/ATen/native/cpu/SumKernel.cpp,
// torch 2.10, AVX2 build), so reductions on the GPU round exactly like the reference's
// torch.sum / .sum(dim) calls.  Model validated bit-exactly against torch on every length
// 1..80, 128..1000 (inner and stride-3 outer reductions) before being ported here.
//
//   row_sum_ilp4(x, n): 4 interleaved accumulators (x[4i+k]) with the 16-row cascade of
//       multi_row_sum, leftovers into accumulator 0, then ((P0 + P1) + P2) + P3.
//       = torch's scalar row sum; used for the stride-3 (B,S,3) -> (B,3) rgb sum.
//   inner_sum(x, n): contiguous last-dim sum.  n >= 8: 8-lane vectors v_j = x[8j..8j+7];
//       lane c reduces v_0..v_{m-1} with row_sum_ilp4; result = (tail x[8m..n) summed from 0)
//       + lane0 + ... + lane7.  n < 8: row_sum_ilp4.
#pragma once

namespace aon {

__host__ __device__ inline int ceil_log2_torch(int x) {
  if (x <= 2) return 1;
  int v = x - 1, b = 0;
  while (v) {
    ++b;
    v >>= 1;
  }
  return b;
}

// x(i) for i in [0, n)
template <typename F>
__device__ inline float row_sum_ilp4(F x, int n) {
  const int size_ilp = n / 4;
  int lp = ceil_log2_torch(size_ilp) / 4;
  if (lp < 4) lp = 4;
  const int step = 1 << lp, mask = step - 1;
  float acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[a][k] = 0.f;
  int i = 0;
  while (i + step <= size_ilp) {
    for (int s = 0; s < step; ++s, ++i) {
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[0][k] = __fadd_rn(acc[0][k], x(4 * i + k));
    }
#pragma unroll
    for (int j = 1; j < 4; ++j) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        acc[j][k] = __fadd_rn(acc[j][k], acc[j - 1][k]);
        acc[j - 1][k] = 0.f;
      }
      if ((i & (mask << (j * lp))) != 0) break;
    }
  }
  for (; i < size_ilp; ++i) {
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[0][k] = __fadd_rn(acc[0][k], x(4 * i + k));
  }
  float p[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) p[k] = acc[0][k];
#pragma unroll
  for (int j = 1; j < 4; ++j)
#pragma unroll
    for (int k = 0; k < 4; ++k) p[k] = __fadd_rn(p[k], acc[j][k]);
  for (int e = size_ilp * 4; e < n; ++e) p[0] = __fadd_rn(p[0], x(e));
  return __fadd_rn(__fadd_rn(__fadd_rn(p[0], p[1]), p[2]), p[3]);
}

// lane c (0..7) partial of the vectorised inner sum: row_sum_ilp4 over x[8j + c], j < n/8
template <typename F>
__device__ inline float inner_sum_lane(F x, int n, int c) {
  return row_sum_ilp4([&](int j) { return x(8 * j + c); }, n / 8);
}

template <typename F>
__device__ inline float inner_sum_tail(F x, int n) {
  float s = 0.f;
  for (int e = (n / 8) * 8; e < n; ++e) s = __fadd_rn(s, x(e));
  return s;
}

// whole inner sum in one lane
template <typename F>
__device__ inline float inner_sum(F x, int n) {
  if (n < 8) return row_sum_ilp4(x, n);
  float s = inner_sum_tail(x, n);
  for (int c = 0; c < 8; ++c) s = __fadd_rn(s, inner_sum_lane(x, n, c));
  return s;
}

}  // namespace aon
