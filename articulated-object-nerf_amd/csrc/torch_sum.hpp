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

// ---- the same row_sum_ilp4 evaluated by a whole wave ---------------------------------------
// For n < 1024 (size_ilp = n/4 < 256, so lp = 4 and the cascade never reaches acc[2]) the
// sequential loop above decomposes into independent left folds:
//   chunk c < nch = size_ilp/16, accumulator k:  C[c][k] = fold_s x(4(16c + s) + k), s < 16
//   leftover (i in [16 nch, size_ilp)):          L[k]    = fold_i x(4i + k)
//   p[k] = ((L[k] + fold_c C[c][k]) + 0) + 0,  tail x(4 size_ilp ..) into p[0],
//   result ((p0 + p1) + p2) + p3
// -- identical roundings, but every fold is <= 16 terms and they run on different lanes.
// `spec(sp, base, str)` names row sum sp: term j is base[str * j] (LDS); specs [0, nA) have
// nA_terms terms, specs [nA, nA + nB) have nB_terms.  `scratch` holds
// >= nA*4*(nchA+1) + nB*4*(nchB+1) floats and `out` nA + nB floats, both in LDS private to
// this wave.  Every lane of the wave must call; `sync()` orders the wave's LDS traffic.
// Results are visible to all lanes on return.
template <typename Spec, typename Sync>
__device__ inline void wave_row_sums(Spec spec, int nA, int nA_terms, int nB, int nB_terms,
                                     float* scratch, float* out, int lane, Sync sync) {
  const int silA = nA_terms >> 2, nchA = silA >> 4, TA = 4 * (nchA + 1);
  const int silB = nB_terms >> 2, nchB = silB >> 4, TB = 4 * (nchB + 1);
  const int tasksA = nA * TA, ntask = tasksA + nB * TB;
  for (int t = lane; t < ntask; t += 64) {
    int sp, r, sil, nch;
    if (t < tasksA) {
      sp = t / TA;
      r = t - sp * TA;
      sil = silA;
      nch = nchA;
    } else {
      const int q = (t - tasksA) / TB;
      r = t - tasksA - q * TB;
      sp = nA + q;
      sil = silB;
      nch = nchB;
    }
    const float* base;
    int str;
    spec(sp, base, str);
    const int c = r >> 2, k = r & 3, i0 = c << 4;
    const float* x = base + str * (4 * i0 + k);  // term 4(i0 + s) + k = x[s * 4 str]
    const int step = 4 * str;
    float acc = 0.f;
    if (c < nch) {  // full chunk: 16 independent loads, then the ordered adds
      float v[16];
#pragma unroll
      for (int s = 0; s < 16; ++s) v[s] = x[s * step];
#pragma unroll
      for (int s = 0; s < 16; ++s) acc = __fadd_rn(acc, v[s]);
    } else {
      const int cnt = sil - i0;
      for (int s = 0; s < cnt; ++s) acc = __fadd_rn(acc, x[s * step]);
    }
    scratch[t] = acc;
  }
  sync();
  for (int sp = lane; sp < nA + nB; sp += 64) {
    const bool a = sp < nA;
    const int b0 = a ? sp * TA : tasksA + (sp - nA) * TB;
    const int n = a ? nA_terms : nB_terms, sil = a ? silA : silB, nch = a ? nchA : nchB;
    const float* base;
    int str;
    spec(sp, base, str);
    float p[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float a1 = 0.f;
      for (int c = 0; c < nch; ++c) a1 = __fadd_rn(a1, scratch[b0 + 4 * c + k]);
      p[k] = __fadd_rn(__fadd_rn(__fadd_rn(scratch[b0 + 4 * nch + k], a1), 0.f), 0.f);
    }
    for (int e = 4 * sil; e < n; ++e) p[0] = __fadd_rn(p[0], base[str * e]);
    out[sp] = __fadd_rn(__fadd_rn(__fadd_rn(p[0], p[1]), p[2]), p[3]);
  }
  sync();
}

}  // namespace aon
