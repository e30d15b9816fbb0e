// General fp32-in / fp32-out GEMM on fp16 MFMA with the 3-product hi/lo split (see
// mlp_f16x3.hip for the numerics), for the layer-by-layer training path: the forward layers
// with their activations kept (model.py:95-120), the input-gradient products dX = dY . W and
// the weight gradients dW = dY^T . X of the reference's autograd backward (model.py:256-282).
//
//   C (M x N) = epilogue( A (M x K) . B (K x N) )
//
// Workgroup: 256 threads = 4 waves in 2 x 2, C tile 128 x 128, each wave 64 x 64 = 4 x 4
// MFMA 16x16 tiles with two fp32 accumulators (hi*hi and the 2^11-scaled cross terms: the lo
// parts stay normal in fp16 down to |x * scale| = 2^-14, so a fixed operand scale covers
// gradients over many orders of magnitude).  Per 32-deep k-step the A and B tiles are loaded
// into registers PF steps ahead (the loads fly under the MFMAs; the bias-gradient row sums read
// them only when they are published), split into fp16 hi / lo planes and stored to a
// double-buffered LDS image laid out [row][k] (k contiguous, 80-B rows), from which each lane
// reads its 8-element MFMA fragments with one ds_read_b128; one barrier per k-step.  Operands stored reduction-major (A as [K][M], B as
// [K][N]) are transposed in registers while staging (4 x 4 blocks), so every GEMM of the
// backward pass reads its operands in place.
#include "aon_common.hpp"

#include <type_traits>

namespace aon {
namespace gemm {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));

constexpr int BM = 128, BN = 128, BK = 32, THREADS = 256;
constexpr int ROWH = BK + 8;                 // halves per LDS row: 80 B, 16-B aligned
constexpr int PLANE = BM * ROWH;             // halves per plane (BM == BN)
constexpr int STAGE = 4 * PLANE;             // A hi, A lo, B hi, B lo
constexpr float kLo = 2048.0f;               // lo planes carry (x - hi) * 2^11
constexpr float kInvLo = 1.0f / 2048.0f;
#ifndef AON_GEMM_PF
#define AON_GEMM_PF 1
#endif
constexpr int PF = AON_GEMM_PF;              // k-tiles loaded ahead (register sets)

struct Params {
  int64_t M, N, K;
  const float* A;
  int64_t lda;
  const float* A2;  // a_kc only: columns [K1, K) from A2[(m / a2_rdiv) * lda2 + (k - K1)]
  int64_t lda2, K1, a2_rdiv;
  const float* B;
  int64_t ldb, b_rdiv;  // !b_kc: element (k, n) = B[(k / b_rdiv) * ldb + n]
  float* C;
  int64_t ldc;
  const float* bias;  // per column n
  const float* mask;  // v *= (mask[m * ldm + n] > 0)
  int64_t ldm;
  int relu, accumulate;
  float sa, sb, inv_s;  // operand prescales (powers of two); result * inv_s
  const uint32_t* sa_bits;  // optional: A's scale also times grad_scale(*sa_bits) (per call)
  int64_t kchunk;       // K rows per blockIdx.z (split-K); == K when not split
  float* part;          // split-K partials [z][M][N] (unscaled epilogue-free sums * inv_s)
  float* rowsum;        // !a_kc: rowsum[m] = sum_k A(m, k) (bias gradient of a dW product)
  float* rowsum_part;   // split-K partials [z][M]
  int tiles_m, tiles_n, gm;  // XCD-aware tile order over a 1-D grid.x (see tile_of)
  int zsplit;                // split-K: number of K chunks (1 = not split), see split_of
  int tblocks;               // blocks of one K chunk's tile grid (tile_of's ids, with padding)
  int a_tiled, b_tiled;      // reduction-major operand in the fused training kernels' 16-row
                             // tiled layout (mlp_f16x3_core.hpp act_base; rdiv 1)
  int64_t nstore;            // columns of C written: n < nstore (a zero-padded B, bf16 mode)
  int c_trans;               // C[n * ldc + m]; rowsum = column sums of B (skinny path, aon_gemm_args)
};

// start of the 4-element run (k, row .. row + 3) of a reduction-major operand (row % 4 == 0):
// row-major storage row k / rdiv, or the 16-row tiled layout of the fused training kernels
__device__ __forceinline__ int64_t km_off(int64_t k, int64_t row, int64_t ld, int64_t rdiv,
                                          bool tiled) {
  if (tiled) return (k & ~int64_t(15)) * ld + 256 * (row >> 4) + 16 * (k & 15) + (row & 15);
  // 32-bit division (aon_gemm checks K < 2^32): a 64-bit one is a ~40-instruction sequence
  const int64_t kr = rdiv == 1 ? k : (int64_t)((uint32_t)k / (uint32_t)rdiv);
  return kr * ld + row;
}

// Workgroups are dispatched round-robin over the 8 XCDs (block L -> XCD L mod 8), each with
// its own L2.  The tiles (m, 0..tiles_n-1) that share one A row-block are given block ids
// gm apart -- with gm = 8 the same XCD, dispatched together -- so the A tile is fetched from
// HBM once per XCD: group g of gm m-tiles x tiles_n n-tiles, L = gm tiles_n g + gm n + (m mod gm).
// Grids of fewer than 8 m-tiles (weight gradients) use gm = tiles_m: no padding blocks, which
// would otherwise pile the real tiles onto a few XCDs (measured: 3.5x slower).
// Split-K grids: the tile count T is small (a weight gradient is 2 x 2 tiles) and every K chunk
// is read by the T tiles that share it.  Chunk z's tiles get block ids 8 apart (L = 8 q + x,
// z = 8 (q / T) + x, tile = q mod T): one XCD, dispatched together, so each chunk of both
// operands comes from HBM once and the other tiles hit that XCD's L2.
__device__ __forceinline__ bool split_of(const Params& p, int& tile, int& z) {
  if (p.zsplit <= 1) {
    tile = blockIdx.x;
    z = 0;
    return true;
  }
  const int T = p.tblocks;
  const int L = blockIdx.x, x = L & 7, q = L >> 3;
  z = 8 * (q / T) + x;
  tile = q - (q / T) * T;
  return z < p.zsplit;
}

__device__ __forceinline__ bool tile_of(const Params& p, int L, int& tm, int& tn) {
  const int gsz = p.gm * p.tiles_n;
  const int g = L / gsz, r = L - g * gsz;
  tn = r / p.gm;
  tm = p.gm * g + (r - tn * p.gm);
  return tm < p.tiles_m;
}

__device__ __forceinline__ f4 mfma16(h8 a, h8 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// 4 consecutive k values of one row -> hi / lo halves
__device__ __forceinline__ void split4(f4 v, float s, h4& hi, h4& lo) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float x = v[j] * s;  // power-of-two prescale: exact
    const _Float16 h = static_cast<_Float16>(x);
    hi[j] = h;
    lo[j] = static_cast<_Float16>(__fmul_rn(__fsub_rn(x, static_cast<float>(h)), kLo));
  }
}

// ---- tile loaders: 128 rows x 32 k of one operand into 4 f4 registers per thread -------------
// KC (k-contiguous rows): thread t -> rows (t >> 3) + 32 i, k quad 4 (t & 7).
// KM (k-major storage, rows contiguous): thread t -> rows 16 (t >> 5) + 4 (t & 3) + 0..3, k quad
//     4 ((t >> 2) & 7); register i holds k = kq + i for those 4 rows (transposed when stored).
//     Four lanes cover 64 contiguous bytes of a k row; the stores of a 32-lane half hit rows
//     4 apart in two 16-row groups at 8 k offsets: at most 2-way bank conflicts (80-B rows).
template <bool KC, bool VEC>
struct TileLoad {
  f4 r[4];

  // rows/k outside [0,R) x [k0, kend) read as 0.  KC: k >= K1 from p2 (row / rdiv);
  // KM: storage row k / rdiv.
  __device__ __forceinline__ void load(const float* p, int64_t ld, const float* p2, int64_t ld2,
                                       int64_t K1, int64_t rdiv, int64_t row0, int64_t R,
                                       int64_t k0, int64_t kend, int tid, bool tiled = false) {
    if (KC) {
      const int kq = 4 * (tid & 7);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t row = row0 + (tid >> 3) + 32 * i;
        const int64_t k = k0 + kq;
        f4 v = {0.f, 0.f, 0.f, 0.f};
        if (row < R) {
          if (VEC && k + 3 < kend && k + 3 < K1) {
            v = *reinterpret_cast<const f4*>(p + row * ld + k);
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int64_t kk = k + j;
              if (kk < kend) v[j] = kk < K1 ? p[row * ld + kk] : p2[(row / rdiv) * ld2 + (kk - K1)];
            }
          }
        }
        r[i] = v;
      }
    } else {
      const int kq = 4 * ((tid >> 2) & 7), rq = 16 * (tid >> 5) + 4 * (tid & 3);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t k = k0 + kq + i;
        const int64_t row = row0 + rq;
        f4 v = {0.f, 0.f, 0.f, 0.f};
        if (k < kend) {
          const float* src = p + km_off(k, row, ld, rdiv, tiled);
          if (VEC && row + 3 < R) {
            v = *reinterpret_cast<const f4*>(src);
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (row + j < R) v[j] = src[j];
          }
        }
        r[i] = v;
      }
    }
  }

  // KM only: per-row sums of this thread's 4 k values (rows rq..rq+3), in k order
  __device__ __forceinline__ void add_rows(float (&rs)[4]) const {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      rs[j] = __fadd_rn(rs[j], __fadd_rn(__fadd_rn(__fadd_rn(r[0][j], r[1][j]), r[2][j]), r[3][j]));
  }

  // split and store into the [row][k] hi / lo planes
  __device__ __forceinline__ void store(_Float16* hi, _Float16* lo, float s, int tid) const {
    if (KC) {
      const int kq = 4 * (tid & 7);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = (tid >> 3) + 32 * i;
        h4 h, l;
        split4(r[i], s, h, l);
        *reinterpret_cast<h4*>(hi + row * ROWH + kq) = h;
        *reinterpret_cast<h4*>(lo + row * ROWH + kq) = l;
      }
    } else {
      const int kq = 4 * ((tid >> 2) & 7), rq = 16 * (tid >> 5) + 4 * (tid & 3);
#pragma unroll
      for (int j = 0; j < 4; ++j) {  // row rq + j: k = kq .. kq + 3 from r[0..3][j]
        const f4 v = {r[0][j], r[1][j], r[2][j], r[3][j]};
        h4 h, l;
        split4(v, s, h, l);
        *reinterpret_cast<h4*>(hi + (rq + j) * ROWH + kq) = h;
        *reinterpret_cast<h4*>(lo + (rq + j) * ROWH + kq) = l;
      }
    }
  }
};

template <bool AKC, bool BKC, bool VA, bool VB>
__device__ __forceinline__ void f16x3_body(const Params& p, int tm, int tn, int z, _Float16* smem) {
  // A's prescale: a constant, or per call from the gradient's max |x| (exact powers of two)
  float sa = p.sa, inv_s = p.inv_s;
  if (p.sa_bits) {
    const float gs = grad_scale(*p.sa_bits);
    sa = __fmul_rn(sa, gs);
    inv_s = __fdiv_rn(inv_s, gs);
  }
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int64_t kbeg = (int64_t)z * p.kchunk;
  const int64_t kend = kbeg + p.kchunk < p.K ? kbeg + p.kchunk : p.K;
  const int nk = static_cast<int>((kend - kbeg + BK - 1) / BK);

  // PF register sets: tile kt + 1 waits in one while later tiles' loads fly into the others
  TileLoad<AKC, VA> ta[PF];
  TileLoad<BKC, VB> tb[PF];
  f4 acc_h[4][4], acc_x[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc_h[i][j] = f4{0.f, 0.f, 0.f, 0.f};
      acc_x[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    }

  auto load = [&](int kt, auto set) {
    constexpr int S = decltype(set)::value;
    const int64_t k0 = kbeg + (int64_t)kt * BK;
    ta[S].load(p.A, p.lda, p.A2, p.lda2, p.K1, p.a2_rdiv, m0, p.M, k0, kend, tid, p.a_tiled);
    tb[S].load(p.B, p.ldb, nullptr, 0, INT64_MAX, p.b_rdiv, n0, p.N, k0, kend, tid, p.b_tiled);
  };
  const bool want_rows = !AKC && p.rowsum && tn == 0;
  float rs[4] = {0.f, 0.f, 0.f, 0.f};
  // publish a landed register set to LDS stage `stage` (and add its rows to the row sums, in
  // k-tile order)
  auto store = [&](int stage, auto set) {
    constexpr int S = decltype(set)::value;
    if (!AKC && want_rows) ta[S].add_rows(rs);
    _Float16* s = smem + stage * STAGE;
    ta[S].store(s, s + PLANE, sa, tid);
    tb[S].store(s + 2 * PLANE, s + 3 * PLANE, p.sb, tid);
  };
  using Set0 = std::integral_constant<int, 0>;
  using Set1 = std::integral_constant<int, 1>;

  using SetN = std::integral_constant<int, PF - 1>;
  if (nk > 0) {
    load(0, Set0{});
    if (PF == 2 && nk > 1) load(1, SetN{});
    store(0, Set0{});
  }
  __syncthreads();
  const int g = lane >> 4, r16 = lane & 15;
  // step kt: tile kt is in LDS stage kt & 1 and tile kt + 1 in register set (kt + 1) % PF
  // (PF = 2: loaded last step; PF = 1: loaded now, under this step's MFMAs); tile kt + PF goes
  // into set kt % PF, free since tile kt was published
  auto step = [&](int kt, auto par) {
    constexpr int P = decltype(par)::value;
    using Cur = std::integral_constant<int, P % PF>;
    using Nxt = std::integral_constant<int, (P + 1) % PF>;
    if (kt + PF < nk) load(kt + PF, Cur{});  // global loads in flight under PF steps of MFMAs
    const _Float16* s = smem + P * STAGE;
    h8 bh[4], bl[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = wn * 64 + 16 * j + r16;
      bh[j] = *reinterpret_cast<const h8*>(s + 2 * PLANE + row * ROWH + 8 * g);
      bl[j] = *reinterpret_cast<const h8*>(s + 3 * PLANE + row * ROWH + 8 * g);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wm * 64 + 16 * i + r16;
      const h8 ah = *reinterpret_cast<const h8*>(s + row * ROWH + 8 * g);
      const h8 al = *reinterpret_cast<const h8*>(s + PLANE + row * ROWH + 8 * g);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc_h[i][j] = mfma16(ah, bh[j], acc_h[i][j]);
        acc_x[i][j] = mfma16(ah, bl[j], acc_x[i][j]);
        acc_x[i][j] = mfma16(al, bh[j], acc_x[i][j]);
      }
    }
    if (kt + 1 < nk) store(1 - P, Nxt{});
    __syncthreads();
  };
  for (int kt = 0; kt < nk; kt += 2) {
    step(kt, Set0{});
    if (kt + 1 < nk) step(kt + 1, Set1{});
  }

  const bool split = p.zsplit > 1;
  if (!AKC && want_rows) {
    // combine the 8 k-quad lanes of every row in k order (LDS free after the last barrier)
    float* red = reinterpret_cast<float*>(smem);  // [8 k quads][128 rows]
    const int kqi = (tid >> 2) & 7, rq = 16 * (tid >> 5) + 4 * (tid & 3);
#pragma unroll
    for (int j = 0; j < 4; ++j) red[kqi * BM + rq + j] = rs[j];
    __syncthreads();
    if (tid < BM && m0 + tid < p.M) {
      float v = red[tid];
#pragma unroll
      for (int q = 1; q < 8; ++q) v = __fadd_rn(v, red[q * BM + tid]);
      if (split) p.rowsum_part[(int64_t)z * p.M + m0 + tid] = v;
      else p.rowsum[m0 + tid] = v;
    }
  }

  // ---- epilogue: D lane layout col = lane & 15, rows 4 (lane >> 4) + r
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t n = n0 + wn * 64 + 16 * j + r16;
      if (n >= p.N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t m = m0 + wm * 64 + 16 * i + 4 * g + r;
        if (m >= p.M) continue;
        float v = __fmul_rn(__fadd_rn(acc_h[i][j][r], __fmul_rn(acc_x[i][j][r], kInvLo)), inv_s);
        if (split) {
          p.part[((int64_t)z * p.M + m) * p.N + n] = v;
          continue;
        }
        if (n >= p.nstore) continue;
        float* c = p.C + m * p.ldc + n;
        if (p.accumulate) v = __fadd_rn(*c, v);
        if (p.bias) v = __fadd_rn(v, p.bias[n]);
        if (p.relu) v = fmaxf(v, 0.0f);
        if (p.mask && !(p.mask[m * p.ldm + n] > 0.0f)) v = 0.0f;
        *c = v;
      }
    }
}

template <bool AKC, bool BKC, bool VA, bool VB>
__global__ __launch_bounds__(THREADS, 2) void k_gemm_f16x3(Params p) {
  __shared__ __align__(16) _Float16 smem[2 * STAGE];  // 2 stages x (A hi, A lo, B hi, B lo)
  int tm, tn, tile, z;
  if (!split_of(p, tile, z)) return;      // padding block of the last chunk group
  if (!tile_of(p, tile, tm, tn)) return;  // padding block of the last XCD group (uniform exit)
  f16x3_body<AKC, BKC, VA, VB>(p, tm, tn, z, smem);
}

// split-K: C = epilogue(sum_z part[z]) in z order (deterministic); rowsum likewise.  The loads
// of 8 consecutive z are issued before their (in-order) adds: a thread walks up to 256 partials
// spaced M*N apart, and one load at a time left this kernel latency-bound (~50 us at any size).
__device__ __forceinline__ float sum_z(const float* src, int64_t stride, int splits) {
  float v = src[0];
  int z = 1;
  for (; z + 8 <= splits; z += 8) {
    float t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) t[u] = src[(int64_t)(z + u) * stride];
#pragma unroll
    for (int u = 0; u < 8; ++u) v = __fadd_rn(v, t[u]);
  }
  for (; z < splits; ++z) v = __fadd_rn(v, src[(int64_t)z * stride]);
  return v;
}

// Four lanes per output: lane q sums the partials of the q-th quarter of the chunks in z order,
// then the quarters combine as (q0 + q1) + (q2 + q3) -- a fixed order (deterministic), a quarter
// of the dependent load rounds per thread and 4x the threads of a one-lane-per-output reduce
// (whose 256 workgroups of sequential partial loads took ~11 us per weight gradient).
__device__ __forceinline__ float sum_z4(const float* src, int64_t stride, int splits, int q) {
  const int zq = (splits + 3) / 4;
  const int z0 = q * zq, z1 = z0 + zq < splits ? z0 + zq : splits;
  float v = 0.f;
  if (z0 < z1) v = sum_z(src + (int64_t)z0 * stride, stride, z1 - z0);
  const float w = __shfl_xor(v, 1, 64);  // lanes 4e + q: q0 + q1 and q2 + q3
  const float pair = (q & 1) ? __fadd_rn(w, v) : __fadd_rn(v, w);
  const float other = __shfl_xor(pair, 2, 64);
  return (q & 2) ? __fadd_rn(other, pair) : __fadd_rn(pair, other);
}

// Sixteen lanes per output (the small products -- heads, segment sums -- whose few hundred
// outputs each sum 256-512 chunks: at 4 lanes they ran on ~6 workgroups in 16 dependent load
// rounds, ~8-11 us): lane q sums the q-th sixteenth in z order, then a fixed xor tree combines
// them, lower lane first at every level (deterministic).
__device__ __forceinline__ float sum_z16(const float* src, int64_t stride, int splits, int q) {
  const int zq = (splits + 15) / 16;
  const int z0 = q * zq, z1 = z0 + zq < splits ? z0 + zq : splits;
  float v = 0.f;
  if (z0 < z1) v = sum_z(src + (int64_t)z0 * stride, stride, z1 - z0);
#pragma unroll
  for (int b = 1; b < 16; b <<= 1) {
    const float w = __shfl_xor(v, b, 64);
    v = (q & b) ? __fadd_rn(w, v) : __fadd_rn(v, w);
  }
  return v;
}

template <int L>
__device__ __forceinline__ void reduce_body(const Params& p, int splits) {
  static_assert(L == 4 || L == 16, "lanes per output");
  constexpr int kSh = L == 4 ? 2 : 4;
  const int64_t total = p.M * p.N;
  const int64_t nrs = p.c_trans ? p.N : p.M;  // rowsum entries: row sums of A, or B's column sums
  const int64_t extra = p.rowsum ? nrs : 0;   // they ride along as e >= total
  const int q = threadIdx.x & (L - 1);
  const int64_t nthreads = (int64_t)gridDim.x * blockDim.x;
  auto sum = [&](const float* src, int64_t stride) {
    return L == 4 ? sum_z4(src, stride, splits, q) : sum_z16(src, stride, splits, q);
  };
  // every lane of a wave takes part in the shuffles: the loop bound is per group of L lanes and
  // the grid stride a multiple of L, so a group's lanes run the same iterations
  for (int64_t eL = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; (eL >> kSh) < total + extra;
       eL += nthreads) {
    const int64_t e = eL >> kSh;
    if (e >= total) {
      const int64_t m = e - total;
      const float v = sum(p.rowsum_part + m, nrs);
      if (q == 0) p.rowsum[m] = v;
      continue;
    }
    const int64_t m = e / p.N, n = e - m * p.N;
    float v = sum(p.part + e, total);
    if (q != 0 || n >= p.nstore) continue;
    float* c = p.C + (p.c_trans ? n * p.ldc + m : m * p.ldc + n);
    if (p.accumulate) v = __fadd_rn(*c, v);
    if (p.bias) v = __fadd_rn(v, p.bias[n]);
    if (p.relu) v = fmaxf(v, 0.0f);
    if (p.mask && !(p.mask[m * p.ldm + n] > 0.0f)) v = 0.0f;
    *c = v;
  }
}

template <int L>
__global__ void k_gemm_reduce(Params p, int splits) { reduce_body<L>(p, splits); }
#ifndef AON_GEMM_REDUCE16
#define AON_GEMM_REDUCE16 1  // 0: A/B build -- the small products' reduce at 4 lanes per output
#endif

// aon_gemm_batch: up to AON_GEMM_BATCH_MAX products in one launch, selected by a wave-uniform
// index into the kernel-argument table
struct ParamsBatch {
  Params p[AON_GEMM_BATCH_MAX];
  int count, zsplit;
  int tile0[AON_GEMM_BATCH_MAX + 1];  // 128 x 128-tile batch: first tile of each product
};

static_assert(sizeof(ParamsBatch) <= 4096, "aon_gemm_batch's table must fit the kernel arguments");

// the batch's split-K reduce: grid.y = product
__global__ void k_gemm_reduce_batch(ParamsBatch pb) { reduce_body<4>(pb.p[blockIdx.y], pb.zsplit); }

// fp16x3 weight gradients of one level (aon_gemm_batch): every product's 128 x 128 tiles, chunk z
// of all of them on one XCD (split_of's order), product b owning tiles tile0[b] .. tile0[b+1]-1
__global__ __launch_bounds__(THREADS, 2) void k_gemm_f16x3_batch(ParamsBatch pb) {
  __shared__ __align__(16) _Float16 smem[2 * STAGE];
  const int T = pb.tile0[pb.count], L = blockIdx.x, x = L & 7, q = L >> 3;
  const int z = 8 * (q / T) + x, t = q - (q / T) * T;
  if (z >= pb.zsplit) return;  // padding block of the last chunk group (uniform exit)
  int b = 0;
  while (b + 1 < pb.count && t >= pb.tile0[b + 1]) ++b;
  const Params& p = pb.p[b];
  const int lt = t - pb.tile0[b];
  f16x3_body<false, false, true, true>(p, lt % p.tiles_m, lt / p.tiles_m, z, smem);
}

template <bool AKC, bool BKC, bool VA, bool VB>
static void launch(const Params& p, dim3 grid, hipStream_t st) {
  hipLaunchKernelGGL((k_gemm_f16x3<AKC, BKC, VA, VB>), grid, dim3(THREADS), 0, st, p);
}

template <bool AKC, bool BKC>
static void launch_v(const Params& p, bool va, bool vb, dim3 grid, hipStream_t st) {
  if (va && vb) launch<AKC, BKC, true, true>(p, grid, st);
  else if (va) launch<AKC, BKC, true, false>(p, grid, st);
  else if (vb) launch<AKC, BKC, false, true>(p, grid, st);
  else launch<AKC, BKC, false, false>(p, grid, st);
}


// ---- bf16 mode (the C5 training step's bf16 precision): weight-gradient products
// C (M x N) (+)= A^T B over K rows with both operands reduction-major (A = dY [K][M], B = X
// [K][N], row k of B at (k / b_rdiv) * ldb), each element fp32 or bf16 (template), rounded to
// bf16 while staging; ONE v_mfma_f32_16x16x32_bf16 per 16x16x32 step (fp32 accumulate) where
// the f16x3 kernel issues three.  Same tile grid, XCD-aware order, split-K and deterministic
// reduction as k_gemm_f16x3; rowsum = the fp32 sums of A's staged values (bias gradients).
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf4 __attribute__((ext_vector_type(4)));
constexpr int STAGE_BF = 2 * PLANE;  // A, B planes of bf16 (same [row][k] geometry)

template <typename T>
__device__ __forceinline__ float to_f32(T v) { return static_cast<float>(v); }

// Strength-reduced addressing of a thread's runs in full k-tiles of a reduction-major operand
// (rdiv 1): the run of k-tile kt, k row i, starts at run + kt * tstep + i * istep elements
// (row-major: istep = ld; tiled: 16), so a full tile costs no 64-bit index arithmetic (the
// per-element km_off path left the bf16 kernel VALU-bound).  One per operand, shared by the
// register sets.
struct KmRun {
  const void* run;
  int64_t tstep, istep;
  bool fast;
  template <typename T>
  __device__ __forceinline__ KmRun(const T* p, int64_t ld, int64_t rdiv, int64_t row0, int64_t R,
                                   int64_t kbeg, int tid, bool tiled, bool vec) {
    const int kq = 4 * ((tid >> 2) & 7), rq = 16 * (tid >> 5) + 4 * (tid & 3);
    fast = vec && rdiv == 1 && row0 + rq + 3 < R;
    run = p + (fast ? km_off(kbeg + kq, row0 + rq, ld, 1, tiled) : 0);
    tstep = BK * ld;
    istep = tiled ? 16 : ld;
  }
};

// 128 rows x 32 k of a reduction-major operand: thread t -> rows rq..rq+3 (rq = 16 (t >> 5) +
// 4 (t & 3)), k = kq..kq+3 (kq = 4 ((t >> 2) & 7)); one 4-element row run per k
template <typename T, bool VEC>
struct TileLoadKM {
  float r[4][4];  // [k][row]
  __device__ __forceinline__ void load(const T* p, int64_t ld, int64_t rdiv, int64_t row0,
                                       int64_t R, int64_t k0, int64_t kend, int tid, bool tiled,
                                       const KmRun&, int) {
    const int kq = 4 * ((tid >> 2) & 7), rq = 16 * (tid >> 5) + 4 * (tid & 3);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t k = k0 + kq + i;
      const int64_t row = row0 + rq;
#pragma unroll
      for (int j = 0; j < 4; ++j) r[i][j] = 0.f;
      if (k < kend) {
        const T* src = p + km_off(k, row, ld, rdiv, tiled);
        if (VEC && row + 3 < R) {
          if (sizeof(T) == 4) {
            const f4 v = *reinterpret_cast<const f4*>(src);
#pragma unroll
            for (int j = 0; j < 4; ++j) r[i][j] = v[j];
          } else {
            const bf4 v = *reinterpret_cast<const bf4*>(src);
#pragma unroll
            for (int j = 0; j < 4; ++j) r[i][j] = static_cast<float>(v[j]);
          }
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (row + j < R) r[i][j] = to_f32(src[j]);
        }
      }
    }
  }
  // rows' sums of this thread's 4 k values, in k order (of the bf16-rounded values)
  __device__ __forceinline__ void add_rows(float (&rs)[4]) const {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = static_cast<float>(static_cast<__bf16>(r[i][j]));
      rs[j] = __fadd_rn(rs[j], __fadd_rn(__fadd_rn(__fadd_rn(v[0], v[1]), v[2]), v[3]));
    }
  }
  // transposed into the [row][k] bf16 plane: row rq + j gets k = kq .. kq + 3 (one 8-B store)
  __device__ __forceinline__ void store(__bf16* plane, int tid) const {
    const int kq = 4 * ((tid >> 2) & 7), rq = 16 * (tid >> 5) + 4 * (tid & 3);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bf4 v = {static_cast<__bf16>(r[0][j]), static_cast<__bf16>(r[1][j]),
                     static_cast<__bf16>(r[2][j]), static_cast<__bf16>(r[3][j])};
      *reinterpret_cast<bf4*>(plane + (rq + j) * ROWH + kq) = v;
    }
  }
};

// The same tile from a bf16 source, kept as raw 16-bit lanes (no fp32 round trip): 4 rows of
// each k are one 8-B load, and the 4 x 4 transpose into [row][k] is 2 v_perm_b32 per row.
template <bool VEC>
struct TileLoadKMb {
  uint2 r[4];  // r[i]: rows rq..rq+3 at k = kq + i (bf16 bits, two per dword)
  __device__ __forceinline__ void load(const __bf16* p, int64_t ld, int64_t rdiv, int64_t row0,
                                       int64_t R, int64_t k0, int64_t kend, int tid, bool tiled,
                                       const KmRun& a, int kt) {
    if (a.fast && k0 + BK <= kend) {
      const uint16_t* src = reinterpret_cast<const uint16_t*>(a.run) + kt * a.tstep;
      const int64_t istep = a.istep;
#pragma unroll
      for (int i = 0; i < 4; ++i) r[i] = *reinterpret_cast<const uint2*>(src + i * istep);
      return;
    }
    const int kq = 4 * ((tid >> 2) & 7), rq = 16 * (tid >> 5) + 4 * (tid & 3);
    const uint16_t* q = reinterpret_cast<const uint16_t*>(p);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t k = k0 + kq + i;
      const int64_t row = row0 + rq;
      uint2 v = {0u, 0u};
      if (k < kend) {
        const uint16_t* src = q + km_off(k, row, ld, rdiv, tiled);
        if (VEC && row + 3 < R) {
          v = *reinterpret_cast<const uint2*>(src);
        } else {
          uint32_t e[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) e[j] = row + j < R ? src[j] : 0u;
          v = uint2{e[0] | (e[1] << 16), e[2] | (e[3] << 16)};
        }
      }
      r[i] = v;
    }
  }
  __device__ __forceinline__ static float elem(uint2 v, int j) {  // bf16 -> fp32: exact shift
    const uint32_t w = (j >> 1) ? v.y : v.x;
    return __uint_as_float((j & 1) ? (w & 0xffff0000u) : (w << 16));
  }
  __device__ __forceinline__ void add_rows(float (&rs)[4]) const {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      rs[j] = __fadd_rn(rs[j], __fadd_rn(__fadd_rn(__fadd_rn(elem(r[0], j), elem(r[1], j)),
                                                   elem(r[2], j)), elem(r[3], j)));
  }
  __device__ __forceinline__ void store(__bf16* plane, int tid) const {
    const int kq = 4 * ((tid >> 2) & 7), rq = 16 * (tid >> 5) + 4 * (tid & 3);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      // half (j & 1) of dword (j >> 1) of each k: [k0 | k1 << 16], [k2 | k3 << 16]
      const uint32_t sel = (j & 1) ? 0x07060302u : 0x05040100u;
      const uint32_t d0 = (j >> 1) ? r[0].y : r[0].x, d1 = (j >> 1) ? r[1].y : r[1].x;
      const uint32_t d2 = (j >> 1) ? r[2].y : r[2].x, d3 = (j >> 1) ? r[3].y : r[3].x;
      const uint2 o = {__builtin_amdgcn_perm(d1, d0, sel), __builtin_amdgcn_perm(d3, d2, sel)};
      *reinterpret_cast<uint2*>(plane + (rq + j) * ROWH + kq) = o;
    }
  }
};

template <typename T, bool VEC>
struct KMLoader {
  using type = TileLoadKM<T, VEC>;
};
template <bool VEC>
struct KMLoader<__bf16, VEC> {
  using type = TileLoadKMb<VEC>;
};

// f(integral_constant<I>) for I = B .. E-1 (compile-time register-set indices)
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

#ifndef AON_GEMM_BF_PF
#define AON_GEMM_BF_PF 2  // 1 / 2 / 3 / 4 measured equal (profiles/r02/ab_gemm)
#endif
constexpr int PFB = AON_GEMM_BF_PF;  // k-tiles in registers ahead of the one in LDS

#ifndef AON_GEMM_BF_OCC
#define AON_GEMM_BF_OCC 2  // waves per SIMD the bf16 kernel is built for
#endif

template <typename TA, typename TB, bool VA, bool VB>
__global__ __launch_bounds__(THREADS, AON_GEMM_BF_OCC) void k_gemm_bf16_km(Params p) {
  __shared__ __align__(16) __bf16 smem[2 * STAGE_BF];  // 2 stages x (A, B)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  int tm, tn, tile, z;
  if (!split_of(p, tile, z)) return;
  if (!tile_of(p, tile, tm, tn)) return;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int64_t kbeg = (int64_t)z * p.kchunk;
  const int64_t kend = kbeg + p.kchunk < p.K ? kbeg + p.kchunk : p.K;
  const int nk = static_cast<int>((kend - kbeg + BK - 1) / BK);
  const TA* A = reinterpret_cast<const TA*>(p.A);
  const TB* Bm = reinterpret_cast<const TB*>(p.B);
  // PFB register sets: tile kt + 1 is published from its set at the end of step kt, and the
  // set tile kt came from takes tile kt + PFB -- every load has PFB - 1 steps of MFMAs to land
  // (one set left the kernel waiting on each tile's global load: 0.37 ms per fine-level dW)
  typename KMLoader<TA, VA>::type ta[PFB];
  typename KMLoader<TB, VB>::type tb[PFB];
  const KmRun ra(A, p.lda, 1, m0, p.M, kbeg, tid, p.a_tiled, VA && sizeof(TA) == 2);
  const KmRun rb(Bm, p.ldb, p.b_rdiv, n0, p.N, kbeg, tid, p.b_tiled, VB && sizeof(TB) == 2);
  f4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  const bool want_rows = p.rowsum && tn == 0;
  float rs[4] = {0.f, 0.f, 0.f, 0.f};
  auto load = [&](int kt, auto set) {
    constexpr int S = decltype(set)::value;
    const int64_t k0 = kbeg + (int64_t)kt * BK;
    ta[S].load(A, p.lda, 1, m0, p.M, k0, kend, tid, p.a_tiled, ra, kt);
    tb[S].load(Bm, p.ldb, p.b_rdiv, n0, p.N, k0, kend, tid, p.b_tiled, rb, kt);
  };
  auto store = [&](int stage, auto set) {
    constexpr int S = decltype(set)::value;
    if (want_rows) ta[S].add_rows(rs);
    __bf16* s = smem + stage * STAGE_BF;
    ta[S].store(s, tid);
    tb[S].store(s + PLANE, tid);
  };
  const int g = lane >> 4, r16 = lane & 15;
  // step kt: tile kt in LDS stage kt & 1, set (kt % PFB) free for tile kt + PFB
  auto step = [&](int kt, auto set) {
    constexpr int S = decltype(set)::value;
#ifndef AON_GEMM_ABL_NOLOAD  // timing-only ablations (wrong results)
    if (kt + PFB < nk) load(kt + PFB, set);
#endif
    const __bf16* s = smem + (kt & 1) * STAGE_BF;
    bf8 b[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      b[j] = *reinterpret_cast<const bf8*>(s + PLANE + (wn * 64 + 16 * j + r16) * ROWH + 8 * g);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bf8 a = *reinterpret_cast<const bf8*>(s + (wm * 64 + 16 * i + r16) * ROWH + 8 * g);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#ifndef AON_GEMM_ABL_NOMFMA
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[j], acc[i][j], 0, 0, 0);
#else
        acc[i][j][0] += static_cast<float>(a[0]) * static_cast<float>(b[j][0]);
#endif
    }
#ifndef AON_GEMM_ABL_NOSTORE
    if (kt + 1 < nk) store(1 - (kt & 1), std::integral_constant<int, (S + 1) % PFB>{});
#endif
#ifndef AON_GEMM_ABL_NOSYNC
    __syncthreads();
#endif
  };
  // prologue: tiles 0 .. PFB-1 in flight, tile 0 published
  static_for<0, PFB>([&](auto set) {
    if (decltype(set)::value < nk) load(decltype(set)::value, set);
  });
  if (nk > 0) store(0, std::integral_constant<int, 0>{});
  __syncthreads();
  for (int kt = 0; kt < nk; kt += PFB) {
    static_for<0, PFB>([&](auto set) {
      if (kt + decltype(set)::value < nk) step(kt + decltype(set)::value, set);
    });
  }
  const bool split = p.zsplit > 1;
  if (want_rows) {
    float* red = reinterpret_cast<float*>(smem);  // [8 k quads][128 rows]
    const int kqi = (tid >> 2) & 7, rq = 16 * (tid >> 5) + 4 * (tid & 3);
#pragma unroll
    for (int j = 0; j < 4; ++j) red[kqi * BM + rq + j] = rs[j];
    __syncthreads();
    if (tid < BM && m0 + tid < p.M) {
      float v = red[tid];
#pragma unroll
      for (int q = 1; q < 8; ++q) v = __fadd_rn(v, red[q * BM + tid]);
      if (split) p.rowsum_part[(int64_t)z * p.M + m0 + tid] = v;
      else p.rowsum[m0 + tid] = v;
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t n = n0 + wn * 64 + 16 * j + r16;
      if (n >= p.N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t m = m0 + wm * 64 + 16 * i + 4 * g + r;
        if (m >= p.M) continue;
        float v = acc[i][j][r];
        if (split) {
          p.part[((int64_t)z * p.M + m) * p.N + n] = v;
          continue;
        }
        if (n >= p.nstore) continue;
        float* c = p.C + m * p.ldc + n;
        if (p.accumulate) v = __fadd_rn(*c, v);
        *c = v;
      }
    }
}

// ---- bf16 x bf16 weight gradients with both operands bf16 and reduction-major (the bf16
// training mode's dW = dZ^T H on the fused kernels' tiled tensors, or row-major), M and N
// multiples of 128.  The k-tile of each operand is copied, not transposed, while staging: a
// thread loads two contiguous 16-B runs (8 columns of one k row; a wave reads 1 KB contiguous
// in the tiled layout) and writes them as they are into a [k][128 columns] LDS image (XOR-
// swizzled 16-B chunks, cdna_hip_programming.md T10 (b)); the MFMA fragments, 8 consecutive k
// of one column, come out of ds_read_b64_tr_b16 (the hardware transpose read).  The
// transposing loader of k_gemm_bf16_km (4 x 8-B loads scattered over 32-B pieces per thread)
// held it at 0.34 ms per fine-level product: global loads, not MFMA or LDS, set its pace.
typedef short tt_v4s __attribute__((ext_vector_type(4)));
constexpr int TT_PLANE = BK * 256;  // bytes of one operand's [32 k][128 col] bf16 image

__device__ __forceinline__ int tt_off(int row, int ch) {  // byte offset of 16-B chunk ch of row
  return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

// a thread's two 16-B runs of every k-tile of one operand: run j = k row kl0 + 16 j, columns
// cl .. cl + 7 of the workgroup tile; element offsets from the operand's base
struct TTRun {
  const uint16_t* base;  // run 0 of k-tile 0
  int64_t jstep, tstep;  // run 1 - run 0, k-tile t+1 - k-tile t (elements)
  int kl0, cl;
  __device__ __forceinline__ TTRun(const __bf16* p, int64_t ld, int64_t col0, int64_t kbeg,
                                   int tid, bool tiled) {
    if (tiled) {  // memory order within a 16-row block's 4-KB column range: [tile][row][half]
      const int T = tid >> 5, s = (tid >> 1) & 15, h = tid & 1;
      kl0 = s;
      cl = 16 * T + 8 * h;
      base = reinterpret_cast<const uint16_t*>(p) + kbeg * ld + 256 * ((col0 >> 4) + T) + 16 * s + 8 * h;
    } else {
      kl0 = tid >> 4;
      cl = 8 * (tid & 15);
      base = reinterpret_cast<const uint16_t*>(p) + (kbeg + kl0) * ld + col0 + cl;
    }
    jstep = 16 * ld;
    tstep = BK * ld;
  }
};

struct TTSet {
  uint4 v[2];
  __device__ __forceinline__ void load(const TTRun& r, int kt, int64_t k0, int64_t kend) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      v[j] = uint4{0u, 0u, 0u, 0u};
      if (k0 + r.kl0 + 16 * j < kend)
        v[j] = *reinterpret_cast<const uint4*>(r.base + kt * r.tstep + j * r.jstep);
    }
  }
  __device__ __forceinline__ void store(char* plane, const TTRun& r) const {
#pragma unroll
    for (int j = 0; j < 2; ++j)
      *reinterpret_cast<uint4*>(plane + tt_off(r.kl0 + 16 * j, r.cl >> 3)) = v[j];
  }
  // column sums of the run values (bf16 -> fp32 exact), runs in k order
  __device__ __forceinline__ void add_cols(float (&rs)[8]) const {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const uint32_t w[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const uint32_t d = w[e >> 1];
        rs[e] = __fadd_rn(rs[e], __uint_as_float((e & 1) ? (d & 0xffff0000u) : (d << 16)));
      }
    }
  }
};

// 8 consecutive k (rows 8 g .. 8 g + 7 of the image) of column c0 * 8 + (lane & 15): two
// transposed reads of 4 rows x 16 columns each (lane 4 q + p addresses row q, columns 4 p..)
__device__ __forceinline__ bf8 tt_frag(const char* plane, int c0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  tt_v4s h[2];
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    const char* a = plane + tt_off(8 * g + 4 * hh + q, c0 + (p >> 1)) + 8 * (p & 1);
    h[hh] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        reinterpret_cast<__attribute__((address_space(3))) tt_v4s*>(
            reinterpret_cast<uintptr_t>(a)));
  }
  typedef short v8s __attribute__((ext_vector_type(8)));
  const v8s w = {h[0][0], h[0][1], h[0][2], h[0][3], h[1][0], h[1][1], h[1][2], h[1][3]};
  return __builtin_bit_cast(bf8, w);
}

__global__ __launch_bounds__(THREADS, 2) void k_gemm_bf16_tt(Params p) {
  __shared__ __align__(16) char smem[2 * 2 * TT_PLANE];  // 2 stages x (A, B) images
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  int tm, tn, tile, z;
  if (!split_of(p, tile, z)) return;
  if (!tile_of(p, tile, tm, tn)) return;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int64_t kbeg = (int64_t)z * p.kchunk;
  const int64_t kend = kbeg + p.kchunk < p.K ? kbeg + p.kchunk : p.K;
  const int nk = static_cast<int>((kend - kbeg + BK - 1) / BK);
  const TTRun ra(reinterpret_cast<const __bf16*>(p.A), p.lda, m0, kbeg, tid, p.a_tiled);
  const TTRun rb(reinterpret_cast<const __bf16*>(p.B), p.ldb, n0, kbeg, tid, p.b_tiled);
  TTSet ta[PFB], tb[PFB];
  f4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  const bool want_rows = p.rowsum && tn == 0;
  float rs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  auto load = [&](int kt, auto set) {
    constexpr int S = decltype(set)::value;
    const int64_t k0 = kbeg + (int64_t)kt * BK;
    ta[S].load(ra, kt, k0, kend);
    tb[S].load(rb, kt, k0, kend);
  };
  auto store = [&](int stage, auto set) {
    constexpr int S = decltype(set)::value;
    if (want_rows) ta[S].add_cols(rs);
    char* s = smem + stage * 2 * TT_PLANE;
    ta[S].store(s, ra);
    tb[S].store(s + TT_PLANE, rb);
  };
  auto step = [&](int kt, auto set) {
    constexpr int S = decltype(set)::value;
    if (kt + PFB < nk) load(kt + PFB, set);
    const char* s = smem + (kt & 1) * 2 * TT_PLANE;
    bf8 b[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = tt_frag(s + TT_PLANE, 8 * wn + 2 * j, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bf8 a = tt_frag(s, 8 * wm + 2 * i, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) store(1 - (kt & 1), std::integral_constant<int, (S + 1) % PFB>{});
    __syncthreads();
  };
  static_for<0, PFB>([&](auto set) {
    if (decltype(set)::value < nk) load(decltype(set)::value, set);
  });
  if (nk > 0) store(0, std::integral_constant<int, 0>{});
  __syncthreads();
  for (int kt = 0; kt < nk; kt += PFB) {
    static_for<0, PFB>([&](auto set) {
      if (kt + decltype(set)::value < nk) step(kt + decltype(set)::value, set);
    });
  }
  const bool split = p.zsplit > 1;
  if (want_rows) {
    // the 16 threads sharing a column range hold k rows kl0 (+ 16 j + 32 kt): summed in kl0 order
    float* red = reinterpret_cast<float*>(smem);  // [16][128]
#pragma unroll
    for (int e = 0; e < 8; ++e) red[ra.kl0 * BM + ra.cl + e] = rs[e];
    __syncthreads();
    if (tid < BM) {
      float v = red[tid];
#pragma unroll
      for (int q = 1; q < 16; ++q) v = __fadd_rn(v, red[q * BM + tid]);
      if (split) p.rowsum_part[(int64_t)z * p.M + m0 + tid] = v;
      else p.rowsum[m0 + tid] = v;
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t n = n0 + wn * 64 + 16 * j + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t m = m0 + wm * 64 + 16 * i + 4 * (lane >> 4) + r;
        float v = acc[i][j][r];
        if (split) {
          p.part[((int64_t)z * p.M + m) * p.N + n] = v;
          continue;
        }
        if (n >= p.nstore) continue;
        float* c = p.C + m * p.ldc + n;
        if (p.accumulate) v = __fadd_rn(*c, v);
        *c = v;
      }
    }
}

// ---- the same product with the operand tiles copied HBM/L2 -> LDS by global_load_lds_dwordx4
// (no register staging): a DNB-deep ring of [32 k][128 col] image pairs, DNB - 1 k-tiles in
// flight ahead of the one in use.  The register-staged kernel above kept ~2 MB in flight
// chip-wide (PMC: 1,363-cycle HBM queue latency, 3.2 TB/s); the ring keeps DNB - 1 tiles of
// 16 KB per workgroup in flight.  The LDS image is lane-linear per copy (lane i of a wave's
// copy lands at 16 i), so the XOR swizzle is applied on the global side: lane i fetches the
// logical chunk that belongs at its physical slot.  A k-tile past the end of the reduction
// (only the last one of the last chunk) goes through registers with zero fill.
#ifndef AON_GEMM_BF_DMA
#define AON_GEMM_BF_DMA 1  // 0: the register-staged copy kernel k_gemm_bf16_tt (A/B)
#endif
#ifndef AON_GEMM_DMA_NBUF
#define AON_GEMM_DMA_NBUF 3  // 2 / 4: within 2-10%, 6: 50% slower (profiles/r02/ab_gemm)
#endif
constexpr int DNB = AON_GEMM_DMA_NBUF;

// s_waitcnt vmcnt(n) (lgkmcnt, expcnt untouched); n a small constant after unrolling
__device__ __forceinline__ void dma_wait_vm(int n) {
#define AON_DW(n_) __builtin_amdgcn_s_waitcnt(((n_) & 0xF) | (((n_) >> 4) << 14) | (0x7 << 4) | (0xF << 8))
  switch (n) {
    case 0: AON_DW(0); break;
    case 1: AON_DW(1); break;
    case 2: AON_DW(2); break;
    case 3: AON_DW(3); break;
    case 4: AON_DW(4); break;
    case 5: AON_DW(5); break;
    case 6: AON_DW(6); break;
    case 7: AON_DW(7); break;
    case 8: AON_DW(8); break;
    case 9: AON_DW(9); break;
    case 10: AON_DW(10); break;
    case 11: AON_DW(11); break;
    default: AON_DW(12); break;
  }
#undef AON_DW
}

// one operand's copies: lane `lane` of wave w, copy c (0, 1) fills image row r = 8 w + 4 c +
// lane / 16, physical chunk lane % 16 <- logical chunk (lane % 16) ^ swz(r)
struct DmaOperand {
  const char* gbase;  // byte address of k-tile 0's (row 0, column col0) origin, kbeg applied
  int64_t tstep;      // bytes between k-tiles
  uint32_t voff[2];   // per-lane byte offset of copy c within a k-tile
  __device__ __forceinline__ DmaOperand(const __bf16* p, int64_t ld, int64_t col0, int64_t kbeg,
                                        int wave, int lane, bool tiled) {
    gbase = reinterpret_cast<const char*>(p) + 2 * (kbeg * ld + (tiled ? 16 * col0 : col0));
    tstep = 2 * BK * ld;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int r = 8 * wave + 4 * c + (lane >> 4);
      const int ch = (lane & 15) ^ (((r & 3) << 2) | ((r >> 2) & 3));
      const int64_t e = tiled ? (int64_t)(r & 16) * ld + 256 * (ch >> 1) + 16 * (r & 15) + 8 * (ch & 1)
                              : (int64_t)r * ld + 8 * ch;
      voff[c] = static_cast<uint32_t>(2 * e);
    }
  }
  // copy k-tile kt into the image at LDS byte address `plane` (this wave's rows)
  __device__ __forceinline__ void issue(uint32_t plane, int wave, int kt) const {
    const char* g = gbase + kt * tstep;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const uint32_t m0 = __builtin_amdgcn_readfirstlane(plane + 256u * (8 * wave + 4 * c));
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
      asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, %2"
                   :
                   : "s"(m0), "v"(voff[c]), "s"(g)
                   : "memory", "m0");
#pragma clang diagnostic pop
    }
  }
  // the same copies through registers, rows at or past `rows_left` zero (the ragged last tile)
  __device__ __forceinline__ void issue_ragged(char* plane, int wave, int lane, int kt,
                                               int64_t rows_left) const {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int r = 8 * wave + 4 * c + (lane >> 4);
      uint4 v = {0u, 0u, 0u, 0u};
      if (r < rows_left) v = *reinterpret_cast<const uint4*>(gbase + kt * tstep + voff[c]);
      *reinterpret_cast<uint4*>(plane + 256 * (8 * wave + 4 * c) + 16 * lane) = v;
    }
    // s_barrier does not wait for LDS writes: land them before the tile's barrier
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
};

__device__ __forceinline__ void dma128_body(const Params& p, int tm, int tn, int z, char* smem) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int64_t kbeg = (int64_t)z * p.kchunk;
  const int64_t kend = kbeg + p.kchunk < p.K ? kbeg + p.kchunk : p.K;
  const int nk = static_cast<int>((kend - kbeg + BK - 1) / BK);
  const DmaOperand da(reinterpret_cast<const __bf16*>(p.A), p.lda, m0, kbeg, wave, lane, p.a_tiled);
  const DmaOperand db(reinterpret_cast<const __bf16*>(p.B), p.ldb, n0, kbeg, wave, lane, p.b_tiled);
  const uint32_t lds0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(smem));
  // copies of k-tile kt into stage kt % DNB (4 per wave: 2 per operand)
  auto issue = [&](int kt) {
    const int st = kt % DNB;
    const int64_t left = kend - (kbeg + (int64_t)kt * BK);
    if (left >= BK) {
      da.issue(lds0 + st * 2 * TT_PLANE, wave, kt);
      db.issue(lds0 + st * 2 * TT_PLANE + TT_PLANE, wave, kt);
    } else {
      dma_wait_vm(0);
      da.issue_ragged(smem + st * 2 * TT_PLANE, wave, lane, kt, left);
      db.issue_ragged(smem + st * 2 * TT_PLANE + TT_PLANE, wave, lane, kt, left);
    }
  };
  f4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  const bool want_rows = p.rowsum && tn == 0;
  float rs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  // this thread's column-sum runs in the A image: rows kl0, kl0 + 16, columns cl .. cl + 7
  const int kl0 = tid >> 4, cl = 8 * (tid & 15);
  for (int kt = 0; kt < DNB - 1 && kt < nk; ++kt) issue(kt);
  for (int kt = 0; kt < nk; ++kt) {
    // this wave's copies of tile kt have landed once only the later tiles' may be pending
    const int later = (kt + DNB - 2 < nk - 1 ? kt + DNB - 2 : nk - 1) - kt;
    dma_wait_vm(4 * later);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // every wave is past tile kt - 1's reads: its stage takes tile kt + DNB - 1
    if (kt + DNB - 1 < nk) issue(kt + DNB - 1);
    const char* s = smem + (kt % DNB) * 2 * TT_PLANE;
    if (want_rows) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const uint4 v = *reinterpret_cast<const uint4*>(s + tt_off(kl0 + 16 * j, cl >> 3));
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint32_t d = w[e >> 1];
          rs[e] = __fadd_rn(rs[e], __uint_as_float((e & 1) ? (d & 0xffff0000u) : (d << 16)));
        }
      }
    }
    bf8 b[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = tt_frag(s + TT_PLANE, 8 * wn + 2 * j, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bf8 a = tt_frag(s, 8 * wm + 2 * i, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[j], acc[i][j], 0, 0, 0);
    }
  }
  dma_wait_vm(0);
  __syncthreads();  // LDS free for the row-sum reduction
  const bool split = p.zsplit > 1;
  if (want_rows) {
    float* red = reinterpret_cast<float*>(smem);  // [16][128]
#pragma unroll
    for (int e = 0; e < 8; ++e) red[kl0 * BM + cl + e] = rs[e];
    __syncthreads();
    if (tid < BM) {
      float v = red[tid];
#pragma unroll
      for (int q = 1; q < 16; ++q) v = __fadd_rn(v, red[q * BM + tid]);
      if (split) p.rowsum_part[(int64_t)z * p.M + m0 + tid] = v;
      else p.rowsum[m0 + tid] = v;
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t n = n0 + wn * 64 + 16 * j + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t m = m0 + wm * 64 + 16 * i + 4 * (lane >> 4) + r;
        float v = acc[i][j][r];
        if (split) {
          p.part[((int64_t)z * p.M + m) * p.N + n] = v;
          continue;
        }
        if (n >= p.nstore) continue;
        float* c = p.C + m * p.ldc + n;
        if (p.accumulate) v = __fadd_rn(*c, v);
        *c = v;
      }
    }
}

__global__ __launch_bounds__(THREADS, 2) void k_gemm_bf16_dma(Params p) {
  __shared__ __align__(16) char smem[DNB * 2 * TT_PLANE];  // DNB stages x (A, B) images
  int tm, tn, tile, z;
  if (!split_of(p, tile, z)) return;
  if (!tile_of(p, tile, tm, tn)) return;
  dma128_body(p, tm, tn, z, smem);
}

// A batch of products in whole 128 x 128 tiles over the same K (aon_gemm_batch): T = all the
// products' tiles, chunk z of every tile on one XCD (split_of's order), product b owning tiles
// tile0[b] .. tile0[b + 1] - 1 (its own grid, m fastest)
__global__ __launch_bounds__(THREADS, 2) void k_gemm_bf16_dma_batch(ParamsBatch pb) {
  __shared__ __align__(16) char smem[DNB * 2 * TT_PLANE];
  const int T = pb.tile0[pb.count], L = blockIdx.x, x = L & 7, q = L >> 3;
  const int z = 8 * (q / T) + x, t = q - (q / T) * T;
  if (z >= pb.zsplit) return;  // padding block of the last chunk group (uniform exit)
  int b = 0;
  while (b + 1 < pb.count && t >= pb.tile0[b + 1]) ++b;
  const Params& p = pb.p[b];
  const int lt = t - pb.tile0[b];
  dma128_body(p, lt % p.tiles_m, lt / p.tiles_m, z, smem);
}

// ---- the same product with a 256 x 256 C tile per workgroup (k_gemm_bf16_dma256): the
// training step's 256 x 256 weight gradients (pts_linears, bottleneck) are ONE tile, so every
// workgroup is a K chunk and each operand byte crosses into a CU once -- the 128 x 128 kernel
// reads every k-tile of both operands into two workgroups (the 2 x 2 tile grid), twice the
// bytes per CU for the same product (0.195 ms per fine-level product at ~15 B/cycle/CU).
// 512 threads = 8 waves in 4 (m) x 2 (n), each wave 64 x 128 = 4 x 8 MFMA tiles (128 fp32
// accumulator VGPRs), one workgroup per CU: DNB2 stages of a [32 k][256 col] image pair
// (32 KB), the same XOR swizzle on the low four 16-B chunks of each 512-B image row
// (ds_read_b64_tr_b16 banks repeat every 256 B, so the 128-column analysis holds).
#ifndef AON_GEMM_DMA256
#define AON_GEMM_DMA256 1  // 0: the 256 x 256 products take the 128 x 128 kernel (A/B)
#endif
#ifndef AON_GEMM_DMA256_NBUF
#define AON_GEMM_DMA256_NBUF 3
#endif
constexpr int DNB2 = AON_GEMM_DMA256_NBUF;
constexpr int BM2 = 256, THREADS2 = 512;
constexpr int TT_PLANE2 = BK * 512;  // bytes of one operand's [32 k][256 col] bf16 image

__device__ __forceinline__ int tt_off2(int row, int ch) {  // byte offset of 16-B chunk ch of row
  return 512 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

__device__ __forceinline__ bf8 tt_frag2(const char* plane, int c0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  tt_v4s h[2];
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    const char* a = plane + tt_off2(8 * g + 4 * hh + q, c0 + (p >> 1)) + 8 * (p & 1);
    h[hh] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        reinterpret_cast<__attribute__((address_space(3))) tt_v4s*>(
            reinterpret_cast<uintptr_t>(a)));
  }
  typedef short v8s __attribute__((ext_vector_type(8)));
  const v8s w = {h[0][0], h[0][1], h[0][2], h[0][3], h[1][0], h[1][1], h[1][2], h[1][3]};
  return __builtin_bit_cast(bf8, w);
}

// one operand's copies into a 256-column image: copy c of wave w fills image rows
// 2 (2 w + c) + lane / 32, physical chunk lane % 32 <- logical chunk (lane % 32) ^ swz(row)
struct DmaOperand2 {
  const char* gbase;
  int64_t tstep;
  uint32_t voff[2];
  __device__ __forceinline__ DmaOperand2(const __bf16* p, int64_t ld, int64_t col0, int64_t kbeg,
                                         int wave, int lane, bool tiled) {
    gbase = reinterpret_cast<const char*>(p) + 2 * (kbeg * ld + (tiled ? 16 * col0 : col0));
    tstep = 2 * BK * ld;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int r = 2 * (2 * wave + c) + (lane >> 5);
      const int ch = (lane & 31) ^ (((r & 3) << 2) | ((r >> 2) & 3));
      const int64_t e = tiled ? (int64_t)(r & 16) * ld + 256 * (ch >> 1) + 16 * (r & 15) + 8 * (ch & 1)
                              : (int64_t)r * ld + 8 * ch;
      voff[c] = static_cast<uint32_t>(2 * e);
    }
  }
  __device__ __forceinline__ void issue(uint32_t plane, int wave, int kt) const {
    const char* g = gbase + kt * tstep;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const uint32_t m0 = __builtin_amdgcn_readfirstlane(plane + 1024u * (2 * wave + c));
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
      asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, %2"
                   :
                   : "s"(m0), "v"(voff[c]), "s"(g)
                   : "memory", "m0");
#pragma clang diagnostic pop
    }
  }
  __device__ __forceinline__ void issue_ragged(char* plane, int wave, int lane, int kt,
                                               int64_t rows_left) const {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int r = 2 * (2 * wave + c) + (lane >> 5);
      uint4 v = {0u, 0u, 0u, 0u};
      if (r < rows_left) v = *reinterpret_cast<const uint4*>(gbase + kt * tstep + voff[c]);
      *reinterpret_cast<uint4*>(plane + 1024 * (2 * wave + c) + 16 * lane) = v;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
};

__device__ __forceinline__ void dma256_body(const Params& p, int tm, int tn, int z, char* smem) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t m0 = (int64_t)tm * BM2, n0 = (int64_t)tn * BM2;
  const int64_t kbeg = (int64_t)z * p.kchunk;
  const int64_t kend = kbeg + p.kchunk < p.K ? kbeg + p.kchunk : p.K;
  const int nk = static_cast<int>((kend - kbeg + BK - 1) / BK);
  const DmaOperand2 da(reinterpret_cast<const __bf16*>(p.A), p.lda, m0, kbeg, wave, lane, p.a_tiled);
  const DmaOperand2 db(reinterpret_cast<const __bf16*>(p.B), p.ldb, n0, kbeg, wave, lane, p.b_tiled);
  const uint32_t lds0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(smem));
  auto issue = [&](int kt) {
    const int st = kt % DNB2;
    const int64_t left = kend - (kbeg + (int64_t)kt * BK);
    if (left >= BK) {
      da.issue(lds0 + st * 2 * TT_PLANE2, wave, kt);
      db.issue(lds0 + st * 2 * TT_PLANE2 + TT_PLANE2, wave, kt);
    } else {
      dma_wait_vm(0);
      da.issue_ragged(smem + st * 2 * TT_PLANE2, wave, lane, kt, left);
      db.issue_ragged(smem + st * 2 * TT_PLANE2 + TT_PLANE2, wave, lane, kt, left);
    }
  };
  f4 acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  const bool want_rows = p.rowsum && tn == 0;
  float rs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  // this thread's column-sum runs in the A image: rows kl0, kl0 + 16, columns cl .. cl + 7
  const int kl0 = tid >> 5, cl = 8 * (tid & 31);
  for (int kt = 0; kt < DNB2 - 1 && kt < nk; ++kt) issue(kt);
  for (int kt = 0; kt < nk; ++kt) {
    const int later = (kt + DNB2 - 2 < nk - 1 ? kt + DNB2 - 2 : nk - 1) - kt;
    dma_wait_vm(4 * later);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + DNB2 - 1 < nk) issue(kt + DNB2 - 1);
    const char* s = smem + (kt % DNB2) * 2 * TT_PLANE2;
    if (want_rows) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const uint4 v = *reinterpret_cast<const uint4*>(s + tt_off2(kl0 + 16 * j, cl >> 3));
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint32_t d = w[e >> 1];
          rs[e] = __fadd_rn(rs[e], __uint_as_float((e & 1) ? (d & 0xffff0000u) : (d << 16)));
        }
      }
    }
    bf8 b[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) b[j] = tt_frag2(s + TT_PLANE2, 16 * wn + 2 * j, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bf8 a = tt_frag2(s, 8 * wm + 2 * i, lane);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[j], acc[i][j], 0, 0, 0);
    }
  }
  dma_wait_vm(0);
  __syncthreads();  // LDS free for the row-sum reduction
  const bool split = p.zsplit > 1;
  if (want_rows) {
    float* red = reinterpret_cast<float*>(smem);  // [16][256]
#pragma unroll
    for (int e = 0; e < 8; ++e) red[kl0 * BM2 + cl + e] = rs[e];
    __syncthreads();
    if (tid < BM2) {
      float v = red[tid];
#pragma unroll
      for (int q = 1; q < 16; ++q) v = __fadd_rn(v, red[q * BM2 + tid]);
      if (split) p.rowsum_part[(int64_t)z * p.M + m0 + tid] = v;
      else p.rowsum[m0 + tid] = v;
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int64_t n = n0 + wn * 128 + 16 * j + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t m = m0 + wm * 64 + 16 * i + 4 * (lane >> 4) + r;
        float v = acc[i][j][r];
        if (split) {
          p.part[((int64_t)z * p.M + m) * p.N + n] = v;
          continue;
        }
        if (n >= p.nstore) continue;
        float* c = p.C + m * p.ldc + n;
        if (p.accumulate) v = __fadd_rn(*c, v);
        *c = v;
      }
    }
}

__global__ __launch_bounds__(THREADS2, 2) void k_gemm_bf16_dma256(Params p) {
  __shared__ __align__(16) char smem[DNB2 * 2 * TT_PLANE2];  // DNB2 stages x (A, B) images
  int tm, tn, tile, z;
  if (!split_of(p, tile, z)) return;
  if (!tile_of(p, tile, tm, tn)) return;
  dma256_body(p, tm, tn, z, smem);
}

// A batch of one-tile (256 x 256) products over the same K (one level's weight gradients): the
// 256 workgroups are count products x zsplit K chunks -- chunk z of every product on one XCD
// (split_of's order, the product index in place of the tile) -- so each product's chunks are
// count times longer than in its own launch: count times fewer fp32 partials written and summed
// (each launch of a lone product wrote 256 x 257 KB = 67 MB of partials for 0.27-0.81 GB of
// operands), and one launch + one reduce per level instead of count of each.
__global__ __launch_bounds__(THREADS2, 2) void k_gemm_bf16_dma256_batch(ParamsBatch pb) {
  __shared__ __align__(16) char smem[DNB2 * 2 * TT_PLANE2];
  const int T = pb.count, L = blockIdx.x, x = L & 7, q = L >> 3;
  const int z = 8 * (q / T) + x, b = q - (q / T) * T;
  if (z >= pb.zsplit) return;  // padding block of the last chunk group (uniform exit)
  dma256_body(pb.p[b], 0, 0, z, smem);
}

// ---- fp16x3 weight gradients in one 256 x 256 tile per workgroup, ONE fp32 accumulator
// (aon_gemm_args.f16_single): the parity mode's 256 x 256 products dW = dY^T X of the fused
// training kernels' tiled fp32 tensors (pts_linears, bottleneck).  k_gemm_f16x3 runs them as a
// 2 x 2 grid of 128 x 128 tiles with two accumulators per tile (hi*hi and the 2^11-scaled cross
// terms), each operand byte staged into two workgroups; at 0.57 ms per fine-level product it was
// at 0.21 of the MFMA peak.  Here the operands carry the fused kernels' own scales -- A (dY) at
// the backward chain's per-call gradient scale, B (the activations) at 2^3 -- where the lo parts
// x s - fp16(x s) stay normal fp16 for |x s| >= 2^-3 (below it they keep an absolute 2^-25), so
// hi*hi + hi*lo + lo*hi share one accumulator (the fused MLP kernels' V2 numerics) and a wave's
// 64 x 128 sub-tile fits in 128 accumulator VGPRs.  The caller guarantees |x s| < 65504 for both
// operands (the chain and the forward range-guard their own splits at exactly these scales).
// 512 threads = 8 waves in 4 (m) x 2 (n), one workgroup per CU.  Per 32-row k-tile each thread
// loads two 32-B runs of each operand (a wave reads 2 KB contiguous of the tiled layout), splits
// them once into fp16 hi / lo and writes them (16-B stores) into [32 k][256 col] planes with
// the bf16 kernels' XOR swizzle, from which the MFMA fragments come by ds_read_b64_tr_b16; two
// LDS stages (128 KB), the split of tile kt + 1 and the loads of tile kt + 2 ride between the
// MFMAs of tile kt, one barrier per k-tile.  rowsum: A's fp32 values in row order per thread,
// then a fixed order over the 16 threads of a column run.
// Shapes (MW x NW, the operands' widths): 256 x 256 (pts_linears, bottleneck), 128 x 256
// (views_linear.0's bottleneck columns) and 256 x 64 (pts_linears.0's and the skip layer's
// pos_enc columns, B the tiled 64-column encodings of aon_cast_rays_tiled).  Waves in MW / 64
// (m) x 8 / (MW / 64) (n): every wave 64 rows x NW / WN columns.  An operand of width W < 128
// is staged into a 128-column image (the 128-column swizzle of the bf16 kernels).
template <int W>
struct F1Img {
  static constexpr int kCols = W < 128 ? 128 : W;  // image columns
  static constexpr int kPlane = BK * kCols * 2;    // bytes of one [32 k][kCols] fp16 plane
  static constexpr int kRuns = (4 * W + THREADS2 - 1) / THREADS2;  // 8-float runs per thread
  __device__ __forceinline__ static int off(int row, int ch) {
    return kCols == 256 ? tt_off2(row, ch) : tt_off(row, ch);
  }
  __device__ __forceinline__ static h8 frag(const char* plane, int c0, int lane) {
    return __builtin_bit_cast(h8, kCols == 256 ? tt_frag2(plane, c0, lane) : tt_frag(plane, c0, lane));
  }
};

// one thread's runs of a k-tile of a tiled fp32 operand of width W: run u = tid + 512 i (< 4 W)
// is floats 8 u .. 8 u + 7 of the k-tile's contiguous 32 W floats -- k row 16 (8 u / 16 W) +
// (8 u % 256) / 16, columns 16 ((8 u % 16 W) / 256) + (8 u % 16) .. + 7 (a wave reads 2 KB
// contiguous)
template <int W>
struct F1Run {
  static constexpr int NR = F1Img<W>::kRuns;
  f4 v[NR][2];
  __device__ __forceinline__ static bool valid(int tid, int i) {
    return (4 * W) % THREADS2 == 0 || tid + THREADS2 * i < 4 * W;  // every thread's: no branch
  }
  __device__ __forceinline__ static int row(int tid, int i) {
    const int u = tid + THREADS2 * i;
    return 16 * (8 * u / (16 * W)) + (8 * u % 256) / 16;
  }
  __device__ __forceinline__ static int col(int tid, int i) {
    const int u = tid + THREADS2 * i;
    return 16 * ((8 * u % (16 * W)) / 256) + (8 * u % 16);
  }
  __device__ __forceinline__ void load(const float* base, int64_t k0, int64_t kend, int tid, int i) {
    if (!valid(tid, i)) return;
    const f4* src = reinterpret_cast<const f4*>(base + k0 * W + 8 * (tid + THREADS2 * i));
    if (k0 + row(tid, i) < kend) {
      v[i][0] = src[0];
      v[i][1] = src[1];
    } else {
      v[i][0] = f4{0.f, 0.f, 0.f, 0.f};
      v[i][1] = f4{0.f, 0.f, 0.f, 0.f};
    }
  }
  // split run i at scale s into the hi / lo planes (16-B stores)
  __device__ __forceinline__ void store(char* hi, char* lo, float s, int tid, int i) const {
    if (!valid(tid, i)) return;
    h8 h, l;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float x = v[i][e >> 2][e & 3] * s;  // power of two: exact
      const _Float16 hh = static_cast<_Float16>(x);
      h[e] = hh;
      l[e] = static_cast<_Float16>(__fsub_rn(x, static_cast<float>(hh)));  // exact in fp32
    }
    const int off = F1Img<W>::off(row(tid, i), col(tid, i) >> 3);
    *reinterpret_cast<h8*>(hi + off) = h;
    *reinterpret_cast<h8*>(lo + off) = l;
  }
  // run i added to the thread's 8 running column sums, in row order
  __device__ __forceinline__ void add_rows(float (&rs)[8], int i) const {
#pragma unroll
    for (int e = 0; e < 8; ++e) rs[e] = __fadd_rn(rs[e], v[i][e >> 2][e & 3]);
  }
};


template <int MW, int NW>
struct F1Shape {
  static constexpr int kWM = MW / 64, kWN = 8 / kWM;  // waves in m / n
  static constexpr int kTJ = NW / kWN / 16;           // 16-column tiles per wave
  static constexpr int kStage = 2 * F1Img<MW>::kPlane + 2 * F1Img<NW>::kPlane;  // A hi, lo, B hi, lo
  static constexpr int kLds = 2 * kStage;
  // row sums: a thread's A runs share their columns when it has two (rows r, 16 + r: 16 slots
  // per column), else its one run is row 16 h + r (32 slots)
  static constexpr int kSlots = F1Img<MW>::kRuns == 2 ? 16 : 32;
  static_assert(MW % 64 == 0 && 8 % kWM == 0 && kTJ >= 1 && kSlots * MW * 4 <= kLds, "f1 shape");
};

// INTER: split-K by interleaved k-tiles (a lone product), else contiguous chunks (a batch)
template <int MW, int NW, bool INTER>
__device__ __forceinline__ void f1_body(const Params& p, int z, char* smem) {
  using S = F1Shape<MW, NW>;
  using IA = F1Img<MW>;
  using IB = F1Img<NW>;
  float sa = p.sa, inv_s = p.inv_s;
  if (p.sa_bits) {
    const float gs = grad_scale(*p.sa_bits);
    sa = __fmul_rn(sa, gs);
    inv_s = __fdiv_rn(inv_s, gs);
  }
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / S::kWN, wn = wave % S::kWN;
  // INTER: workgroup z takes k-tiles z, z + zsplit, z + 2 zsplit, ... so a lone product's
  // workgroups read one contiguous run of zsplit k-tiles at a time (its contiguous chunks put
  // 256 read streams a fixed multiple of 3 MB apart: 0.51-0.54 ms against 0.45-0.48 interleaved;
  // a batch's 8 products x 32 chunks measured the other way round, 3.08-3.17 ms contiguous
  // against 3.57-3.71 interleaved, profiles/r05/f1_ab)
  const int64_t ntiles = (p.K + BK - 1) / BK, zs = INTER ? p.zsplit : 1;
  const int64_t kbeg = INTER ? 0 : (int64_t)z * p.kchunk;
  const int64_t kend = INTER ? p.K : (kbeg + p.kchunk < p.K ? kbeg + p.kchunk : p.K);
  const int64_t t0 = INTER ? z : kbeg / BK;  // first k-tile; then every zs-th
  const int nk = INTER ? (z < ntiles ? static_cast<int>((ntiles - 1 - z) / zs + 1) : 0)
                       : static_cast<int>((kend - kbeg + BK - 1) / BK);
  const bool want_rows = p.rowsum != nullptr;
  float rs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  F1Run<MW> ra;
  F1Run<NW> rb;
  constexpr int NRUN = IA::kRuns > IB::kRuns ? IA::kRuns : IB::kRuns;
  auto load = [&](int kt, int i) {
    const int64_t k0 = (t0 + (int64_t)kt * zs) * BK;
    if (i < IA::kRuns) ra.load(p.A, k0, kend, tid, i);
    if (i < IB::kRuns) rb.load(p.B, k0, kend, tid, i);
  };
  // publish run i of both operands to stage st (and A's values to the row sums, in row order)
  auto publish = [&](int st, int i) {
    char* s = smem + st * S::kStage;
    if (i < IA::kRuns) {
      if (want_rows && ra.valid(tid, i)) ra.add_rows(rs, i);
      ra.store(s, s + IA::kPlane, sa, tid, i);
    }
    if (i < IB::kRuns) rb.store(s + 2 * IA::kPlane, s + 2 * IA::kPlane + IB::kPlane, p.sb, tid, i);
  };
  f4 acc[4][S::kTJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < S::kTJ; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  if (nk > 0) {
#pragma unroll
    for (int i = 0; i < NRUN; ++i) load(0, i);
#pragma unroll
    for (int i = 0; i < NRUN; ++i) publish(0, i);
    if (nk > 1) {
#pragma unroll
      for (int i = 0; i < NRUN; ++i) load(1, i);
    }
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const char* s = smem + (kt & 1) * S::kStage;
    const char* sb = s + 2 * IA::kPlane;
    const bool more = kt + 1 < nk;
    h8 ah[4], al[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ah[i] = IA::frag(s, 8 * wm + 2 * i, lane);
      al[i] = IA::frag(s + IA::kPlane, 8 * wm + 2 * i, lane);
    }
#pragma unroll
    for (int j = 0; j < S::kTJ; ++j) {
      const int c0 = 2 * (S::kTJ * wn + j);
      const h8 bh = IB::frag(sb, c0, lane);
      const h8 bl = IB::frag(sb + IB::kPlane, c0, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        acc[i][j] = mfma16(ah[i], bh, acc[i][j]);
        acc[i][j] = mfma16(ah[i], bl, acc[i][j]);
        acc[i][j] = mfma16(al[i], bh, acc[i][j]);
      }
      // tile kt + 1 (in registers) into the other stage between the MFMAs, each run's
      // registers refilled with tile kt + 2's at once: its loads fly under a whole k-tile
      if (more && j < NRUN) {
        publish((kt + 1) & 1, j);
        if (kt + 2 < nk) load(kt + 2, j);
      }
    }
    if (more && S::kTJ < NRUN) {  // narrow B: the runs left after the MFMAs
#pragma unroll
      for (int i = S::kTJ; i < NRUN; ++i) {
        publish((kt + 1) & 1, i);
        if (kt + 2 < nk) load(kt + 2, i);
      }
    }
    __syncthreads();
  }
  const bool split = p.zsplit > 1;
  if (want_rows) {
    // combine the slots of every column in slot order (LDS free after the last barrier)
    float* red = reinterpret_cast<float*>(smem);  // [kSlots][MW]
    if (ra.valid(tid, 0)) {
      const int slot = S::kSlots == 16 ? ra.row(tid, 0) : ra.row(tid, 0) & 31;
      const int c = ra.col(tid, 0);
#pragma unroll
      for (int e = 0; e < 8; ++e) red[slot * MW + c + e] = rs[e];
    }
    __syncthreads();
    if (tid < MW) {
      float v = red[tid];
#pragma unroll
      for (int q = 1; q < S::kSlots; ++q) v = __fadd_rn(v, red[q * MW + tid]);
      if (split) p.rowsum_part[(int64_t)z * p.M + tid] = v;
      else p.rowsum[tid] = v;
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < S::kTJ; ++j) {
      const int64_t n = (NW / S::kWN) * wn + 16 * j + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t m = 64 * wm + 16 * i + 4 * (lane >> 4) + r;
        float v = __fmul_rn(acc[i][j][r], inv_s);
        if (split) {
          p.part[((int64_t)z * p.M + m) * p.N + n] = v;
          continue;
        }
        if (n >= p.nstore) continue;
        float* c = p.C + m * p.ldc + n;
        if (p.accumulate) v = __fadd_rn(*c, v);
        *c = v;
      }
    }
}

template <int MW, int NW>
__global__ __launch_bounds__(THREADS2, 1) void k_gemm_f1(Params p) {
  __shared__ __align__(16) char smem[F1Shape<MW, NW>::kLds];
  int tile, z;
  if (!split_of(p, tile, z)) return;
  f1_body<MW, NW, true>(p, z, smem);
}

// a batch of 256 x 256 products over the same K (one level's): chunk z of every product on one
// XCD, as k_gemm_bf16_dma256_batch
__global__ __launch_bounds__(THREADS2, 1) void k_gemm_f1_256_batch(ParamsBatch pb) {
  __shared__ __align__(16) char smem[F1Shape<256, 256>::kLds];
  const int T = pb.count, L = blockIdx.x, x = L & 7, q = L >> 3;
  const int z = 8 * (q / T) + x, b = q - (q / T) * T;
  if (z >= pb.zsplit) return;  // padding block of the last chunk group (uniform exit)
  f1_body<256, 256, false>(pb.p[b], z, smem);
}

// The batch's 256 x 256 products as two 256 x 128 half tiles each (k_gemm_f1h_batch): a
// workgroup keeps 64 accumulator VGPRs per wave instead of 128, which buys AON_F1H_SETS
// register sets of staged runs -- that many k-tiles of loads in flight instead of one -- for
// twice the A reads, the second from L2 (the two halves of a chunk are dispatched together on
// one XCD: block ids 8 apart).
#ifndef AON_F1H_SETS
#define AON_F1H_SETS 2  // 3 spills (22 VGPRs): 5.13 ms against 3.62-3.71 for 2, 4.08-4.12 whole tiles
#endif
#ifndef AON_F1_HALF
#define AON_F1_HALF 1  // 0: A/B build -- the batch on whole 256 x 256 tiles (k_gemm_f1_256_batch)
#endif
constexpr int F1H_SETS = AON_F1H_SETS;

// one thread's run of a k-tile of the 128-column half h of a tiled fp32 operand of width 256:
// run u = tid: k row 16 (u / 256) + (u % 32) / 2, columns 16 ((u % 256) / 32) + 8 (u % 2) of
// the half (a wave reads two 1-KB runs of the tiled layout)
struct F1HalfRun {
  f4 v[2];
  __device__ __forceinline__ static int row(int tid) { return 16 * (tid >> 8) + ((tid & 31) >> 1); }
  __device__ __forceinline__ static int col(int tid) { return 16 * ((tid & 255) >> 5) + 8 * (tid & 1); }
  __device__ __forceinline__ void load(const float* base, int h, int64_t k0, int64_t kend, int tid) {
    const int rr = row(tid);
    const f4* src = reinterpret_cast<const f4*>(base + (k0 + 16 * (tid >> 8)) * 256 +
                                                256 * (8 * h + ((tid & 255) >> 5)) +
                                                16 * ((tid & 31) >> 1) + 8 * (tid & 1));
    if (k0 + rr < kend) {
      v[0] = src[0];
      v[1] = src[1];
    } else {
      v[0] = f4{0.f, 0.f, 0.f, 0.f};
      v[1] = f4{0.f, 0.f, 0.f, 0.f};
    }
  }
  __device__ __forceinline__ void store(char* hi, char* lo, float s, int tid) const {
    h8 hh, ll;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float x = v[e >> 2][e & 3] * s;
      const _Float16 q = static_cast<_Float16>(x);
      hh[e] = q;
      ll[e] = static_cast<_Float16>(__fsub_rn(x, static_cast<float>(q)));
    }
    const int off = tt_off(row(tid), col(tid) >> 3);
    *reinterpret_cast<h8*>(hi + off) = hh;
    *reinterpret_cast<h8*>(lo + off) = ll;
  }
};

struct F1HSet {
  F1Run<256> a;
  F1HalfRun b;
};

constexpr int F1H_STAGE = 2 * F1Img<256>::kPlane + 2 * F1Img<128>::kPlane;  // 48 KB

// product p's half h (columns 128 h ..) of K chunk z
__device__ __forceinline__ void f1h_body(const Params& p, int h, int z, char* smem) {
  float sa = p.sa, inv_s = p.inv_s;
  if (p.sa_bits) {
    const float gs = grad_scale(*p.sa_bits);
    sa = __fmul_rn(sa, gs);
    inv_s = __fdiv_rn(inv_s, gs);
  }
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;  // 4 x 2 waves of 64 x 64
  const int64_t kbeg = (int64_t)z * p.kchunk;
  const int64_t kend = kbeg + p.kchunk < p.K ? kbeg + p.kchunk : p.K;
  const int nk = static_cast<int>((kend - kbeg + BK - 1) / BK);
  const bool want_rows = p.rowsum != nullptr && h == 0;
  float rs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  F1HSet set[F1H_SETS];
  auto load = [&](F1HSet& st, int kt) {
    const int64_t k0 = kbeg + (int64_t)kt * BK;
    st.a.load(p.A, k0, kend, tid, 0);
    st.a.load(p.A, k0, kend, tid, 1);
    st.b.load(p.B, h, k0, kend, tid);
  };
  auto publish = [&](const F1HSet& st, int stage) {
    char* s = smem + stage * F1H_STAGE;
    if (want_rows) {
      st.a.add_rows(rs, 0);
      st.a.add_rows(rs, 1);
    }
    st.a.store(s, s + F1Img<256>::kPlane, sa, tid, 0);
    st.a.store(s, s + F1Img<256>::kPlane, sa, tid, 1);
    char* sb = s + 2 * F1Img<256>::kPlane;
    st.b.store(sb, sb + F1Img<128>::kPlane, p.sb, tid);
  };
  f4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  // tiles 0 .. SETS-1 into the sets, tile 0 to stage 0, its set refilled with tile SETS
#pragma unroll
  for (int q = 0; q < F1H_SETS; ++q)
    if (q < nk) load(set[q], q);
  if (nk > 0) {
    publish(set[0], 0);
    if (F1H_SETS < nk) load(set[0], F1H_SETS);
  }
  __syncthreads();
  // step kt: tile kt in stage kt & 1; tile kt + 1 in set (kt + 1) % SETS, published between
  // this step's MFMAs and that set refilled with tile kt + 1 + SETS (loaded SETS steps ahead)
  auto step = [&](int kt, auto cur) {
    constexpr int NXT = (decltype(cur)::value + 1) % F1H_SETS;
    const char* s = smem + (kt & 1) * F1H_STAGE;
    const char* sb = s + 2 * F1Img<256>::kPlane;
    h8 ah[4], al[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ah[i] = F1Img<256>::frag(s, 8 * wm + 2 * i, lane);
      al[i] = F1Img<256>::frag(s + F1Img<256>::kPlane, 8 * wm + 2 * i, lane);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c0 = 2 * (4 * wn + j);
      const h8 bh = F1Img<128>::frag(sb, c0, lane);
      const h8 bl = F1Img<128>::frag(sb + F1Img<128>::kPlane, c0, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        acc[i][j] = mfma16(ah[i], bh, acc[i][j]);
        acc[i][j] = mfma16(ah[i], bl, acc[i][j]);
        acc[i][j] = mfma16(al[i], bh, acc[i][j]);
      }
      if (j == 0 && kt + 1 < nk) {
        publish(set[NXT], (kt + 1) & 1);
        if (kt + 1 + F1H_SETS < nk) load(set[NXT], kt + 1 + F1H_SETS);
      }
    }
    __syncthreads();
  };
  for (int kt = 0; kt < nk; kt += F1H_SETS) {
    step(kt, std::integral_constant<int, 0>{});
    if (F1H_SETS > 1 && kt + 1 < nk) step(kt + 1, std::integral_constant<int, 1 % F1H_SETS>{});
    if (F1H_SETS > 2 && kt + 2 < nk) step(kt + 2, std::integral_constant<int, 2 % F1H_SETS>{});
    if (F1H_SETS > 3 && kt + 3 < nk) step(kt + 3, std::integral_constant<int, 3 % F1H_SETS>{});
  }
  const bool split = p.zsplit > 1;
  if (want_rows) {
    float* red = reinterpret_cast<float*>(smem);  // [16 r][256]
    const int r = (tid & 31) >> 1, c = 16 * (tid >> 5) + 8 * (tid & 1);
#pragma unroll
    for (int e = 0; e < 8; ++e) red[r * 256 + c + e] = rs[e];
    __syncthreads();
    if (tid < 256) {
      float v = red[tid];
#pragma unroll
      for (int q = 1; q < 16; ++q) v = __fadd_rn(v, red[q * 256 + tid]);
      if (split) p.rowsum_part[(int64_t)z * p.M + tid] = v;
      else p.rowsum[tid] = v;
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t n = 128 * h + 64 * wn + 16 * j + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t m = 64 * wm + 16 * i + 4 * (lane >> 4) + r;
        float v = __fmul_rn(acc[i][j][r], inv_s);
        if (split) {
          p.part[((int64_t)z * p.M + m) * p.N + n] = v;
          continue;
        }
        float* c = p.C + m * p.ldc + n;
        if (p.accumulate) v = __fadd_rn(*c, v);
        *c = v;
      }
    }
}

// T = 2 count half tiles: chunk z of every half of every product on one XCD, the two halves of
// a (product, chunk) 8 block ids apart
__global__ __launch_bounds__(THREADS2, 1) void k_gemm_f1h_batch(ParamsBatch pb) {
  __shared__ __align__(16) char smem[2 * F1H_STAGE];
  const int T = 2 * pb.count, L = blockIdx.x, x = L & 7, q = L >> 3;
  const int z = 8 * (q / T) + x, t = q - (q / T) * T;
  if (z >= pb.zsplit) return;  // padding block of the last chunk group (uniform exit)
  f1h_body(pb.p[t >> 1], t & 1, z, smem);
}

// ---- fp16x3 weight gradients on the LDS-DMA ring (fp32 operands, both reduction-major):
// k_gemm_f16x3<false, false> staged each k-tile through registers (global loads -> transpose ->
// split -> LDS), one tile ahead, and ran the fine level's 256 x 256 x 790k products at ~3 TB/s
// (0.38 of HBM): like the bf16 kernel before its DMA rewrite, too few bytes in flight for the
// HBM latency.  Here global_load_lds_dwordx4 copies each operand's [32 k][128 col] fp32 image
// into a DNBF-deep ring (DNBF - 1 k-tiles in flight per workgroup); once a tile has landed every
// thread reads ITS 4 x 4 block of it from LDS -- the same block the register loader held -- and
// runs the same row sums, split and [row][k] hi / lo plane stores (TileLoad::add_rows / store),
// and the MFMA loop reads the planes exactly as k_gemm_f16x3: every value, every product and
// every sum in the same order, so the result is bit-identical to the register-staged kernel.
// Two barriers per k-tile (tile landed + previous MFMAs done; planes written).  LDS: ring
// DNBF x 32 KB + one 40-KB plane stage -- one workgroup per CU where the register-staged kernel
// runs two, and that costs more than the deeper ring gains: 0.68-0.71 ms (DNBF 2 / 3) against
// 0.57-0.59 ms for the fine product, same sha (profiles/r03/ab_gemm_f16).  Off by default
// (AON_GEMM_F16_DMA = 1 selects it for A/B).
#ifndef AON_GEMM_F16_DNB
#define AON_GEMM_F16_DNB 3
#endif
constexpr int DNBF = AON_GEMM_F16_DNB;
constexpr int F32_IMG = BK * BM * 4;  // bytes of one operand's [32 k][128 col] fp32 image

// one operand's copies of a k-tile: wave w, copy c (0..3) fills image rows 8 w + 2 c + lane / 32,
// 16-B chunk lane % 32 (4 columns)
struct DmaOperandF32 {
  const char* gbase;  // byte address of k-tile 0's (k row 0, column col0) origin, kbeg applied
  int64_t tstep;      // bytes between k-tiles
  uint32_t voff[4];   // per-lane byte offset of copy c within a k-tile
  __device__ __forceinline__ DmaOperandF32(const float* p, int64_t ld, int64_t col0, int64_t kbeg,
                                           int wave, int lane, bool tiled) {
    gbase = reinterpret_cast<const char*>(p) + 4 * (kbeg * ld + (tiled ? 16 * col0 : col0));
    tstep = 4 * BK * ld;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int r = 8 * wave + 2 * c + (lane >> 5), col = 4 * (lane & 31);
      const int64_t e = tiled ? (int64_t)(r & 16) * ld + 256 * (col >> 4) + 16 * (r & 15) + (col & 15)
                              : (int64_t)r * ld + col;
      voff[c] = static_cast<uint32_t>(4 * e);
    }
  }
  __device__ __forceinline__ void issue(uint32_t img, int wave, int kt) const {
    const char* g = gbase + kt * tstep;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const uint32_t m0 = __builtin_amdgcn_readfirstlane(img + 512u * (8 * wave + 2 * c));
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
      asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, %2"
                   :
                   : "s"(m0), "v"(voff[c]), "s"(g)
                   : "memory", "m0");
#pragma clang diagnostic pop
    }
  }
  // the ragged last tile through registers: k rows at or past rows_left read as zero
  __device__ __forceinline__ void issue_ragged(char* img, int wave, int lane, int kt,
                                               int64_t rows_left) const {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int r = 8 * wave + 2 * c + (lane >> 5);
      uint4 v = {0u, 0u, 0u, 0u};
      if (r < rows_left) v = *reinterpret_cast<const uint4*>(gbase + kt * tstep + voff[c]);
      *reinterpret_cast<uint4*>(img + 512 * (8 * wave + 2 * c) + 16 * lane) = v;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
};

__global__ __launch_bounds__(THREADS, 1) void k_gemm_f16x3_dma(Params p) {
  float sa = p.sa, inv_s = p.inv_s;
  if (p.sa_bits) {
    const float gs = grad_scale(*p.sa_bits);
    sa = __fmul_rn(sa, gs);
    inv_s = __fdiv_rn(inv_s, gs);
  }
  __shared__ __align__(16) char smem[DNBF * 2 * F32_IMG + STAGE * 2];  // ring | A hi, A lo, B hi, B lo
  _Float16* planes = reinterpret_cast<_Float16*>(smem + DNBF * 2 * F32_IMG);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  int tm, tn, tile, z;
  if (!split_of(p, tile, z)) return;
  if (!tile_of(p, tile, tm, tn)) return;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int64_t kbeg = (int64_t)z * p.kchunk;
  const int64_t kend = kbeg + p.kchunk < p.K ? kbeg + p.kchunk : p.K;
  const int nk = static_cast<int>((kend - kbeg + BK - 1) / BK);
  const DmaOperandF32 da(p.A, p.lda, m0, kbeg, wave, lane, p.a_tiled);
  const DmaOperandF32 db(p.B, p.ldb, n0, kbeg, wave, lane, p.b_tiled);
  const uint32_t lds0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(smem));
  auto issue = [&](int kt) {
    const int st = kt % DNBF;
    const int64_t left = kend - (kbeg + (int64_t)kt * BK);
    if (left >= BK) {
      da.issue(lds0 + st * 2 * F32_IMG, wave, kt);
      db.issue(lds0 + st * 2 * F32_IMG + F32_IMG, wave, kt);
    } else {
      dma_wait_vm(0);
      da.issue_ragged(smem + st * 2 * F32_IMG, wave, lane, kt, left);
      db.issue_ragged(smem + st * 2 * F32_IMG + F32_IMG, wave, lane, kt, left);
    }
  };
  f4 acc_h[4][4], acc_x[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc_h[i][j] = f4{0.f, 0.f, 0.f, 0.f};
      acc_x[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    }
  const bool want_rows = p.rowsum && tn == 0;
  float rs[4] = {0.f, 0.f, 0.f, 0.f};
  // this thread's 4 x 4 block of an image: rows rq .. rq + 3 (16 B) of k rows kq .. kq + 3
  const int kq = 4 * ((tid >> 2) & 7), rq = 16 * (tid >> 5) + 4 * (tid & 3);
  const int g = lane >> 4, r16 = lane & 15;
  for (int kt = 0; kt < DNBF - 1 && kt < nk; ++kt) issue(kt);
  for (int kt = 0; kt < nk; ++kt) {
    // this wave's copies of tile kt have landed once only the later tiles' may be pending
    const int later = (kt + DNBF - 2 < nk - 1 ? kt + DNBF - 2 : nk - 1) - kt;
    dma_wait_vm(8 * later);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();  // tile kt in LDS for every wave; the planes' readers are done
    asm volatile("" ::: "memory");
    if (kt + DNBF - 1 < nk) issue(kt + DNBF - 1);  // its stage held tile kt - 1, split last step
    const char* img = smem + (kt % DNBF) * 2 * F32_IMG;
    TileLoad<false, true> ta, tb;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ta.r[i] = *reinterpret_cast<const f4*>(img + 512 * (kq + i) + 4 * rq);
      tb.r[i] = *reinterpret_cast<const f4*>(img + F32_IMG + 512 * (kq + i) + 4 * rq);
    }
    if (want_rows) ta.add_rows(rs);
    ta.store(planes, planes + PLANE, sa, tid);
    tb.store(planes + 2 * PLANE, planes + 3 * PLANE, p.sb, tid);
    __syncthreads();  // planes written
    h8 bh[4], bl[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = wn * 64 + 16 * j + r16;
      bh[j] = *reinterpret_cast<const h8*>(planes + 2 * PLANE + row * ROWH + 8 * g);
      bl[j] = *reinterpret_cast<const h8*>(planes + 3 * PLANE + row * ROWH + 8 * g);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wm * 64 + 16 * i + r16;
      const h8 ah = *reinterpret_cast<const h8*>(planes + row * ROWH + 8 * g);
      const h8 al = *reinterpret_cast<const h8*>(planes + PLANE + row * ROWH + 8 * g);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc_h[i][j] = mfma16(ah, bh[j], acc_h[i][j]);
        acc_x[i][j] = mfma16(ah, bl[j], acc_x[i][j]);
        acc_x[i][j] = mfma16(al, bh[j], acc_x[i][j]);
      }
    }
  }
  dma_wait_vm(0);
  __syncthreads();  // LDS free for the row-sum reduction
  const bool split = p.zsplit > 1;
  if (want_rows) {
    float* red = reinterpret_cast<float*>(smem);  // [8 k quads][128 rows]
    const int kqi = (tid >> 2) & 7;
#pragma unroll
    for (int j = 0; j < 4; ++j) red[kqi * BM + rq + j] = rs[j];
    __syncthreads();
    if (tid < BM) {
      float v = red[tid];
#pragma unroll
      for (int q = 1; q < 8; ++q) v = __fadd_rn(v, red[q * BM + tid]);
      if (split) p.rowsum_part[(int64_t)z * p.M + m0 + tid] = v;
      else p.rowsum[m0 + tid] = v;
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t n = n0 + wn * 64 + 16 * j + r16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t m = m0 + wm * 64 + 16 * i + 4 * g + r;
        float v = __fmul_rn(__fadd_rn(acc_h[i][j][r], __fmul_rn(acc_x[i][j][r], kInvLo)), inv_s);
        if (split) {
          p.part[((int64_t)z * p.M + m) * p.N + n] = v;
          continue;
        }
        if (n >= p.nstore) continue;
        float* c = p.C + m * p.ldc + n;
        if (p.accumulate) v = __fadd_rn(*c, v);
        *c = v;
      }
    }
}

// ---- bf16 weight gradients with M <= 4 rows (the rgb / density heads: dW = d raw^T X with
// X = hv3 / h7): a 128 x 128 MFMA tile would run 97% empty and the km kernel's transposing
// loads held these at ~130 us for 0.2-0.4 GB, so the product streams instead.  Thread (r, cg):
// row phase r of every 16-row block of its K chunk, columns 8 cg .. 8 cg + 7 (one 16-B run of B:
// a wave reads two whole 16 x 16 tiles, 1 KB contiguous, of the tiled layout); A's M values of
// the row rounded to bf16 as the MFMA paths stage them, products exact in fp32, fp32 sums in
// row order, then a fixed xor tree over the 16 row phases; one chunk's partial per workgroup
// (k_gemm_reduce sums the chunks in z order: deterministic).  TB = float: the parity mode's
// heads (fp32 A and B, the fused forward's tiled fp32 h7 / hv3), the same kernel with nothing
// rounded -- fp32 products and sums, more accurate than the fp16x3 split it replaces for M <= 4
// (a 128 x 128 tile 97-99% empty, 0.23-0.28 ms per fine-level head).
constexpr int kSkinnyRows = 16;
#ifndef AON_GEMM_SKINNY_SK
#define AON_GEMM_SKINNY_SK 4  // rows in flight per thread of the skinny kernel; 1: A/B
#endif
#ifndef AON_GEMM_SEGSUM_SK
#define AON_GEMM_SEGSUM_SK 16  // ... of the segment-sum kernel (one workgroup of 4 waves per CU;
                               // 16 vs 4: 60.4 vs 62.4 us fine level, neutral)
#endif
#ifndef AON_GEMM_SKINNY_SK2
#define AON_GEMM_SKINNY_SK2 4  // ... of the skinny kernel on B of <= 128 columns (A/B knob: 8 measured
                               // 81 -> 108 us on the fine level's rgb head, profiles/r04/final2)
#endif
template <int M, typename TA, bool BT, int SK = AON_GEMM_SKINNY_SK, typename TB = __bf16>
__global__ __launch_bounds__(512) void k_gemm_skinny_bf16(Params p) {
  constexpr bool RND = std::is_same<TB, __bf16>::value;  // the bf16 mode: A staged as bf16
  constexpr int NB = sizeof(TB) / 2;                      // 16-B loads per 8-column run of B
  const int tid = threadIdx.x, r = tid & 15, cg = tid >> 4;
  const int64_t n0 = 8 * (int64_t)cg;
  const int64_t kbeg = (int64_t)blockIdx.x * p.kchunk;
  const int64_t kend = kbeg + p.kchunk < p.K ? kbeg + p.kchunk : p.K;
  const TA* A = reinterpret_cast<const TA*>(p.A);
  const TB* B = reinterpret_cast<const TB*>(p.B);
  float acc[M][8], rs[M], cs[8];  // cs: B's column sums (c_trans)
  const bool ct = p.c_trans != 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) cs[j] = 0.f;
#pragma unroll
  for (int m = 0; m < M; ++m) {
    rs[m] = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[m][j] = 0.f;
  }
  auto boff = [&](int64_t k) {
    return BT ? (k & ~int64_t(15)) * p.ldb + 256 * (n0 >> 4) + 16 * (k & 15) + (n0 & 15)
              : k * p.ldb + n0;
  };
  auto row = [&](const uint4 (&bv)[NB], const TA* ar) {
    float b[8];
    if (RND) {
      const uint32_t bw[4] = {bv[0].x, bv[0].y, bv[0].z, bv[0].w};
#pragma unroll
      for (int j = 0; j < 8; ++j) b[j] = __uint_as_float((j & 1) ? (bw[j >> 1] & 0xffff0000u) : (bw[j >> 1] << 16));
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint4& q = bv[(j >> 2) & (NB - 1)];
        const uint32_t w = (j & 3) == 0 ? q.x : (j & 3) == 1 ? q.y : (j & 3) == 2 ? q.z : q.w;
        b[j] = __uint_as_float(w);
      }
    }
    if (ct) {
#pragma unroll
      for (int j = 0; j < 8; ++j) cs[j] = __fadd_rn(cs[j], b[j]);
    }
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const float a = RND ? static_cast<float>(static_cast<__bf16>(static_cast<float>(ar[m])))
                          : static_cast<float>(ar[m]);
      rs[m] = __fadd_rn(rs[m], a);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[m][j] = fmaf(a, b[j], acc[m][j]);  // bf16: a * b exact
    }
  };
  auto load_b = [&](int64_t kk, uint4 (&bv)[NB]) {
    const uint4* src = reinterpret_cast<const uint4*>(B + boff(kk));
#pragma unroll
    for (int h = 0; h < NB; ++h) bv[h] = src[h];
  };
  // SK rows per thread in flight: their loads are issued before the first is consumed (one
  // dependent load per row left this kernel latency-bound: rgb's 0.27 GB at ~2.2 TB/s); the
  // rows are still summed in k order (bit-identical); SK2 for B of <= 128 columns (half the waves
  // per workgroup)
  int64_t k = kbeg + r;
  for (; k + (SK - 1) * kSkinnyRows < kend; k += SK * kSkinnyRows) {
    uint4 bv[SK][NB];
    TA av[SK][M];
#pragma unroll
    for (int u = 0; u < SK; ++u) {
      load_b(k + u * kSkinnyRows, bv[u]);
#pragma unroll
      for (int m = 0; m < M; ++m) av[u][m] = A[(k + u * kSkinnyRows) * p.lda + m];
    }
#pragma unroll
    for (int u = 0; u < SK; ++u) row(bv[u], av[u]);
  }
  for (; k < kend; k += kSkinnyRows) {
    TA av[M];
#pragma unroll
    for (int m = 0; m < M; ++m) av[m] = A[k * p.lda + m];
    uint4 bv[NB];
    load_b(k, bv);
    row(bv, av);
  }
  // the 16 row phases of a column group are lanes 16 q .. 16 q + 15 of one wave
#pragma unroll
  for (int sh = 1; sh < 16; sh <<= 1) {
#pragma unroll
    for (int m = 0; m < M; ++m) {
      rs[m] = __fadd_rn(rs[m], __shfl_xor(rs[m], sh, 64));
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[m][j] = __fadd_rn(acc[m][j], __shfl_xor(acc[m][j], sh, 64));
    }
    if (ct) {
#pragma unroll
      for (int j = 0; j < 8; ++j) cs[j] = __fadd_rn(cs[j], __shfl_xor(cs[j], sh, 64));
    }
  }
  if (r != 0) return;
  const bool split = p.zsplit > 1;
  const int z = blockIdx.x;
  if (ct && p.rowsum) {  // B's column sums: columns n0 .. n0 + 7 of this column group
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (split) p.rowsum_part[(int64_t)z * p.N + n0 + j] = cs[j];
      else p.rowsum[n0 + j] = cs[j];
    }
  }
#pragma unroll
  for (int m = 0; m < M; ++m) {
    if (!ct && p.rowsum && cg == 0) {
      if (split) p.rowsum_part[(int64_t)z * p.M + m] = rs[m];
      else p.rowsum[m] = rs[m];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = acc[m][j];
      if (split) {
        p.part[((int64_t)z * p.M + m) * p.N + n0 + j] = v;
        continue;
      }
      float* c = p.C + (ct ? (n0 + j) * p.ldc + m : m * p.ldc + n0 + j);
      if (p.accumulate) v = __fadd_rn(*c, v);
      *c = v;
    }
  }
}

// ---- bf16 weight gradient against a per-ray operand: C = A^T B with row k of B at k / rdiv
// (views_linear.0's enc_dir columns: B = pos_enc(viewdirs), one row per ray, rdiv = S).  Every
// B row meets rdiv consecutive A rows, so C = sum_ray (sum_{s<rdiv} A[ray rdiv + s]) B[ray]:
// thread (ray, cg) sums its ray's rdiv rows of columns 8 cg .. 8 cg + 7 in row order (A's
// values rounded to bf16 as staged; fp32 sums, kept unrounded), the workgroup's RB rays' sums go
// to LDS, and their outer products with bf16(B) make the chunk's partial of C (and of A's
// column sums).  The km kernel read A with the reduction-major transposing loads at ~130 us for
// the fine level's 0.2 GB; this reads A once, in 16-B runs, and does 1/rdiv of the products.
// RND = false: the parity mode's (fp32 A and B), nothing rounded -- fp32 sums and products.
template <typename TA, typename TB, bool AT, bool RND = true>
__global__ __launch_bounds__(256) void k_gemm_segsum_bf16(Params p) {
  __shared__ float seg[256 * 8];  // [RB rays][M]: RB * M = 8 * 256
  const int M = static_cast<int>(p.M), N = static_cast<int>(p.N);
  const int cgs = M / 8, rb = 256 / cgs;
  const int tid = threadIdx.x, cg = tid % cgs, rl = tid / cgs;
  const int64_t rdiv = p.b_rdiv;
  const int64_t ray = (int64_t)blockIdx.x * rb + rl;
  const TA* A = reinterpret_cast<const TA*>(p.A);
  const int64_t n0 = 8 * (int64_t)cg;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int64_t kb = ray * rdiv, ke = kb + rdiv < p.K ? kb + rdiv : p.K;
  auto aoff = [&](int64_t k) {
    return AT ? (k & ~int64_t(15)) * p.lda + 256 * (n0 >> 4) + 16 * (k & 15) + (n0 & 15)
              : k * p.lda + n0;
  };
  auto add_row = [&](int64_t o, const uint4& w) {
    float v[8];
    if (std::is_same<TA, __bf16>::value) {
      const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = __uint_as_float((j & 1) ? (ww[j >> 1] & 0xffff0000u) : (ww[j >> 1] << 16));
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        v[j] = static_cast<float>(static_cast<__bf16>(static_cast<float>(A[o + j])));
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = __fadd_rn(acc[j], v[j]);
  };
  // fp32 A unrounded: one row's 8 columns as two 16-B loads
  auto add_row32 = [&](const uint4 (&w)[2]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint4& q = w[j >> 2];
      const uint32_t u = (j & 3) == 0 ? q.x : (j & 3) == 1 ? q.y : (j & 3) == 2 ? q.z : q.w;
      acc[j] = __fadd_rn(acc[j], __uint_as_float(u));
    }
  };
  int64_t k = kb;
  if (!RND && std::is_same<TA, float>::value) {
    constexpr int SK = AON_GEMM_SEGSUM_SK / 2;
    for (; k + SK - 1 < ke; k += SK) {
      uint4 w[SK][2];
#pragma unroll
      for (int u = 0; u < SK; ++u) {
        const uint4* src = reinterpret_cast<const uint4*>(A + aoff(k + u));
        w[u][0] = src[0];
        w[u][1] = src[1];
      }
#pragma unroll
      for (int u = 0; u < SK; ++u) add_row32(w[u]);
    }
    for (; k < ke; ++k) {
      const uint4* src = reinterpret_cast<const uint4*>(A + aoff(k));
      const uint4 w[2] = {src[0], src[1]};
      add_row32(w);
    }
  }
  if (std::is_same<TA, __bf16>::value) {
    // AON_GEMM_SEGSUM_SK rows' 16-B loads in flight per thread before the first is summed (one
    // dependent load per row left one workgroup of 4 waves per CU latency-bound; 4 rows still
    // held the fine level's 0.2 GB at ~3.3 TB/s); the rows are still summed in k order
    // (bit-identical)
    constexpr int SK = AON_GEMM_SEGSUM_SK;
    for (; k + SK - 1 < ke; k += SK) {
      uint4 w[SK];
#pragma unroll
      for (int u = 0; u < SK; ++u) w[u] = *reinterpret_cast<const uint4*>(A + aoff(k + u));
#pragma unroll
      for (int u = 0; u < SK; ++u) add_row(0, w[u]);
    }
  }
  for (; k < ke; ++k) {
    const int64_t o = aoff(k);
    uint4 w = {0u, 0u, 0u, 0u};
    if (std::is_same<TA, __bf16>::value) w = *reinterpret_cast<const uint4*>(A + o);
    add_row(o, w);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) seg[rl * M + n0 + j] = acc[j];
  __syncthreads();
  const int64_t ray0 = (int64_t)blockIdx.x * rb;
  const int64_t nray = (p.K + rdiv - 1) / rdiv;
  const int nr = static_cast<int>(nray - ray0 < rb ? nray - ray0 : rb);
  const TB* Bm = reinterpret_cast<const TB*>(p.B);
  const bool split = p.zsplit > 1;
  const int z = blockIdx.x;
  for (int e = tid; e < M * N + M; e += 256) {
    float v = 0.f;
    if (e < M * N) {
      const int m = e / N, n = e - m * N;
      for (int q = 0; q < nr; ++q) {
        const float b = RND ? static_cast<float>(static_cast<__bf16>(static_cast<float>(Bm[(ray0 + q) * p.ldb + n])))
                            : static_cast<float>(Bm[(ray0 + q) * p.ldb + n]);
        v = fmaf(seg[q * M + m], b, v);
      }
      if (split) {
        p.part[((int64_t)z * M + m) * N + n] = v;
        continue;
      }
      float* c = p.C + m * p.ldc + n;
      if (p.accumulate) v = __fadd_rn(*c, v);
      *c = v;
    } else if (p.rowsum) {
      const int m = e - M * N;
      for (int q = 0; q < nr; ++q) v = __fadd_rn(v, seg[q * M + m]);
      if (split) p.rowsum_part[(int64_t)z * M + m] = v;
      else p.rowsum[m] = v;
    }
  }
}

// ---- tiny fp32 products (the latent-code terms of the articulated step: per-call folded biases
// b + W_l l, dW_l = db l^T, dl = db^T W_l -- M x N <= 64K outputs, K <= 1024): the 128 x 128
// tiled kernel spent 17-27 us on each (a K pass one or two k-tiles deep, PF register sets and
// split epilogues for a few hundred outputs).  Exact fp32 fmaf (the operand scales are powers
// of two and cancel exactly).  K <= 16: one thread per output, k in order; longer K: one wave
// per output, lane l summing k = l, l + 64, ... in order, then a fixed xor tree (deterministic).
__device__ __forceinline__ void small_store(const Params& p, int64_t m, int64_t n, float v) {
  float* c = p.C + m * p.ldc + n;
  if (p.accumulate) v = __fadd_rn(*c, v);
  if (p.bias) v = __fadd_rn(v, p.bias[n]);
  *c = v;
}
__global__ __launch_bounds__(256) void k_gemm_small_f32(Params p, int a_kc, int b_kc) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= p.M * p.N) return;
  const int64_t m = e / p.N, n = e - m * p.N;
  float v = 0.f;
  for (int64_t k = 0; k < p.K; ++k) {
    const float a = a_kc ? p.A[m * p.lda + k] : p.A[k * p.lda + m];
    const float b = b_kc ? p.B[n * p.ldb + k] : p.B[k * p.ldb + n];
    v = fmaf(a, b, v);
  }
  small_store(p, m, n, v);
}
__global__ __launch_bounds__(256) void k_gemm_small_f32_wave(Params p, int a_kc, int b_kc) {
  const int64_t e = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);  // one wave per output
  const int lane = threadIdx.x & 63;
  if (e >= p.M * p.N) return;  // wave-uniform
  const int64_t m = e / p.N, n = e - m * p.N;
  float v = 0.f;
  for (int64_t k = lane; k < p.K; k += 64) {
    const float a = a_kc ? p.A[m * p.lda + k] : p.A[k * p.lda + m];
    const float b = b_kc ? p.B[n * p.ldb + k] : p.B[k * p.ldb + n];
    v = fmaf(a, b, v);
  }
#pragma unroll
  for (int sh = 32; sh >= 1; sh >>= 1) v = __fadd_rn(v, __shfl_xor(v, sh, 64));
  if (lane == 0) small_store(p, m, n, v);
}

// aon_gemm_small_batch: up to AON_GEMM_SMALL_BATCH_MAX exact-fp32 tiny products in ONE launch,
// each computed exactly as its own aon_gemm launch would (k_gemm_small_f32 for K <= 16: one
// lane per output, a k-ordered fma chain; k_gemm_small_f32_wave above: one wave per output,
// lane-strided chains and the same xor butterfly), and products writing the same C applied in
// argument order in registers (c = accumulate ? c + v : v; + bias), so the result is bit for bit
// that of the launches in sequence.  Work units: 64 outputs (lane kind) or 1 output (wave kind)
// per wave; group g (one C) owns units unit0[g] .. unit0[g + 1] - 1.
struct SmallItem {
  const float* A;
  const float* B;
  float* C;
  const float* bias;
  int64_t lda, ldb, ldc, M, N, K;
  int a_kc, b_kc, accumulate, pad;
};
struct SmallBatch {
  SmallItem it[AON_GEMM_SMALL_BATCH_MAX];   // in group order (a group's items consecutive)
  int gfirst[AON_GEMM_SMALL_BATCH_MAX + 1];  // first item of each group
  int64_t unit0[AON_GEMM_SMALL_BATCH_MAX + 1];
  int ngroups;
};
static_assert(sizeof(SmallBatch) <= 4096, "aon_gemm_small_batch's table must fit the kernel arguments");

__device__ __forceinline__ float small_dot_lane(const SmallItem& f, int64_t m, int64_t n) {
  float v = 0.f;
  for (int64_t k = 0; k < f.K; ++k) {
    const float a = f.a_kc ? f.A[m * f.lda + k] : f.A[k * f.lda + m];
    const float b = f.b_kc ? f.B[n * f.ldb + k] : f.B[k * f.ldb + n];
    v = fmaf(a, b, v);
  }
  return v;
}
__device__ __forceinline__ float small_dot_wave(const SmallItem& f, int64_t m, int64_t n, int lane) {
  float v = 0.f;
  for (int64_t k = lane; k < f.K; k += 64) {
    const float a = f.a_kc ? f.A[m * f.lda + k] : f.A[k * f.lda + m];
    const float b = f.b_kc ? f.B[n * f.ldb + k] : f.B[k * f.ldb + n];
    v = fmaf(a, b, v);
  }
#pragma unroll
  for (int sh = 32; sh >= 1; sh >>= 1) v = __fadd_rn(v, __shfl_xor(v, sh, 64));
  return v;
}
__global__ __launch_bounds__(256) void k_gemm_small_batch(SmallBatch sb) {
  const int64_t u = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);  // wave-uniform
  const int lane = threadIdx.x & 63;
  if (u >= sb.unit0[sb.ngroups]) return;
  int g = 0;
  while (g + 1 < sb.ngroups && u >= sb.unit0[g + 1]) ++g;
  const SmallItem& f0 = sb.it[sb.gfirst[g]];
  const bool wave = f0.K > 16;
  const int64_t e = wave ? u - sb.unit0[g] : (u - sb.unit0[g]) * 64 + lane;
  if (e >= f0.M * f0.N) return;
  const int64_t m = e / f0.N, n = e - m * f0.N;
  float* c = f0.C + m * f0.ldc + n;
  float acc = f0.accumulate ? *c : 0.f;
  for (int i = sb.gfirst[g]; i < sb.gfirst[g + 1]; ++i) {
    const SmallItem& f = sb.it[i];
    const float v = wave ? small_dot_wave(f, m, n, lane) : small_dot_lane(f, m, n);
    acc = f.accumulate ? __fadd_rn(acc, v) : v;
    if (f.bias) acc = __fadd_rn(acc, f.bias[n]);
  }
  if (!wave || lane == 0) *c = acc;
}

template <typename TA, bool BT, typename TB = __bf16>
static void launch_skinny(const Params& p, dim3 grid, hipStream_t st) {
  const dim3 block((unsigned)(2 * p.N));  // 16 row phases x N / 8 column groups
  constexpr int SK = AON_GEMM_SKINNY_SK, SK2 = AON_GEMM_SKINNY_SK2;
  const bool narrow = p.N <= 128;
  switch (p.M) {
#define AON_SKINNY_L(M_)                                                                            \
  if (narrow) hipLaunchKernelGGL((k_gemm_skinny_bf16<M_, TA, BT, SK2, TB>), grid, block, 0, st, p); \
  else hipLaunchKernelGGL((k_gemm_skinny_bf16<M_, TA, BT, SK, TB>), grid, block, 0, st, p)
    case 1: AON_SKINNY_L(1); break;
    case 2: AON_SKINNY_L(2); break;
    case 3: AON_SKINNY_L(3); break;
    default: AON_SKINNY_L(4); break;
#undef AON_SKINNY_L
  }
}

template <typename TA, typename TB>
static void launch_bf(const Params& p, bool va, bool vb, dim3 grid, hipStream_t st) {
#define AON_BF_L(VA_, VB_) \
  hipLaunchKernelGGL((k_gemm_bf16_km<TA, TB, VA_, VB_>), grid, dim3(THREADS), 0, st, p)
  if (va && vb) AON_BF_L(true, true);
  else if (va) AON_BF_L(true, false);
  else if (vb) AON_BF_L(false, true);
  else AON_BF_L(false, false);
#undef AON_BF_L
}

}  // namespace gemm
}  // namespace aon

using namespace aon;
using namespace aon::gemm;

// both operands bf16 and reduction-major in whole 128 x 128 tiles with 16-B runs: the LDS-DMA
// kernel (k_gemm_bf16_dma)
static bool bf16_copy_path(const aon_gemm_args* a) {
  const int64_t b_rdiv = a->b_kc ? 1 : a->b_rdiv;
  return a->mma_bf16 && a->a_bf16 && a->b_bf16 && a->M % BM == 0 && a->N % BN == 0 &&
         b_rdiv == 1 && aligned16(a->A) && aligned16(a->B) && a->lda % 8 == 0 && a->ldb % 8 == 0;
}

// ... in whole 256 x 256 tiles: k_gemm_bf16_dma256 (one tile per 256 x 256 weight gradient)
static bool bf16_copy256_path(const aon_gemm_args* a) {
  return AON_GEMM_DMA256 && AON_GEMM_BF_DMA && bf16_copy_path(a) && a->M % BM2 == 0 &&
         a->N % BM2 == 0;
}

// weight gradient of at most 4 rows on a B of up to 256 columns (k_gemm_skinny_bf16): the bf16
// mode's (B bf16), or the parity mode's in exact fp32 (A and B fp32, no epilogue)
#ifndef AON_GEMM_F32_STREAM
#define AON_GEMM_F32_STREAM 1  // 0: A/B build -- the parity mode's heads / per-ray columns on k_gemm_f16x3
#endif
static bool skinny32(const aon_gemm_args* a) {
  return AON_GEMM_F32_STREAM && !a->mma_bf16 && !a->a_bf16 && !a->b_bf16 && !a->a_kc && !a->b_kc && !a->A2 &&
         !a->bias && !a->mask && !a->relu && !a->exact_fp32;
}
static bool skinny_path(const aon_gemm_args* a) {
  const int64_t b_rdiv = a->b_kc ? 1 : a->b_rdiv;
  return ((a->mma_bf16 && a->b_bf16) || skinny32(a)) && a->M >= 1 && a->M <= 4 && !a->a_tiled &&
         b_rdiv == 1 && a->N % 8 == 0 && a->N <= 256 && aligned16(a->B) && a->ldb % 8 == 0 &&
         !a->k_splits && (a->n_store == 0 || a->n_store == a->N);
}

// tiny fp32 products (k_gemm_small_f32)
static bool small_path(const aon_gemm_args* a) {
  return a->exact_fp32 && !a->mma_bf16 && a->M * a->N <= 65536 && a->K <= 1024 && !a->A2 && !a->mask && !a->relu &&
         !a->rowsum && !a->a_amax && !a->a_tiled && !a->b_tiled && (a->b_kc || a->b_rdiv == 1) &&
         !a->k_splits && (a->n_store == 0 || a->n_store == a->N);
}

// weight gradient against a per-ray B (rdiv > 1): k_gemm_segsum_bf16 -- the bf16 mode's, or
// the parity mode's in exact fp32 (as skinny32)
static bool segsum_path(const aon_gemm_args* a) {
  return (a->mma_bf16 || skinny32(a)) && !a->a_kc && !a->b_kc && a->b_rdiv > 1 && !a->b_tiled &&
         a->M % 8 == 0 && a->M >= 8 && a->M <= 256 && aligned16(a->A) && a->lda % 8 == 0 &&
         !a->k_splits && (a->n_store == 0 || a->n_store == a->N);
}

// fp32 reduction-major x reduction-major weight gradients in whole 128 x 128 tiles with 16-B
// runs: the fp16x3 LDS-DMA kernel (k_gemm_f16x3_dma)
#ifndef AON_GEMM_F16_DMA
#define AON_GEMM_F16_DMA 0  // 1: A/B build of k_gemm_f16x3_dma (bit-identical, measured slower)
#endif
static bool f16_copy_path(const aon_gemm_args* a) {
  const int64_t b_rdiv = a->b_kc ? 1 : a->b_rdiv;
  return AON_GEMM_F16_DMA && !a->mma_bf16 && !a->a_bf16 && !a->b_bf16 && !a->a_kc && !a->b_kc &&
         !a->A2 && !a->bias && !a->mask && !a->relu && a->M % BM == 0 && a->N % BN == 0 &&
         b_rdiv == 1 && aligned16(a->A) && aligned16(a->B) && a->lda % 4 == 0 && a->ldb % 4 == 0;
}

// fp32 reduction-major x reduction-major weight gradients of the fused kernels' tiled tensors
// in one of k_gemm_f1's shapes (M x N = 256 x 256, 128 x 256, 256 x 64), with the caller's
// single-accumulator licence (f16_single)
static bool f1_path(const aon_gemm_args* a) {
  const bool shape = (a->M == 256 && (a->N == 256 || a->N == 64)) || (a->M == 128 && a->N == 256);
  return a->f16_single && !a->mma_bf16 && !a->a_bf16 && !a->b_bf16 && !a->a_kc && !a->b_kc &&
         !a->A2 && !a->bias && !a->mask && !a->relu && !a->exact_fp32 && !a->c_trans &&
         a->a_tiled && a->b_tiled && shape && a->lda == a->M && a->ldb == a->N &&
         a->b_rdiv == 1 && aligned16(a->A) && aligned16(a->B) && a->K >= 8 * 1024;
}
static bool f1_256_path(const aon_gemm_args* a) { return f1_path(a) && a->M == 256 && a->N == 256; }

static int64_t gemm_splits(const aon_gemm_args* a) {
  const int64_t tiles = ((a->M + BM - 1) / BM) * ((a->N + BN - 1) / BN);
  if (small_path(a)) return 1;
  if ((bf16_copy256_path(a) || f1_path(a)) && a->k_splits <= 0) {
    // one workgroup per CU: 256 K chunks of a single 256 x 256 tile (chunks of >= 1024 rows;
    // the coarse level's 266k rows still fill the chip -- 2048-row chunks left half of it idle)
    const int64_t t2 = f1_path(a) ? 1 : (a->M / BM2) * (a->N / BM2);
    if (t2 >= 256 || a->K < 8 * 1024) return 1;
    const int64_t cap = a->K / 1024 < 256 ? a->K / 1024 : 256;
    const int64_t s = 256 / t2 < cap ? 256 / t2 : cap;
    return s >= 8 ? s / 8 * 8 : (s < 1 ? 1 : s);
  }
  // the segment-sum kernel: one chunk of 2048 / M rays (whole segments) per workgroup
  if (segsum_path(a)) {
    const int64_t rays = (a->K + a->b_rdiv - 1) / a->b_rdiv, rb = 2048 / a->M;
    return rays > 0 ? (rays + rb - 1) / rb : 1;
  }
  // the skinny kernel: ~512 chunks of whole 16-row blocks (two workgroups per CU)
  if (skinny_path(a)) {
    const int64_t kc = ((a->K + 511) / 512 + kSkinnyRows - 1) / kSkinnyRows * kSkinnyRows;
    return a->K > 0 ? (a->K + kc - 1) / kc : 1;
  }
  // split the reduction only when the tile grid alone cannot fill the chip and K is long
  if (a->k_splits > 0) return a->k_splits;
  if (tiles >= 512 || a->K < 8 * 1024 || a->A2) return 1;
  if (bf16_copy_path(a) && AON_GEMM_BF_DMA) {
    // one round of 512 workgroups: 128 splits of a 2 x 2 tile grid measured 0.196 ms against
    // 0.216 / 0.233 ms for 192 / 256 (profiles/r02/ab_gemm)
    const int64_t cap = a->K / 2048 < 256 ? a->K / 2048 : 256;
    const int64_t s = 512 / tiles < cap ? 512 / tiles : cap;
    return s >= 8 ? s / 8 * 8 : (s < 1 ? 1 : s);
  }
  // whole rounds of 512 workgroups (2 per CU): two rounds when K is long enough, else one --
  // a grid a few workgroups past a round runs its tail as a second, nearly empty round (a
  // 266k-row weight gradient on 544 workgroups took as long as one on 1024)
  int64_t cap = a->K / 2048;
  if (cap > 256) cap = 256;
  int64_t s = cap * tiles >= 1024 ? 1024 / tiles : (cap < 512 / tiles ? cap : 512 / tiles);
  if (s >= 8) s = s / 8 * 8;  // split_of places chunks in groups of 8 (one per XCD)
  return s < 1 ? 1 : s;
}

extern "C" size_t aon_gemm_workspace_bytes(const aon_gemm_args* a) {
  if (!a) return 0;
  const int64_t s = gemm_splits(a);
  return s > 1 ? (size_t)s * (a->M * a->N + (a->c_trans ? a->N : a->M)) * sizeof(float) : 0;
}

extern "C" int aon_gemm(const aon_gemm_args* a, void* work, size_t work_bytes,
                        aon_stream_t stream) {
  AON_REQUIRE(a, "null args");
  AON_REQUIRE(a->A && a->B && a->C, "null operand");
  AON_REQUIRE(a->M >= 0 && a->N >= 0 && a->K >= 0, "bad shape");
  AON_REQUIRE(a->lda >= 1 && a->ldb >= 1 &&
                  a->ldc >= (a->c_trans ? a->M : (a->n_store > 0 ? a->n_store : a->N)),
              "bad leading dimension (c_trans: ldc >= M, C holds N rows)");
  AON_REQUIRE(!a->A2 || (a->a_kc && a->K1 >= 0 && a->K1 <= a->K && a->lda2 >= 1 && a->a2_rdiv >= 1),
              "A2 needs a_kc, 0 <= K1 <= K, lda2 >= 1, a2_rdiv >= 1");
  AON_REQUIRE(!a->mask || a->ldm >= a->N, "bad mask leading dimension");
  AON_REQUIRE(a->b_kc || a->b_rdiv >= 1, "b_rdiv must be >= 1");
  AON_REQUIRE(a->K < (int64_t(1) << 32) && (a->b_kc || a->b_rdiv < (int64_t(1) << 32)),
              "K and b_rdiv must be below 2^32");
  AON_REQUIRE(a->a_scale > 0.f && a->b_scale > 0.f, "operand scales must be positive");
  const bool bf = a->mma_bf16 != 0;
  AON_REQUIRE(bf || (!a->a_bf16 && !a->b_bf16), "bf16 operands need mma_bf16");
  AON_REQUIRE(!bf || (!a->a_kc && !a->b_kc && !a->A2 && !a->bias && !a->mask && !a->relu &&
                      !a->a_amax),
              "mma_bf16 computes reduction-major weight gradients only (a_kc = b_kc = 0, no A2 / "
              "bias / mask / relu / a_amax)");
  AON_REQUIRE(!a->a_tiled || (!a->a_kc && a->lda == a->M && a->M % 16 == 0),
              "a_tiled: reduction-major A of width lda = M (a multiple of 16)");
  AON_REQUIRE(!a->b_tiled || (!a->b_kc && a->b_rdiv == 1 && a->ldb == a->N && a->N % 16 == 0),
              "b_tiled: reduction-major B of width ldb = N (a multiple of 16), b_rdiv = 1");
  AON_REQUIRE(a->n_store >= 0 && a->n_store <= a->N, "n_store must be in [0, N]");
  AON_REQUIRE(!a->exact_fp32 || small_path(a),
              "exact_fp32: tiny fp32 products only (M N <= 65536, K <= 1024, no A2 / mask / relu / "
              "rowsum / a_amax / tiled operands / k_splits / n_store)");
  AON_REQUIRE(a->n_store == 0 || a->n_store == a->N || bf16_copy_path(a) ||
                  (!a->mma_bf16 && !a->exact_fp32),
              "n_store < N: the bf16 LDS-DMA weight-gradient path (both operands bf16, M and N "
              "multiples of 128) or an fp32 product");
  if (a->M == 0 || a->N == 0) return 0;
  AON_REQUIRE(!a->c_trans || skinny_path(a), "c_trans: the skinny path only (M <= 4)");
  Params p;
  p.c_trans = a->c_trans;
  p.a_tiled = a->a_tiled;
  p.b_tiled = a->b_tiled;
  p.nstore = a->n_store > 0 ? a->n_store : a->N;
  p.M = a->M; p.N = a->N; p.K = a->K;
  p.A = a->A; p.lda = a->lda;
  p.A2 = a->A2; p.lda2 = a->A2 ? a->lda2 : 0; p.K1 = a->A2 ? a->K1 : INT64_MAX;
  p.a2_rdiv = a->A2 ? a->a2_rdiv : 1;
  p.B = a->B; p.ldb = a->ldb; p.b_rdiv = a->b_kc ? 1 : a->b_rdiv;
  p.C = a->C; p.ldc = a->ldc;
  p.bias = a->bias; p.mask = a->mask; p.ldm = a->ldm;
  p.relu = a->relu; p.accumulate = a->accumulate;
  p.sa = a->a_scale; p.sb = a->b_scale; p.inv_s = 1.0f / (a->a_scale * a->b_scale);
  p.sa_bits = a->a_amax;
  const int64_t splits = gemm_splits(a);
  const int64_t kround = skinny_path(a) ? kSkinnyRows : BK;
  p.kchunk = splits > 1 ? ((a->K + splits - 1) / splits + kround - 1) / kround * kround : (a->K > 0 ? a->K : 1);
  if (segsum_path(a)) p.kchunk = 2048 / a->M * a->b_rdiv;  // whole segments per workgroup
  const int64_t zs = a->K > 0 ? (a->K + p.kchunk - 1) / p.kchunk : 1;
  AON_REQUIRE(!a->rowsum || !a->a_kc, "rowsum needs a reduction-major A (a_kc = 0)");
  p.part = nullptr;
  p.rowsum = a->rowsum;
  p.rowsum_part = nullptr;
  if (zs > 1) {
    AON_REQUIRE(work && work_bytes >= (size_t)zs * (a->M * a->N + (a->c_trans ? a->N : a->M)) * sizeof(float),
                "split-K needs aon_gemm_workspace_bytes() of workspace");
    p.part = static_cast<float*>(work);
    p.rowsum_part = p.part + zs * a->M * a->N;
  }
  const bool f1 = f1_path(a);
  const bool t256 = a->mma_bf16 && bf16_copy256_path(a);
  const int64_t bmt = t256 ? BM2 : BM;  // C tile edge of the kernel that runs
  // (k_gemm_f1: the whole product is one tile)
  const int64_t tiles_m = f1 ? 1 : (a->M + bmt - 1) / bmt, tiles_n = f1 ? 1 : (a->N + bmt - 1) / bmt;
  const int64_t gm = tiles_m < 8 ? tiles_m : 8;
  const int64_t blocks = (tiles_m + gm - 1) / gm * gm * tiles_n;
  AON_REQUIRE(blocks < (1ll << 31), "too large");
  p.tiles_m = (int)tiles_m;
  p.tiles_n = (int)tiles_n;
  p.gm = (int)gm;
  p.tblocks = (int)blocks;
  p.zsplit = (int)zs;
  // split-K: one 1-D grid, the tiles of a K chunk on one XCD (split_of)
  const int64_t gx = zs > 1 ? 8 * blocks * ((zs + 7) / 8) : blocks;
  AON_REQUIRE(gx < (1ll << 31), "too large");
  const dim3 grid((unsigned)gx, 1, 1);
  // float4 staging when the 4-element runs are 16-B aligned
  const bool va = aligned16(a->A) && a->lda % 4 == 0 && (!a->A2 || a->K1 % 4 == 0);
  const bool vb = aligned16(a->B) && a->ldb % 4 == 0;
  hipStream_t st = (hipStream_t)stream;
  if (small_path(a)) {
    if (a->K <= 16)
      hipLaunchKernelGGL(k_gemm_small_f32, grid_for(a->M * a->N, 256, 1 << 20), 256, 0, st, p,
                         a->a_kc, a->b_kc);
    else
      hipLaunchKernelGGL(k_gemm_small_f32_wave, grid_for(a->M * a->N, 4, 1 << 20), 256, 0, st, p,
                         a->a_kc, a->b_kc);
    return launch_status(__func__);
  }
  if (bf) {
    // element size of each operand: 8-B (bf16) or 16-B (fp32) runs of 4 rows
    const bool va16 = a->a_bf16 ? (reinterpret_cast<uintptr_t>(a->A) & 7) == 0 && a->lda % 4 == 0 : va;
    const bool vb16 = a->b_bf16 ? (reinterpret_cast<uintptr_t>(a->B) & 7) == 0 && a->ldb % 4 == 0 : vb;
    // both bf16, whole 128 x 128 tiles, 16-B runs: the copy-staged kernels
    const bool tt = bf16_copy_path(a);
    if (segsum_path(a)) {
      const dim3 g((unsigned)zs, 1, 1);
#define AON_SEG_L(TA_, TB_, AT_) hipLaunchKernelGGL((k_gemm_segsum_bf16<TA_, TB_, AT_>), g, dim3(256), 0, st, p)
      if (a->a_bf16 && a->b_bf16) { if (a->a_tiled) AON_SEG_L(__bf16, __bf16, true); else AON_SEG_L(__bf16, __bf16, false); }
      else if (a->a_bf16) { if (a->a_tiled) AON_SEG_L(__bf16, float, true); else AON_SEG_L(__bf16, float, false); }
      else if (a->b_bf16) { if (a->a_tiled) AON_SEG_L(float, __bf16, true); else AON_SEG_L(float, __bf16, false); }
      else { if (a->a_tiled) AON_SEG_L(float, float, true); else AON_SEG_L(float, float, false); }
#undef AON_SEG_L
    } else if (skinny_path(a)) {
      const dim3 g((unsigned)zs, 1, 1);
      if (a->a_bf16 && a->b_tiled) launch_skinny<__bf16, true>(p, g, st);
      else if (a->a_bf16) launch_skinny<__bf16, false>(p, g, st);
      else if (a->b_tiled) launch_skinny<float, true>(p, g, st);
      else launch_skinny<float, false>(p, g, st);
    } else if (t256) hipLaunchKernelGGL(k_gemm_bf16_dma256, grid, dim3(THREADS2), 0, st, p);
    else if (tt && AON_GEMM_BF_DMA) hipLaunchKernelGGL(k_gemm_bf16_dma, grid, dim3(THREADS), 0, st, p);
    else if (tt) hipLaunchKernelGGL(k_gemm_bf16_tt, grid, dim3(THREADS), 0, st, p);
    else if (a->a_bf16 && a->b_bf16) launch_bf<__bf16, __bf16>(p, va16, vb16, grid, st);
    else if (a->a_bf16) launch_bf<__bf16, float>(p, va16, vb16, grid, st);
    else if (a->b_bf16) launch_bf<float, __bf16>(p, va16, vb16, grid, st);
    else launch_bf<float, float>(p, va16, vb16, grid, st);
  } else if (segsum_path(a)) {  // the parity mode's, exact fp32
    const dim3 g((unsigned)zs, 1, 1);
    if (a->a_tiled) hipLaunchKernelGGL((k_gemm_segsum_bf16<float, float, true, false>), g, dim3(256), 0, st, p);
    else hipLaunchKernelGGL((k_gemm_segsum_bf16<float, float, false, false>), g, dim3(256), 0, st, p);
  } else if (skinny_path(a)) {  // the parity mode's, exact fp32
    const dim3 g((unsigned)zs, 1, 1);
    if (a->b_tiled) launch_skinny<float, true, float>(p, g, st);
    else launch_skinny<float, false, float>(p, g, st);
  } else if (f1) {
    if (a->M == 128) hipLaunchKernelGGL((k_gemm_f1<128, 256>), grid, dim3(THREADS2), 0, st, p);
    else if (a->N == 64) hipLaunchKernelGGL((k_gemm_f1<256, 64>), grid, dim3(THREADS2), 0, st, p);
    else hipLaunchKernelGGL((k_gemm_f1<256, 256>), grid, dim3(THREADS2), 0, st, p);
  } else if (f16_copy_path(a)) {
    hipLaunchKernelGGL(k_gemm_f16x3_dma, grid, dim3(THREADS), 0, st, p);
  } else if (a->a_kc && a->b_kc) launch_v<true, true>(p, va, vb, grid, st);
  else if (a->a_kc) launch_v<true, false>(p, va, vb, grid, st);
  else if (a->b_kc) launch_v<false, true>(p, va, vb, grid, st);
  else launch_v<false, false>(p, va, vb, grid, st);
  if (zs > 1) {
    const int rc = launch_status(__func__);
    if (rc) return rc;
    const int64_t outs = a->M * a->N + (a->c_trans ? a->N : a->M);
    if (AON_GEMM_REDUCE16 && outs <= 4096)  // a few hundred outputs: 16 lanes each (sum_z16)
      hipLaunchKernelGGL(k_gemm_reduce<16>, grid_for(16 * outs, 256, 16384), 256, 0, st, p, (int)zs);
    else
      hipLaunchKernelGGL(k_gemm_reduce<4>, grid_for(4 * outs, 256, 16384), 256, 0, st, p, (int)zs);
  }
  return launch_status(__func__);
}

// ---- aon_gemm_batch: one level's bf16 weight gradients in two launches (+ their reduces):
// the one-tile 256 x 256 products on k_gemm_bf16_dma256_batch, the other whole-128 x 128-tile
// products on k_gemm_bf16_dma_batch; any other product runs as aon_gemm.
enum { kBatchNone = 0, kBatch256 = 1, kBatch128 = 2, kBatchF16 = 3, kBatchF1 = 4 };
constexpr int kBatchClasses[] = {kBatchF1, kBatchF16, kBatch256, kBatch128};

static int batch_class(const aon_gemm_args* a) {
  if (a->k_splits > 0 || a->K < 8 * 1024) return kBatchNone;
  if (f1_256_path(a)) return kBatchF1;
  if (f1_path(a)) return kBatchNone;  // k_gemm_f1's other shapes: their own launch
  if (!a->mma_bf16) {
    // fp16x3 weight gradients dW = dY^T X: fp32 reduction-major operands in 16-B runs, whole
    // 128 x 128 tiles, no epilogue beyond accumulate (k_gemm_f16x3<false, false, true, true>)
    const bool ok = !a->a_bf16 && !a->b_bf16 && !a->a_kc && !a->b_kc && !a->A2 && !a->bias &&
                    !a->mask && !a->relu && !a->exact_fp32 && a->b_rdiv == 1 &&
                    a->M % BM == 0 && a->N % BN == 0 && (a->n_store == 0 || a->n_store == a->N) &&
                    aligned16(a->A) && a->lda % 4 == 0 && aligned16(a->B) && a->ldb % 4 == 0 &&
                    !f16_copy_path(a) && (a->M / BM) * (a->N / BN) < 512;
    return ok ? kBatchF16 : kBatchNone;
  }
  if (bf16_copy256_path(a) && a->M == BM2 && a->N == BM2) return kBatch256;
  if (AON_GEMM_BF_DMA && bf16_copy_path(a) && !bf16_copy256_path(a) &&
      (a->M / BM) * (a->N / BN) < 512)
    return kBatch128;
  return kBatchNone;
}

struct BatchPlan {
  int idx[AON_GEMM_BATCH_MAX];  // products of the class, in argument order
  int n;
  int64_t K, kchunk, zs, tiles;
};

static BatchPlan plan_class(const aon_gemm_args* a, int count, int cls) {
  BatchPlan pl{};
  for (int i = 0; i < count; ++i)
    if (batch_class(&a[i]) == cls) {
      if (pl.n == 0) pl.K = a[i].K;
      if (a[i].K == pl.K) pl.idx[pl.n++] = i;  // other K: run alone (aon_gemm)
    }
  if (pl.n < 2) { pl.n = 0; return pl; }
  for (int j = 0; j < pl.n; ++j) {
    const aon_gemm_args* g = &a[pl.idx[j]];
    pl.tiles += cls == kBatch256 ? 1 : cls == kBatchF1 ? (AON_F1_HALF ? 2 : 1)
                                                   : (g->M / BM) * (g->N / BN);
  }
  // 256 x 256 tiles: one workgroup per CU (256 in all), chunks >= 1024 rows; 128 x 128 tiles:
  // two per CU (512), chunks >= 2048 rows -- each product's chunks longer by the batch size;
  // fp16x3: whole rounds of 512 as aon_gemm's split (two when K is long enough)
  const bool one = cls == kBatch256 || cls == kBatchF1;  // one 256 x 256 tile, one WG per CU
  const int64_t wgs = one ? 256 : 512, minrows = one ? 1024 : 2048;
  const int64_t cap = pl.K / minrows < 256 ? pl.K / minrows : 256;
  int64_t s = wgs / pl.tiles < cap ? wgs / pl.tiles : cap;
  if (cls == kBatchF16 && cap * pl.tiles >= 1024) s = 1024 / pl.tiles;
  s = s >= 8 ? s / 8 * 8 : (s < 1 ? 1 : s);
  pl.kchunk = s > 1 ? ((pl.K + s - 1) / s + BK - 1) / BK * BK : pl.K;
  pl.zs = (pl.K + pl.kchunk - 1) / pl.kchunk;
  return pl;
}

static size_t plan_bytes(const aon_gemm_args* a, const BatchPlan& pl) {
  if (pl.n == 0 || pl.zs <= 1) return 0;
  size_t f = 0;
  for (int j = 0; j < pl.n; ++j) f += (size_t)pl.zs * (a[pl.idx[j]].M * a[pl.idx[j]].N + a[pl.idx[j]].M);
  return f * sizeof(float);
}

static bool in_plan(const BatchPlan& pl, int i) {
  for (int j = 0; j < pl.n; ++j)
    if (pl.idx[j] == i) return true;
  return false;
}

// the batch's plans, one per class (kBatchClasses order)
struct BatchPlans {
  BatchPlan pl[4];
  bool planned(int i) const {
    for (const BatchPlan& p : pl)
      if (in_plan(p, i)) return true;
    return false;
  }
};
static BatchPlans plan_all(const aon_gemm_args* a, int count) {
  BatchPlans b;
  for (int c = 0; c < 4; ++c) b.pl[c] = plan_class(a, count, kBatchClasses[c]);
  return b;
}

extern "C" size_t aon_gemm_batch_workspace_bytes(const aon_gemm_args* a, int count) {
  if (!a || count < 1 || count > AON_GEMM_BATCH_MAX) return 0;
  const BatchPlans bp = plan_all(a, count);
  // the launches are stream-ordered: one workspace serves each in turn
  size_t m = 0;
  for (const BatchPlan& p : bp.pl) m = plan_bytes(a, p) > m ? plan_bytes(a, p) : m;
  for (int i = 0; i < count; ++i)
    if (!bp.planned(i)) {
      const size_t b = aon_gemm_workspace_bytes(&a[i]);
      m = b > m ? b : m;
    }
  return m;
}

static int run_plan(const aon_gemm_args* a, const BatchPlan& pl, int cls, void* work,
                    size_t work_bytes, hipStream_t st) {
  ParamsBatch pb;
  pb.count = pl.n;
  pb.zsplit = (int)pl.zs;
  pb.tile0[0] = 0;
  AON_REQUIRE(pl.zs == 1 || (work && work_bytes >= plan_bytes(a, pl)),
              "aon_gemm_batch needs aon_gemm_batch_workspace_bytes() of workspace");
  float* part = static_cast<float*>(work);
  for (int j = 0; j < pl.n; ++j) {
    const aon_gemm_args* g = &a[pl.idx[j]];
    AON_REQUIRE(g->A && g->B && g->C && g->ldc >= (g->n_store > 0 ? g->n_store : g->N),
                "null operand or bad leading dimension");
    AON_REQUIRE(!g->a_tiled || (g->lda == g->M && g->M % 16 == 0), "a_tiled: lda = M");
    AON_REQUIRE(!g->b_tiled || (g->ldb == g->N && g->N % 16 == 0), "b_tiled: ldb = N");
    AON_REQUIRE(g->n_store >= 0 && g->n_store <= g->N, "n_store must be in [0, N]");
    AON_REQUIRE(g->K < (int64_t(1) << 32), "K must be below 2^32");
    Params& p = pb.p[j];
    p = Params{};
    p.a_tiled = g->a_tiled;
    p.b_tiled = g->b_tiled;
    p.nstore = g->n_store > 0 ? g->n_store : g->N;
    p.M = g->M; p.N = g->N; p.K = g->K;
    p.A = g->A; p.lda = g->lda;
    p.K1 = INT64_MAX; p.a2_rdiv = 1;
    p.B = g->B; p.ldb = g->ldb; p.b_rdiv = 1;
    p.C = g->C; p.ldc = g->ldc;
    p.accumulate = g->accumulate;
    p.sa = p.sb = p.inv_s = 1.0f;
    if (cls == kBatchF16 || cls == kBatchF1) {
      AON_REQUIRE(g->a_scale > 0.f && g->b_scale > 0.f, "operand scales must be positive");
      p.sa = g->a_scale; p.sb = g->b_scale; p.inv_s = 1.0f / (g->a_scale * g->b_scale);
      p.sa_bits = g->a_amax;
    }
    p.kchunk = pl.kchunk;
    p.rowsum = g->rowsum;
    p.zsplit = (int)pl.zs;
    const int bmt = cls == kBatch256 || cls == kBatchF1 ? BM2 : BM;
    p.tiles_m = (int)(g->M / bmt);
    p.tiles_n = (int)(g->N / bmt);
    p.gm = p.tiles_m;
    p.tblocks = p.tiles_m * p.tiles_n;
    pb.tile0[j + 1] = pb.tile0[j] + p.tblocks;
    if (pl.zs > 1) {
      p.part = part;
      p.rowsum_part = p.part + pl.zs * g->M * g->N;
      part += pl.zs * (g->M * g->N + g->M);
    }
  }
  // (k_gemm_f1h_batch: two half tiles per product)
  const int wtiles = cls == kBatchF1 && AON_F1_HALF ? 2 * pl.n : pb.tile0[pl.n];
  const dim3 grid((unsigned)(8 * wtiles * ((pl.zs + 7) / 8)), 1, 1);
  if (cls == kBatch256) hipLaunchKernelGGL(k_gemm_bf16_dma256_batch, grid, dim3(THREADS2), 0, st, pb);
  else if (cls == kBatchF1 && AON_F1_HALF) hipLaunchKernelGGL(k_gemm_f1h_batch, grid, dim3(THREADS2), 0, st, pb);
  else if (cls == kBatchF1) hipLaunchKernelGGL(k_gemm_f1_256_batch, grid, dim3(THREADS2), 0, st, pb);
  else if (cls == kBatch128) hipLaunchKernelGGL(k_gemm_bf16_dma_batch, grid, dim3(THREADS), 0, st, pb);
  else hipLaunchKernelGGL(k_gemm_f16x3_batch, grid, dim3(THREADS), 0, st, pb);
  if (pl.zs > 1) {
    const int rc = launch_status("aon_gemm_batch");
    if (rc) return rc;
    int64_t mx = 0;
    for (int j = 0; j < pl.n; ++j) {
      const int64_t w = 4 * (pb.p[j].M * pb.p[j].N + pb.p[j].M);
      mx = w > mx ? w : mx;
    }
    const dim3 rg((unsigned)grid_for(mx, 256, 16384), (unsigned)pl.n, 1);
    hipLaunchKernelGGL(k_gemm_reduce_batch, rg, dim3(256), 0, st, pb);
  }
  return launch_status("aon_gemm_batch");
}

extern "C" int aon_gemm_batch(const aon_gemm_args* a, int count, void* work, size_t work_bytes,
                              aon_stream_t stream) {
  AON_REQUIRE(a && count >= 0 && count <= AON_GEMM_BATCH_MAX, "bad batch");
  hipStream_t st = (hipStream_t)stream;
  const BatchPlans bp = plan_all(a, count);
  for (int c = 0; c < 4; ++c)
    if (bp.pl[c].n) {
      const int rc = run_plan(a, bp.pl[c], kBatchClasses[c], work, work_bytes, st);
      if (rc) return rc;
    }
  for (int i = 0; i < count; ++i)
    if (!bp.planned(i)) {
      const int rc = aon_gemm(&a[i], work, work_bytes, stream);
      if (rc) return rc;
    }
  return 0;
}

// whether two row-major views (rows x cols at row stride ld, cols <= ld) share an element:
// views of one matrix with the same ld compare as row / column rectangles (column slices of one
// dW -- the latent segments -- do not overlap), others by their byte extents
static bool views_overlap(const float* p, int64_t rp, int64_t cp, int64_t lp, const float* q,
                          int64_t rq, int64_t cq, int64_t lq) {
  const intptr_t a = reinterpret_cast<intptr_t>(p), b = reinterpret_cast<intptr_t>(q);
  const intptr_t ae = a + (intptr_t)(((rp - 1) * lp + cp) * 4), be = b + (intptr_t)(((rq - 1) * lq + cq) * 4);
  if (ae <= b || be <= a) return false;
  if (lp != lq || (b - a) % 4 != 0 || cp > lp || cq > lq) return true;
  int64_t d = (b - a) / 4;  // q's first element relative to p's, in elements
  int64_t row = d / lp, col = d % lp;
  if (col < 0) {
    col += lp;
    row -= 1;
  }
  // q covers columns [col, col + cq) of rows row.., wrapping into the next row past ld
  for (int w = 0; w < 2; ++w) {
    const int64_t c0 = w == 0 ? col : 0, c1 = w == 0 ? (col + cq < lp ? col + cq : lp) : col + cq - lp;
    const int64_t r0 = row + w;
    if (c1 <= c0) continue;
    if (r0 < rp && r0 + rq > 0 && c0 < cp && c1 > 0) return true;
  }
  return false;
}

extern "C" int aon_gemm_small_batch(const aon_gemm_args* a, int count, aon_stream_t stream) {
  AON_REQUIRE(a && count >= 0 && count <= AON_GEMM_SMALL_BATCH_MAX, "bad batch");
  if (count == 0) return 0;
  SmallBatch sb{};
  int group_of[AON_GEMM_SMALL_BATCH_MAX];
  int ng = 0;
  const aon_gemm_args* head[AON_GEMM_SMALL_BATCH_MAX];
  for (int i = 0; i < count; ++i) {
    const aon_gemm_args* g = &a[i];
    AON_REQUIRE(small_path(g) && g->A && g->B && g->C && g->M > 0 && g->N > 0 && g->K > 0 &&
                    g->ldc >= g->N,
                "aon_gemm_small_batch: exact_fp32 tiny products only (as aon_gemm's exact_fp32)");
    int gi = -1;
    for (int j = 0; j < ng; ++j)
      if (head[j]->C == g->C) gi = j;
    if (gi < 0) {
      head[ng] = g;
      gi = ng++;
    } else {
      const aon_gemm_args* h = head[gi];
      AON_REQUIRE(h->M == g->M && h->N == g->N && h->ldc == g->ldc && (h->K > 16) == (g->K > 16) &&
                      g->accumulate,
                  "aon_gemm_small_batch: products on one C must match in shape and accumulate");
    }
    group_of[i] = gi;
  }
  // no product may read or write what ANOTHER group writes (groups run concurrently), and no
  // product may read its own group's C other than through `accumulate`
  for (int x = 0; x < ng; ++x) {
    const aon_gemm_args* h = head[x];
    for (int i = 0; i < count; ++i) {
      const aon_gemm_args* g = &a[i];
      const int64_t ar = g->a_kc ? g->M : g->K, ac = g->a_kc ? g->K : g->M;
      const int64_t br = g->b_kc ? g->N : g->K, bc = g->b_kc ? g->K : g->N;
      AON_REQUIRE(group_of[i] == x || !views_overlap(h->C, h->M, h->N, h->ldc, g->C, g->M, g->N, g->ldc),
                  "aon_gemm_small_batch: outputs overlap");
      AON_REQUIRE(!views_overlap(h->C, h->M, h->N, h->ldc, g->A, ar, ac, g->lda) &&
                      !views_overlap(h->C, h->M, h->N, h->ldc, g->B, br, bc, g->ldb) &&
                      (!g->bias || !views_overlap(h->C, h->M, h->N, h->ldc, g->bias, 1, g->N, g->N)),
                  "aon_gemm_small_batch: a product reads a batch output");
    }
  }
  int k = 0;
  sb.unit0[0] = 0;
  for (int x = 0; x < ng; ++x) {
    sb.gfirst[x] = k;
    for (int i = 0; i < count; ++i) {
      if (group_of[i] != x) continue;
      const aon_gemm_args* g = &a[i];
      SmallItem& f = sb.it[k++];
      f.A = g->A; f.B = g->B; f.C = g->C; f.bias = g->bias;
      f.lda = g->lda; f.ldb = g->ldb; f.ldc = g->ldc;
      f.M = g->M; f.N = g->N; f.K = g->K;
      f.a_kc = g->a_kc; f.b_kc = g->b_kc; f.accumulate = g->accumulate;
    }
    const int64_t outs = head[x]->M * head[x]->N;
    sb.unit0[x + 1] = sb.unit0[x] + (head[x]->K > 16 ? outs : (outs + 63) / 64);
  }
  sb.gfirst[ng] = k;
  sb.ngroups = ng;
  const int64_t blocks = (sb.unit0[ng] + 3) / 4;
  AON_REQUIRE(blocks < (1ll << 31), "too large");
  hipLaunchKernelGGL(k_gemm_small_batch, (unsigned)blocks, 256, 0, (hipStream_t)stream, sb);
  return launch_status(__func__);
}
