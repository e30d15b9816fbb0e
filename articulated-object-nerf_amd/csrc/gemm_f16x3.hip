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
};

// start of the 4-element run (k, row .. row + 3) of a reduction-major operand (row % 4 == 0):
// row-major storage row k / rdiv, or the 16-row tiled layout of the fused training kernels
__device__ __forceinline__ int64_t km_off(int64_t k, int64_t row, int64_t ld, int64_t rdiv,
                                          bool tiled) {
  if (tiled) return (k & ~int64_t(15)) * ld + 256 * (row >> 4) + 16 * (k & 15) + (row & 15);
  return (rdiv == 1 ? k : k / rdiv) * ld + row;
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
__global__ __launch_bounds__(THREADS, 2) void k_gemm_f16x3(Params p) {
  // A's prescale: a constant, or per call from the gradient's max |x| (exact powers of two)
  float sa = p.sa, inv_s = p.inv_s;
  if (p.sa_bits) {
    const float gs = grad_scale(*p.sa_bits);
    sa = __fmul_rn(sa, gs);
    inv_s = __fdiv_rn(inv_s, gs);
  }
  __shared__ __align__(16) _Float16 smem[2 * STAGE];  // 2 stages x (A hi, A lo, B hi, B lo)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  int tm, tn;
  int tile, z;
  if (!split_of(p, tile, z)) return;      // padding block of the last chunk group
  if (!tile_of(p, tile, tm, tn)) return;  // padding block of the last XCD group (uniform exit)
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
        float* c = p.C + m * p.ldc + n;
        if (p.accumulate) v = __fadd_rn(*c, v);
        if (p.bias) v = __fadd_rn(v, p.bias[n]);
        if (p.relu) v = fmaxf(v, 0.0f);
        if (p.mask && !(p.mask[m * p.ldm + n] > 0.0f)) v = 0.0f;
        *c = v;
      }
    }
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

__global__ void k_gemm_reduce(Params p, int splits) {
  const int64_t total = p.M * p.N;
  const int64_t extra = p.rowsum ? p.M : 0;  // rowsum entries ride along as e >= total
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total + extra;
       e += (int64_t)gridDim.x * blockDim.x) {
    if (e >= total) {
      const int64_t m = e - total;
      p.rowsum[m] = sum_z(p.rowsum_part + m, p.M, splits);
      continue;
    }
    const int64_t m = e / p.N, n = e - m * p.N;
    float v = sum_z(p.part + e, total, splits);
    float* c = p.C + m * p.ldc + n;
    if (p.accumulate) v = __fadd_rn(*c, v);
    if (p.bias) v = __fadd_rn(v, p.bias[n]);
    if (p.relu) v = fmaxf(v, 0.0f);
    if (p.mask && !(p.mask[m * p.ldm + n] > 0.0f)) v = 0.0f;
    *c = v;
  }
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

// 128 rows x 32 k of a reduction-major operand: thread t -> rows rq..rq+3 (rq = 16 (t >> 5) +
// 4 (t & 3)), k = kq..kq+3 (kq = 4 ((t >> 2) & 7)); one 4-element row run per k
template <typename T, bool VEC>
struct TileLoadKM {
  float r[4][4];  // [k][row]
  __device__ __forceinline__ void load(const T* p, int64_t ld, int64_t rdiv, int64_t row0,
                                       int64_t R, int64_t k0, int64_t kend, int tid, bool tiled) {
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
                                       int64_t R, int64_t k0, int64_t kend, int tid, bool tiled) {
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

template <typename TA, typename TB, bool VA, bool VB>
__global__ __launch_bounds__(THREADS, 2) void k_gemm_bf16_km(Params p) {
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
  typename KMLoader<TA, VA>::type ta;
  typename KMLoader<TB, VB>::type tb;
  f4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  const bool want_rows = p.rowsum && tn == 0;
  float rs[4] = {0.f, 0.f, 0.f, 0.f};
  auto load = [&](int kt) {
    const int64_t k0 = kbeg + (int64_t)kt * BK;
    ta.load(A, p.lda, 1, m0, p.M, k0, kend, tid, p.a_tiled);
    tb.load(Bm, p.ldb, p.b_rdiv, n0, p.N, k0, kend, tid, p.b_tiled);
  };
  auto store = [&](int stage) {
    if (want_rows) ta.add_rows(rs);
    __bf16* s = smem + stage * STAGE_BF;
    ta.store(s, tid);
    tb.store(s + PLANE, tid);
  };
  if (nk > 0) {
    load(0);
    store(0);
  }
  __syncthreads();
  const int g = lane >> 4, r16 = lane & 15;
  for (int kt = 0; kt < nk; ++kt) {
    const int P = kt & 1;
    if (kt + 1 < nk) load(kt + 1);  // global loads in flight under this step's MFMAs
    const __bf16* s = smem + P * STAGE_BF;
    bf8 b[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      b[j] = *reinterpret_cast<const bf8*>(s + PLANE + (wn * 64 + 16 * j + r16) * ROWH + 8 * g);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bf8 a = *reinterpret_cast<const bf8*>(s + (wm * 64 + 16 * i + r16) * ROWH + 8 * g);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) store(1 - P);
    __syncthreads();
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
        float* c = p.C + m * p.ldc + n;
        if (p.accumulate) v = __fadd_rn(*c, v);
        *c = v;
      }
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

static int64_t gemm_splits(const aon_gemm_args* a) {
  const int64_t tiles = ((a->M + BM - 1) / BM) * ((a->N + BN - 1) / BN);
  // split the reduction only when the tile grid alone cannot fill the chip and K is long
  if (a->k_splits > 0) return a->k_splits;
  if (tiles >= 512 || a->K < 8 * 1024 || a->A2) return 1;
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
  return s > 1 ? (size_t)s * (a->M * a->N + a->M) * sizeof(float) : 0;
}

extern "C" int aon_gemm(const aon_gemm_args* a, void* work, size_t work_bytes,
                        aon_stream_t stream) {
  AON_REQUIRE(a, "null args");
  AON_REQUIRE(a->A && a->B && a->C, "null operand");
  AON_REQUIRE(a->M >= 0 && a->N >= 0 && a->K >= 0, "bad shape");
  AON_REQUIRE(a->lda >= 1 && a->ldb >= 1 && a->ldc >= a->N, "bad leading dimension");
  AON_REQUIRE(!a->A2 || (a->a_kc && a->K1 >= 0 && a->K1 <= a->K && a->lda2 >= 1 && a->a2_rdiv >= 1),
              "A2 needs a_kc, 0 <= K1 <= K, lda2 >= 1, a2_rdiv >= 1");
  AON_REQUIRE(!a->mask || a->ldm >= a->N, "bad mask leading dimension");
  AON_REQUIRE(a->b_kc || a->b_rdiv >= 1, "b_rdiv must be >= 1");
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
  if (a->M == 0 || a->N == 0) return 0;
  Params p;
  p.a_tiled = a->a_tiled;
  p.b_tiled = a->b_tiled;
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
  p.kchunk = splits > 1 ? ((a->K + splits - 1) / splits + BK - 1) / BK * BK : (a->K > 0 ? a->K : 1);
  const int64_t zs = a->K > 0 ? (a->K + p.kchunk - 1) / p.kchunk : 1;
  AON_REQUIRE(!a->rowsum || !a->a_kc, "rowsum needs a reduction-major A (a_kc = 0)");
  p.part = nullptr;
  p.rowsum = a->rowsum;
  p.rowsum_part = nullptr;
  if (zs > 1) {
    AON_REQUIRE(work && work_bytes >= (size_t)zs * (a->M * a->N + a->M) * sizeof(float),
                "split-K needs aon_gemm_workspace_bytes() of workspace");
    p.part = static_cast<float*>(work);
    p.rowsum_part = p.part + zs * a->M * a->N;
  }
  const int64_t tiles_m = (a->M + BM - 1) / BM, tiles_n = (a->N + BN - 1) / BN;
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
  if (bf) {
    // element size of each operand: 8-B (bf16) or 16-B (fp32) runs of 4 rows
    const bool va16 = a->a_bf16 ? (reinterpret_cast<uintptr_t>(a->A) & 7) == 0 && a->lda % 4 == 0 : va;
    const bool vb16 = a->b_bf16 ? (reinterpret_cast<uintptr_t>(a->B) & 7) == 0 && a->ldb % 4 == 0 : vb;
    if (a->a_bf16 && a->b_bf16) launch_bf<__bf16, __bf16>(p, va16, vb16, grid, st);
    else if (a->a_bf16) launch_bf<__bf16, float>(p, va16, vb16, grid, st);
    else if (a->b_bf16) launch_bf<float, __bf16>(p, va16, vb16, grid, st);
    else launch_bf<float, float>(p, va16, vb16, grid, st);
  } else if (a->a_kc && a->b_kc) launch_v<true, true>(p, va, vb, grid, st);
  else if (a->a_kc) launch_v<true, false>(p, va, vb, grid, st);
  else if (a->b_kc) launch_v<false, true>(p, va, vb, grid, st);
  else launch_v<false, false>(p, va, vb, grid, st);
  if (zs > 1) {
    const int rc = launch_status(__func__);
    if (rc) return rc;
    hipLaunchKernelGGL(k_gemm_reduce, grid_for(a->M * a->N + a->M, 256, 4096), 256, 0, st, p, (int)zs);
  }
  return launch_status(__func__);
}
