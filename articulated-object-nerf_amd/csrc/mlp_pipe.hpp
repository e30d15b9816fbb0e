// LDS weight-stream pipeline shared by the MLP kernels (see mlp_layout.hpp).
//
// The packed stream is cut into kChunk-block (16-KB) chunks.  Chunk c travels HBM/L2 ->
// registers (issued when chunk c-1 is first used) -> LDS buffer c & 1 (written when chunk c is
// first used, then one workgroup barrier).  Buffer c & 1 was last read during chunk c - 2, which
// every wave finished before the barrier of chunk c - 1, so one barrier per chunk suffices.
#pragma once

#include "aon_common.hpp"
#include "mlp_layout.hpp"

namespace aon {
namespace mlp {

template <int THREADS>
struct Pipe {
  static constexpr int kStageRegs = kChunk * 64 / THREADS;  // f4 per thread per chunk
  static_assert(kStageRegs * THREADS == kChunk * 64, "chunk must split evenly over threads");
  f4* wbuf;  // [2][kChunk * 64] f4 in LDS
  const f4* __restrict__ src;
  f4 stage[kStageRegs];
  int tid, lane;

  __device__ __forceinline__ void load(int c) {
#pragma unroll
    for (int i = 0; i < kStageRegs; ++i) stage[i] = src[(size_t)c * kChunk * 64 + tid + i * THREADS];
  }
  // first use of chunk c: publish it to LDS, then prefetch chunk c + 1
  __device__ __forceinline__ void begin(int c) {
    f4* dst = wbuf + (c & 1) * kChunk * 64;
#pragma unroll
    for (int i = 0; i < kStageRegs; ++i) dst[tid + i * THREADS] = stage[i];
    __syncthreads();
    if (c + 1 < kNumChunks) load(c + 1);
  }
  __device__ __forceinline__ f4 block(int b) const {
    return wbuf[((b / kChunk) & 1) * kChunk * 64 + (b % kChunk) * 64 + lane];
  }
};

}  // namespace mlp
}  // namespace aon
