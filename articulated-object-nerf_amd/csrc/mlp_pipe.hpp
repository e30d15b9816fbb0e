// LDS weight-stream pipeline shared by the MLP kernels (see mlp_layout.hpp).
//
// The packed stream is cut into kChunk-block (16-KB) chunks.  Chunk c travels HBM/L2 ->
// registers (issued when chunk c-1 is first used) -> LDS buffer c & 1 (written when chunk c is
// first used, then one workgroup barrier).  Buffer c & 1 was last read during chunk c - 2, which
// every wave finished before the barrier of chunk c - 1, so one barrier per chunk suffices.
#pragma once

#include "aon_common.hpp"
#include "mlp_layout.hpp"

#ifndef AON_DMA_ASM
#define AON_DMA_ASM 1
#endif

namespace aon {
namespace mlp {

template <int THREADS>
struct Pipe {
  static constexpr int kChunk = mlp::kChunk;
  static constexpr int kUsedBlocks = kBlocks;
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
  __device__ __forceinline__ void start() { load(0); }
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

namespace aon {
namespace mlp {

typedef __attribute__((address_space(3))) const f4 lds_f4;
typedef __attribute__((address_space(3))) const float lds_float;
// LDS address of a __shared__ pointer, hidden from the compiler so it stays a base register:
// ds_read's immediate offset reaches only 64 KB, and past that hipcc rebuilds every address
// from the kernel's LDS origin with a v_or per read
template <typename T>
__device__ __forceinline__ __attribute__((address_space(3))) const T* opaque_lds(const T* p) {
  uint32_t a = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(p));
  asm volatile("" : "+v"(a));
  return reinterpret_cast<__attribute__((address_space(3))) const T*>(static_cast<uintptr_t>(a));
}

// s_waitcnt vmcnt(n) lgkmcnt(0) (gfx9 encoding: vmcnt[3:0] | [15:14], expcnt[6:4], lgkmcnt[11:8]).
// The builtin wants a literal: after unrolling n is a constant and the switch folds to one case.
// (vmcnt has 6 bits; the switch covers the 0..31 the pipelines can need.)
// LGKM = 0 also drains the LDS reads, LGKM = 15 leaves them alone.
#define AON_WAIT_VM(n) \
  __builtin_amdgcn_s_waitcnt(((n) & 0xF) | (((n) >> 4) << 14) | (0x7 << 4) | (LGKM << 8))
template <int LGKM>
__device__ __forceinline__ void wait_vm(int n) {
  switch (n) {
    case 0: AON_WAIT_VM(0); break;
    case 1: AON_WAIT_VM(1); break;
    case 2: AON_WAIT_VM(2); break;
    case 3: AON_WAIT_VM(3); break;
    case 4: AON_WAIT_VM(4); break;
    case 5: AON_WAIT_VM(5); break;
    case 6: AON_WAIT_VM(6); break;
    case 7: AON_WAIT_VM(7); break;
    case 8: AON_WAIT_VM(8); break;
    case 9: AON_WAIT_VM(9); break;
    case 10: AON_WAIT_VM(10); break;
    case 11: AON_WAIT_VM(11); break;
    case 12: AON_WAIT_VM(12); break;
    case 13: AON_WAIT_VM(13); break;
    case 14: AON_WAIT_VM(14); break;
    case 15: AON_WAIT_VM(15); break;
    case 16: AON_WAIT_VM(16); break;
    case 17: AON_WAIT_VM(17); break;
    case 18: AON_WAIT_VM(18); break;
    case 19: AON_WAIT_VM(19); break;
    case 20: AON_WAIT_VM(20); break;
    case 21: AON_WAIT_VM(21); break;
    case 22: AON_WAIT_VM(22); break;
    case 23: AON_WAIT_VM(23); break;
    case 24: AON_WAIT_VM(24); break;
    case 25: AON_WAIT_VM(25); break;
    case 26: AON_WAIT_VM(26); break;
    case 27: AON_WAIT_VM(27); break;
    case 28: AON_WAIT_VM(28); break;
    case 29: AON_WAIT_VM(29); break;
    case 30: AON_WAIT_VM(30); break;
    default: AON_WAIT_VM(31); break;
  }
}
#undef AON_WAIT_VM
__device__ __forceinline__ void wait_vm_lgkm0(int n) { wait_vm<0>(n); }

// LDS-DMA ring: chunk c is copied HBM/L2 -> LDS buffer c % NBUF by global_load_lds (16 B per
// lane, no VGPR staging), NBUF - 1 chunks ahead of its first use.  At the first use of chunk c
// every wave waits until its own copies of chunk c have landed (counted vmcnt: the copies of the
// chunks after c stay in flight), drains its LDS reads, and joins one workgroup barrier; then
// the buffer of chunk c - 1 (fully read: every wave is past its last use) is refilled with
// chunk c + NBUF - 1.  All LDS of the kernel lives in ONE __shared__ array (a second object can
// make hipcc drain vmcnt before every ds_read, cdna_hip_programming.md section 5 item 4a).
//
// LEAD < NBUF - 1 (chunks in flight ahead of the one in use) refills the buffer of chunk
// c + LEAD - NBUF <= c - 2 instead: every wave finished reading it before it could reach chunk
// c - 1's fragments (LDS reads complete in order and the prefetch reaches less than a chunk
// ahead), so begin() need not drain the wave's LDS reads before the barrier.
template <int THREADS, int NBUF, int CHUNK, int STREAM_BLOCKS = kStreamBlocks,
          int USED_BLOCKS = kBlocks, int LEAD = NBUF - 1>
struct DmaPipe {
  static constexpr int kChunk = CHUNK;  // 1-KB blocks per chunk (shadows the fp32 pipe's)
  static constexpr int kNumChunks = STREAM_BLOCKS / CHUNK;
  static constexpr int kUsedBlocks = USED_BLOCKS;  // blocks past this are padding, never read
  static_assert(kNumChunks * CHUNK == STREAM_BLOCKS, "stream must be whole chunks");
  static constexpr int kCopies = kChunk * 64 / THREADS;  // 16-B copies per thread per chunk
  static_assert(kCopies * THREADS == kChunk * 64, "chunk must split evenly over threads");
  static_assert(NBUF >= 2, "ring needs two buffers");
  static_assert(LEAD >= 1 && LEAD <= NBUF - 1, "chunks ahead");
  f4* wbuf;  // [NBUF][kChunk * 64] f4
  const f4* __restrict__ src;
  int tid, lane;
  uint32_t voff = 0, m0_wave = 0;  // 16 * tid; LDS byte address of wbuf + this wave's 64 f4

  __device__ __forceinline__ void issue(int c) {
#pragma unroll
    for (int i = 0; i < kCopies; ++i) {
#if AON_DMA_ASM
      // Opaque to the compiler: with a visible LDS-DMA in flight hipcc drains lgkmcnt to 0
      // before every ds_read (defeating the fragment prefetch); hidden, it keeps counted
      // lgkmcnt(N) waits.  Ordering is ours: begin() waits vmcnt for this wave's copies and
      // lgkmcnt(0), then s_barrier, before any wave reads the chunk or reuses its slot.
      // Addressing is all scalar: saddr = chunk base + i * THREADS * 16 B (SGPR pair), the
      // per-lane 32-bit offset 16 * tid is loop-invariant, M0 = this wave's 1-KB LDS slot.
      const f4* gbase = src + (size_t)c * kChunk * 64 + i * THREADS;
      const uint32_t m0 = m0_wave + static_cast<uint32_t>(((c % NBUF) * kChunk * 64 + i * THREADS) * 16);
      // M0 is reserved to the compiler, which on gfx950 only uses it for LDS-DMA / sendmsg /
      // GWS -- none of them elsewhere in these kernels (checked in the ISA)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
      asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, %2"
                   :
                   : "s"(m0), "v"(voff), "s"(gbase)
                   : "memory", "m0");
#pragma clang diagnostic pop
#else
      f4* dst = wbuf + (c % NBUF) * kChunk * 64;
      const int e = i * THREADS + tid;  // 16-B element of the chunk; LDS dst is lane-linear
      __builtin_amdgcn_global_load_lds(
          reinterpret_cast<const void*>(src + (size_t)c * kChunk * 64 + e),
          reinterpret_cast<__attribute__((address_space(3))) void*>(
              reinterpret_cast<uintptr_t>(dst + e - lane)),
          16, 0, 0);
#endif
    }
  }
  __device__ __forceinline__ void start() {
    voff = static_cast<uint32_t>(tid) * 16u;
    bases();
    m0_wave = __builtin_amdgcn_readfirstlane(
        static_cast<uint32_t>(reinterpret_cast<uintptr_t>(wbuf + (tid & ~63))));
#pragma unroll
    for (int c = 0; c < LEAD && c < kNumChunks; ++c) issue(c);
  }
  __device__ __forceinline__ void begin(int c) {
#ifdef AON_ABLATE_RING  // timing-only build: every chunk reads buffer 0 (wrong results)
    if (c > 0) return;
#endif
    // copies issued after chunk c's: chunks c+1 .. min(c+LEAD-1, last)
    const int ahead = (c + LEAD - 1 < kNumChunks - 1 ? c + LEAD - 1 : kNumChunks - 1) - c;
    static_assert((LEAD - 1) * kCopies <= 31, "vmcnt budget");
    // chunk 0's barrier also publishes what the kernel staged in LDS before the loop
    if (LEAD == NBUF - 1 || c == 0)
      wait_vm<0>(ahead * kCopies);
    else
      wait_vm<15>(ahead * kCopies);
    __builtin_amdgcn_s_barrier();
    if (c + LEAD < kNumChunks) issue(c + LEAD);
  }
  __device__ __forceinline__ f4 block(int b) const {
#ifdef AON_ABLATE_RING
    return wbuf[(b % kChunk) * 64 + lane];
#endif
    // ds_read's immediate offset reaches 64 KB: blocks past it read from a second per-lane base
    // (else hipcc materialises every such address with a v_or)
    const int off = ((b / kChunk) % NBUF) * kChunk * 64 + (b % kChunk) * 64;
    return off < kHiOff ? lbase[off] : lbase_hi[off - kHiOff];
  }
  static constexpr int kHiOff = 4096;  // f4 = 64 KB
  const f4* lbase = nullptr;           // wbuf + lane
  lds_f4* lbase_hi = nullptr;          // wbuf + lane + 64 KB
  __device__ __forceinline__ void bases() {
    lbase = wbuf + lane;
    lbase_hi = opaque_lds(lbase + kHiOff);
  }
};

}  // namespace mlp
}  // namespace aon
