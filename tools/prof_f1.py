#!/usr/bin/env python3
"""One launch of the parity mode's fine-level 256 x 256 weight-gradient batch (aon_gemm_batch's
f16_single class, k_gemm_f1_256_batch: 8 products of K = 790,528 tiled fp32 rows, distinct
operands) for counter passes (scripts/prof_f1_counters.sh); --reps N times it with HIP events."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "articulated-object-nerf_amd"))

import torch  # noqa: E402

from aonerf import _lib as L  # noqa: E402
from aonerf import tiles  # noqa: E402
from aonerf.linalg import batched, gemm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=1)
    ap.add_argument("--products", type=int, default=8)
    args = ap.parse_args()
    K, M, N, n = 4096 * 193, 256, 256, args.products
    g = torch.Generator(device="cuda").manual_seed(0)
    A = [tiles.tile(torch.randn((K, M), device="cuda", generator=g) * 1e-3) for _ in range(n)]
    B = [tiles.tile(torch.rand((K, N), device="cuda", generator=g)) for _ in range(n)]
    Cs = [torch.empty((M, N), device="cuda") for _ in range(n)]
    rs = [torch.empty((M,), device="cuda") for _ in range(n)]
    word = torch.zeros((1,), dtype=torch.int32, device="cuda")
    L.call("aon_absmax", L.ptr(A[0]), A[0].numel(), L.ptr(word), L.stream())

    def level():
        with batched():
            for i in range(n):
                gemm(Cs[i], A[i], B[i], M, N, K, lda=M, a_kc=False, ldb=N, b_kc=False, ldc=N,
                     rowsum=rs[i], a_scale=1.0, b_scale=8.0, a_amax=word, a_tiled=True,
                     b_tiled=True, f16_single=True)

    torch.cuda.synchronize()
    times = []
    for _ in range(args.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        level()
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1))
    t = sorted(times)[len(times) // 2]
    print(f"f1 batch of {n}: {t:.3f} ms, {n * K * (M + N) * 4 / t / 1e9:.2f} TB/s, "
          f"mfma_frac {3 * n * 2 * K * M * N / (t * 1e-3) / 2.5e15:.3f}")


if __name__ == "__main__":
    main()
