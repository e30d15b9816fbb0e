#!/usr/bin/env python3
"""Time the fine-level weight-gradient GEMM of the C5 training step (aon_gemm, dW = dZ^T X:
K = 4096 x 193 = 790,528 rows, M = N = 256, both operands in the fused kernels' tiled layout)
in the bf16 mode and the f16x3 mode, with HIP events on the launch stream; prints ms, the
algorithmic HBM fraction (K (M + N) operand bytes) and the MFMA fraction.  AONERF_LIB selects
the library (A/B of builds); "sha" hashes C and the row sums (bit-identity across builds)."""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "articulated-object-nerf_amd"))
if os.environ.get("AONERF_LIB"):  # an A/B build of the library (tools only)
    from aonerf import _lib as _aon_lib  # noqa: E402

    _aon_lib.use_library(os.environ["AONERF_LIB"])

import torch  # noqa: E402

from aonerf import tiles  # noqa: E402
from aonerf.linalg import gemm  # noqa: E402


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(reps)]
    for a, b in evs:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return sorted(a.elapsed_time(b) for a, b in evs)[reps // 2]


def main():
    K, M, N = 4096 * 193, 256, 256
    g = torch.Generator(device="cuda").manual_seed(0)
    ks = int(os.environ.get("AON_KSPLITS", "0"))  # 0: aon_gemm's own split of K
    res = {"lib": os.environ.get("AONERF_LIB", "default"), "k_splits": ks}
    for mode, dt, peak in (("bf16", torch.bfloat16, 2500.0), ("f16x3", torch.float32, 2500.0 / 3)):
        A = tiles.tile((torch.randn((K, M), device="cuda", generator=g) * 1e-3).to(dt))
        B = tiles.tile(torch.rand((K, N), device="cuda", generator=g).to(dt))
        C = torch.empty((M, N), device="cuda")
        rs = torch.empty((M,), device="cuda")
        bf = mode == "bf16"

        def run():
            gemm(C, A, B, M, N, K, lda=M, a_kc=False, ldb=N, b_kc=False, ldc=N, rowsum=rs,
                 a_scale=1.0 if bf else 2.0 ** 10, b_scale=1.0 if bf else 8.0, mma_bf16=bf,
                 a_tiled=True, b_tiled=True, k_splits=ks)

        ms = timed(run)
        nbytes = K * (M + N) * A.element_size()
        run()
        torch.cuda.synchronize()
        sha = hashlib.sha256(C.cpu().numpy().tobytes() + rs.cpu().numpy().tobytes()).hexdigest()[:16]
        res[mode] = {"ms": ms, "hbm_frac": nbytes / (ms * 1e-3) / 8e12,
                     "mfma_frac": 2 * K * M * N / (ms * 1e-3) / 1e12 / peak, "sha": sha}
    # the parity mode's 256 x 256 products with the single-accumulator licence (k_gemm_f1_256),
    # alone and as one level's batch of 8 (distinct operands, as the step's products)
    from aonerf.linalg import batched
    A = [tiles.tile(torch.randn((K, M), device="cuda", generator=g) * 1e-3) for _ in range(8)]
    B = [tiles.tile(torch.rand((K, N), device="cuda", generator=g)) for _ in range(8)]
    Cs = [torch.empty((M, N), device="cuda") for _ in range(8)]
    rss = [torch.empty((M,), device="cuda") for _ in range(8)]
    word = torch.zeros((1,), dtype=torch.int32, device="cuda")
    from aonerf import _lib as L
    L.call("aon_absmax", L.ptr(A[0]), A[0].numel(), L.ptr(word), L.stream())

    def one(i):
        gemm(Cs[i], A[i], B[i], M, N, K, lda=M, a_kc=False, ldb=N, b_kc=False, ldc=N,
             rowsum=rss[i], a_scale=1.0, b_scale=8.0, a_amax=word, a_tiled=True, b_tiled=True,
             f16_single=True)

    def level():
        with batched():
            for i in range(8):
                one(i)

    for name, fn, n in (("f16_single", lambda: one(0), 1), ("f16_single_b8", level, 8)):
        ms = timed(fn, 10)
        fn()
        torch.cuda.synchronize()
        sha = hashlib.sha256(b"".join(Cs[i].cpu().numpy().tobytes() + rss[i].cpu().numpy().tobytes()
                                      for i in range(n))).hexdigest()[:16]
        res[name] = {"ms": ms, "hbm_frac": n * K * (M + N) * 4 / (ms * 1e-3) / 8e12,
                     "mfma_frac": n * 2 * K * M * N / (ms * 1e-3) / 1e12 / (2500.0 / 3), "sha": sha}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
