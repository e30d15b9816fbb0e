"""Profiling driver (GPU): bench.py's C5 training records alone, with their per-kernel
breakdown (fine level forward / chain / weight gradients), one JSON line per record:

    python tools/prof_train_records.py [--records bf16,art_bf16,f16x3,art] [--steps 10]
"""
import argparse
import json
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "articulated-object-nerf_amd")]

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", default="bf16,art_bf16")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()
    args = types.SimpleNamespace(steps=a.steps, warmup=a.warmup)
    for name in a.records.split(","):
        art = name.startswith("art")
        prec = "bf16" if name.endswith("bf16") else "f16x3"
        rec = bench.bench_train(args, 1, 0, 0, art=art, precision=prec)
        kern = {k: round(v["ms"], 4) for k, v in rec["roofline"].get("kernels", {}).items()}
        print(json.dumps({"record": name, "ms_per_step": rec["ms_per_step"], "fine": kern}),
              flush=True)


if __name__ == "__main__":
    main()
