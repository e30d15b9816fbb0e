#!/usr/bin/env python3
"""The fused coarse march (aon_composite_march) alone on a 640x480 frame's coarse level
(B = 307,200 rays, S = 65, Ns = 128, eval-mode u), for rocprofv3 counter passes
(scripts/prof_march_counters.sh).  AONERF_LIB selects the library (A/B of builds).  Prints the
median HIP-event time and the algorithmic GB/s (bench.py's march_bytes)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "articulated-object-nerf_amd"))
if os.environ.get("AONERF_LIB"):  # an A/B build of the library (tools only)
    from aonerf import _lib as _aon_lib  # noqa: E402

    _aon_lib.use_library(os.environ["AONERF_LIB"])

import torch  # noqa: E402

from aonerf import _lib as L  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=int, default=640 * 480)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    B, S, Ns = args.rays, 65, 128
    g = torch.Generator(device="cuda").manual_seed(0)
    t = torch.sort(2.0 + 4.0 * torch.rand((B, S), device="cuda", generator=g), -1).values
    raw = torch.rand((B * S, 4), device="cuda", generator=g)
    dirs = torch.nn.functional.normalize(torch.randn((B, 3), device="cuda", generator=g), dim=-1)
    u = torch.linspace(0.0, 1.0 - 2 ** -32, Ns, device="cuda")
    outs = [torch.empty(s, device="cuda") for s in ((B, 3), (B,), (B,), (B, S + Ns))]

    def run():
        L.call("aon_composite_march", L.ptr(raw), L.ptr(t), L.ptr(dirs), B, S, 1, L.ACT_NONE,
               L.ptr(u), 0, Ns, L.ptr(outs[0]), L.ptr(outs[1]), None, L.ptr(outs[2]),
               L.ptr(outs[3]), L.stream())

    run()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.reps)]
    for a, b in ev:
        a.record()
        run()
        b.record()
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) for a, b in ev)[args.reps // 2]
    mb = (16 * S + 4 * S + 12 + 20 + 4 * (S + Ns)) * B
    print(json.dumps({"lib": os.environ.get("AONERF_LIB", "default"), "ms": ms,
                      "GB/s": mb / (ms * 1e-3) / 1e9, "frac_hbm": mb / (ms * 1e-3) / 8e12}))


if __name__ == "__main__":
    main()
