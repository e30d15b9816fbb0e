#!/usr/bin/env python3
"""Time the HBM-bound per-ray kernels of the render on frame-sized inputs (B = 307,200 rays):
k_composite_fwd at the fine (193) and coarse (65) sample counts and k_sample_pdf (65 coarse
t -> 128 fine samples merged), with HIP events on the launch stream.  Prints algorithmic GB/s
(bench.py's composite_bytes; pdf: t 65 + weights 63 read, 193 written = 1,284 B/ray) and the
fraction of the 8 TB/s HBM peak.  AONERF_LIB selects the library (A/B of builds)."""
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


def composite_bytes(S):
    return 16 * S + 4 * S + 12 + 20 + 4 * S


def timed(fn, reps):
    st = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(reps)]
    for a, b in evs:
        a.record(st)
        fn()
        b.record(st)
    torch.cuda.synchronize()
    return sorted(a.elapsed_time(b) for a, b in evs)[reps // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=int, default=640 * 480)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    B = args.rays
    g = torch.Generator(device="cuda").manual_seed(0)
    dev = "cuda"
    res = {"lib": os.environ.get("AONERF_LIB", "default"), "rays": B}
    for S in (193, 65):
        t = torch.sort(2.0 + 4.0 * torch.rand((B, S), device=dev, generator=g), -1).values
        raw = torch.rand((B * S, 4), device=dev, generator=g)
        dirs = torch.nn.functional.normalize(torch.randn((B, 3), device=dev, generator=g), dim=-1)
        outs = [torch.empty(s, device=dev) for s in ((B, 3), (B,), (B, S), (B,))]

        def run():
            L.call("aon_composite_fwd", L.ptr(raw), 4, L.ptr(raw[:, 3:]), 4, L.ptr(t), L.ptr(dirs),
                   B, S, 1, L.ACT_NONE, *[L.ptr(o) for o in outs], L.stream())  # activations ran in the MLP

        ms = timed(run, args.reps)
        gbs = composite_bytes(S) * B / (ms * 1e-3) / 1e9
        res[f"composite_S{S}"] = {"ms": ms, "GB/s": gbs, "frac_hbm": gbs / 8000.0}
    Sc, Nf = 65, 128
    tc = torch.sort(2.0 + 4.0 * torch.rand((B, Sc), device=dev, generator=g), -1).values
    w = torch.rand((B, Sc), device=dev, generator=g)
    u = torch.linspace(0.0, 1.0 - 2 ** -32, Nf, device=dev)  # eval-mode u, shared by every ray
    tn = torch.empty((B, Sc + Nf), device=dev)

    def run_pdf():
        L.call("aon_sample_pdf", None, 0, L.ptr(w[:, 1:]), Sc, B, Sc - 1, Nf, L.ptr(u), 0,
               L.ptr(tc), Sc, None, None, L.ptr(tn), None, L.stream())

    ms = timed(run_pdf, args.reps)
    pb = 4 * (Sc + (Sc - 2) + Sc + Nf)
    gbs = pb * B / (ms * 1e-3) / 1e9
    res["sample_pdf"] = {"ms": ms, "GB/s": gbs, "frac_hbm": gbs / 8000.0, "bytes_per_ray": pb}
    # the fused coarse composite + resample (aon_composite_march) on the coarse level's inputs
    raw = torch.rand((B * Sc, 4), device=dev, generator=g)
    dirs = torch.nn.functional.normalize(torch.randn((B, 3), device=dev, generator=g), dim=-1)
    outs = [torch.empty(s, device=dev) for s in ((B, 3), (B,), (B,))]

    def run_march():
        L.call("aon_composite_march", L.ptr(raw), L.ptr(tc), L.ptr(dirs), B, Sc, 1, L.ACT_NONE,
               L.ptr(u), 0, Nf, L.ptr(outs[0]), L.ptr(outs[1]), None, L.ptr(outs[2]), L.ptr(tn),
               L.stream())

    ms = timed(run_march, args.reps)
    mb = 16 * Sc + 4 * Sc + 12 + 20 + 4 * (Sc + Nf)
    gbs = mb * B / (ms * 1e-3) / 1e9
    import hashlib

    res["march"] = {"ms": ms, "GB/s": gbs, "frac_hbm": gbs / 8000.0, "bytes_per_ray": mb,
                    "sha256_t_fine": hashlib.sha256(tn.cpu().numpy().tobytes()).hexdigest()[:16],
                    "sha256_rgb": hashlib.sha256(outs[0].cpu().numpy().tobytes()).hexdigest()[:16]}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
