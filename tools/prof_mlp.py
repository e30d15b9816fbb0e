"""Run the fused MLP kernel alone (one launch per precision) for counter collection / timing.

    python tools/prof_mlp.py [--rows N] [--precision f16x3|fp32|all] [--reps R]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "articulated-object-nerf_amd")]
if os.environ.get("AONERF_LIB"):  # an A/B build of the library (tools only)
    from aonerf import _lib as _aon_lib  # noqa: E402

    _aon_lib.use_library(os.environ["AONERF_LIB"])
from aonerf.model import NeRF  # noqa: E402
from aonerf.synthetic import init_like_reference  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rays", type=int, default=307200 // 4)
ap.add_argument("--samples", type=int, default=193)
ap.add_argument("--precision", default="all")
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--dump", default="", help="write the last raw output's sha256 here (A/B bit-identity)")
a = ap.parse_args()
g = torch.Generator(device="cuda").manual_seed(0)
B, S = a.rays, a.samples
o = torch.randn(B, 3, device="cuda", generator=g) * 0.1 + torch.tensor([0.0, -3.5, 2.0], device="cuda")
d = torch.nn.functional.normalize(torch.randn(B, 3, device="cuda", generator=g), dim=-1)
t = torch.sort(torch.rand(B, S, device="cuda", generator=g) * 4 + 2, dim=-1).values
net = init_like_reference(NeRF()).cuda()
precs = ["fp32", "f16x3"] if a.precision == "all" else [a.precision]
for p in precs:
    net.set_precision(p)
    for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        raw = net.fine_mlp.forward_rays(o, d, d, t)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        print(f"{p}: {B * S} rows {ms:.2f} ms -> {2 * 593408 * B * S / ms / 1e9:.1f} TFLOP/s algorithmic")
    if a.dump:
        import hashlib
        h = hashlib.sha256(raw.detach().cpu().numpy().tobytes()).hexdigest()
        with open(a.dump, "a") as f:
            f.write(f"{os.environ.get('AONERF_LIB', 'default')} {p} {h}\n")
