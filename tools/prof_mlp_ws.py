"""A/B of the render MLP's two dataflows: the release library's LDS-ring weight stream
(mlp_f16x3.hip) and the weight-streamed kernel of the variant library (mlp_ws.hip,
`make -C articulated-object-nerf_amd/csrc variant-ws`) on the same packed weights, interleaved launches on the fine
level of the bench frame (307,200 rays x 193 samples), raw outputs compared bit for bit.

    python tools/prof_mlp_ws.py [--rays 307200] [--samples 193] [--reps 5]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "articulated-object-nerf_amd")]
from aonerf import _lib as L  # noqa: E402
from aonerf.model import NeRF  # noqa: E402
from aonerf.synthetic import init_like_reference  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rays", type=int, default=307200)
ap.add_argument("--samples", type=int, default=193)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--art", action="store_true", help="the articulated MLP (NeRF_AE_Art fine level)")
a = ap.parse_args()
g = torch.Generator(device="cuda").manual_seed(0)
B, S = a.rays, a.samples
o = torch.randn(B, 3, device="cuda", generator=g) * 0.1 + torch.tensor([0.0, -3.5, 2.0], device="cuda")
d = torch.nn.functional.normalize(torch.randn(B, 3, device="cuda", generator=g), dim=-1)
t = torch.sort(torch.rand(B, S, device="cuda", generator=g) * 4 + 2, dim=-1).values
V = L.variant("ws")
if a.art:
    from aonerf.model_autodecoder import NeRF_AE_Art
    from aonerf.synthetic import art_latents

    net = init_like_reference(NeRF_AE_Art()).cuda()
    lat = art_latents(0, device="cuda")
    MAC = 714_880
    packed = net.fine_mlp.packed_weights(lat)

    def fwd(df):
        if df == 0:
            return net.fine_mlp.forward_rays(o, d, d, t, lat)
        raw = torch.empty((B * S, 4), device="cuda")
        assert V.aon_mlp_art_fwd(L.ptr(packed), L.ptr(o), L.ptr(d), L.ptr(d), L.ptr(t), B, S, 0,
                                 L.ptr(raw), L.stream()) == 0
        return raw
else:
    net = init_like_reference(NeRF()).cuda()
    MAC = 593_408
    packed = net.fine_mlp.packed_weights()

    def fwd(df):
        if df == 0:
            return net.fine_mlp.forward_rays(o, d, d, t)
        raw = torch.empty((B * S, 4), device="cuda")
        assert V.aon_mlp_fwd(L.ptr(packed), L.PREC["f16x3"], L.ptr(o), L.ptr(d), L.ptr(d),
                             L.ptr(t), B, S, 0, L.ptr(raw), L.stream()) == 0
        return raw
ms = {0: [], 1: []}
same = True
for r in range(a.reps):
    outs = {}
    for df in (0, 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        raw = fwd(df)
        e1.record()
        torch.cuda.synchronize()
        ms[df].append(e0.elapsed_time(e1))
        outs[df] = raw
    eq = torch.equal(outs[0], outs[1])
    same &= eq
    if not eq:
        diff = (outs[0] - outs[1]).abs()
        print(f"rep {r}: MISMATCH max {diff.max().item():.3e} at {int(diff.argmax())}, "
              f"{int((diff > 0).sum())} values differ", flush=True)
    print(f"rep {r}: streamed {ms[0][-1]:.2f} ms  ws {ms[1][-1]:.2f} ms  bit-equal {eq}", flush=True)
flop = 2 * MAC * B * S
res = {k: {"median_ms": float(np.median(v[1:] or v)),
           "tflops": flop / float(np.median(v[1:] or v)) / 1e9,
           "frac_f16x3_peak": flop / float(np.median(v[1:] or v)) / 1e9 / (2500 / 3)}
       for k, v in (("streamed", ms[0]), ("ws", ms[1]))}
res["bit_equal"] = bool(same)
print(json.dumps(res))
