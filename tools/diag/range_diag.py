"""Diagnostic: f16x3 range guard on pts_linears.0-scaled golden weights (tests/test_gpu_range.py).
Prints, per scale, the oracle's largest hidden activation, the kernel's raw error vs the oracle,
non-finite outputs and the pack's status word."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "articulated-object-nerf_amd")]
from oracle import nerf_oracle as O  # noqa: E402
import test_gpu_range as R  # noqa: E402
from aonerf import _lib as L  # noqa: E402


def golden(name):
    return np.load(os.path.join(ROOT, "tests", "golden", name))


for target in (6e3, 1e4, 2e4, 1e5):
    g, sd, params, m = R._scaled(golden, target)
    net = R._net(sd)
    rays = {k: torch.from_numpy(g[k]).cuda() for k in ("rays_o", "rays_d", "viewdirs")}
    t = torch.from_numpy(np.ascontiguousarray(g["coarse_t"])).cuda()
    raw = net.coarse_mlp.forward_rays(rays["rays_o"], rays["rays_d"], rays["viewdirs"], t)
    torch.cuda.synchronize()
    packed = net.coarse_mlp._packed
    st = ctypes.c_uint32(7)
    L.call("aon_mlp_read_status", L.ptr(packed), packed.numel() * 4, ctypes.byref(st),
           L.stream(packed.device))
    tc = torch.from_numpy(g["coarse_t"])
    xyz = O.cast_rays(tc, torch.from_numpy(g["rays_o"]), torch.from_numpy(g["rays_d"]))
    rr, rs = O.mlp_forward(params[0], O.pos_enc(xyz, 0, 10), O.pos_enc(torch.from_numpy(g["viewdirs"]), 0, 4))
    ref = torch.cat([rr.reshape(-1, 3), rs.reshape(-1, 1)], -1)
    r = raw.cpu()
    fin = torch.isfinite(r)
    err = (r - ref).abs()[fin].max().item() if fin.any() else float("nan")
    print(f"target {target:.0e}: oracle max |h| {m:.1f}; status {st.value}; non-finite {int((~fin).sum())}; "
          f"max |raw| {r[fin].abs().max().item():.3e}; max |raw - oracle| {err:.3e}; "
          f"max |oracle raw| {ref.abs().max().item():.3e}", flush=True)
