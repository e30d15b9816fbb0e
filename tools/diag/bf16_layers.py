"""Diagnostic: the bf16 training forward's kept activations (h0..h7, bottleneck, hv) and raw
outputs against the fp32 oracle's, layer by layer, on 64 rays x 65 samples."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "articulated-object-nerf_amd")]
from oracle import nerf_oracle as O  # noqa: E402
from oracle import weights as W  # noqa: E402
from aonerf import train  # noqa: E402
from aonerf import _lib as L  # noqa: E402

g = np.load(os.path.join(ROOT, "tests", "golden", "forward_eval.npz"))
rays = {k: torch.from_numpy(g[k][:64]).cuda() for k in ("rays_o", "rays_d", "viewdirs")}
t = torch.from_numpy(np.ascontiguousarray(g["coarse_t"][:64])).cuda()
B, S = t.shape
R = B * S
params = O.split_state_dict(W.nerf_state_dict(0))
p = params[0]
P = [(p[f"pts_linears.{i}.weight"].cuda(), p[f"pts_linears.{i}.bias"].cuda()) for i in range(8)]
P += [(p[f"{n}.weight"].cuda(), p[f"{n}.bias"].cuda()) for n in ("density_layer", "bottleneck_layer", "views_linear.0", "rgb_layer")]
# oracle activations
xyz = O.cast_rays(t.cpu(), rays["rays_o"].cpu(), rays["rays_d"].cpu())
enc = O.pos_enc(xyz, 0, 10).reshape(R, -1)
venc = O.pos_enc(rays["viewdirs"].cpu(), 0, 4)
x = enc
hs = []
for i in range(8):
    x = torch.relu(x @ p[f"pts_linears.{i}.weight"].T + p[f"pts_linears.{i}.bias"])
    hs.append(x)
    if i == 4:
        x = torch.cat([x, enc], -1)
sig = x @ p["density_layer.weight"].T + p["density_layer.bias"]
bot = x @ p["bottleneck_layer.weight"].T + p["bottleneck_layer.bias"]
cond = venc[:, None, :].expand(B, S, -1).reshape(R, -1)
hv = torch.relu(torch.cat([bot, cond], -1) @ p["views_linear.0.weight"].T + p["views_linear.0.bias"])
rgb = hv @ p["rgb_layer.weight"].T + p["rgb_layer.bias"]
for bf in (False, True):
    raw = torch.empty((R, 4), device="cuda")
    h, b, v = train._forward_level_fused(P, rays["rays_o"], rays["rays_d"], rays["viewdirs"], t, raw, bf16=bf)
    torch.cuda.synchronize()
    tag = "bf16" if bf else "f16x3"
    for i in range(8):
        e = (h[i].float().cpu() - hs[i]).abs().max().item() / hs[i].abs().max().item()
        print(f"{tag} h{i}: max rel-to-max err {e:.2e}")
    for name, got, want in (("bot", b, bot), ("hv", v, hv), ("raw_rgb", raw[:, :3], rgb), ("raw_sigma", raw[:, 3:], sig)):
        e = (got.float().cpu() - want).abs().max().item() / want.abs().max().item()
        print(f"{tag} {name}: max rel-to-max err {e:.2e}")

# which permutation of h0's features reproduces the bf16 kernel's h1?
raw = torch.empty((R, 4), device="cuda")
h, b, v = train._forward_level_fused(P, rays["rays_o"], rays["rays_d"], rays["viewdirs"], t, raw, bf16=True)
h0 = h[0].float().cpu()
h1 = h[1].float().cpu()
W1, b1 = p["pts_linears.1.weight"], p["pts_linears.1.bias"]
f = torch.arange(256)
for name, perm in (("identity", f), ("f^1", f ^ 1), ("f^2", f ^ 2), ("f^3", f ^ 3), ("f^4", f ^ 4),
                   ("f^8", f ^ 8), ("f^16", f ^ 16), ("f^12", f ^ 12), ("f^24", f ^ 24)):
    pred = torch.relu(h0[:, perm] @ W1.T + b1)
    e = (pred - h1).abs().max().item() / h1.abs().max().item()
    print(f"h1 from h0[{name}]: {e:.2e}")
