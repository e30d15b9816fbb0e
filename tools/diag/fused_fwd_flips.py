"""Diagnostic: where do the fused training forward's kept activations (aon_mlp_fwd_train) and
the layer-by-layer GEMM forward disagree on ReLU masks, on the train_step golden's rays?"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "articulated-object-nerf_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from aonerf import train  # noqa: E402
from aonerf import _lib as L  # noqa: E402
from aonerf.model import NeRF  # noqa: E402
from aonerf.synthetic import init_like_reference  # noqa: E402

g = dict(np.load(os.path.join(ROOT, "tests/golden/train_step.npz")))
net = init_like_reference(NeRF()).cuda()
b = {k: torch.from_numpy(g[k]).cuda() for k in ("rays_o", "rays_d", "viewdirs")}
with torch.no_grad():
    ret = net(b, True, True, 2.0, 6.0, u_coarse=torch.from_numpy(g["u_coarse"]).cuda(),
              u_fine=torch.from_numpy(g["u_fine"]).cuda(), return_intermediates=True)
for level, mlp in ((0, net.coarse_mlp), (1, net.fine_mlp)):
    t = ret[level][3]["t_vals"].contiguous()
    B, S = t.shape
    P = [(m.weight.detach(), m.bias.detach()) for m in mlp._layers()]
    raw_f = torch.empty((B * S, 4), device="cuda")
    h_f, bot_f, hv_f = train._forward_level_fused(P, b["rays_o"], b["rays_d"], b["viewdirs"], t, raw_f)
    enc = torch.empty((B * S, 63), device="cuda")
    L.call("aon_cast_rays", L.ptr(b["rays_o"]), L.ptr(b["rays_d"]), L.ptr(t), B, S, None, 0, None,
           0, 10, L.ptr(enc), L.stream())
    venc = torch.empty((B, 27), device="cuda")
    L.call("aon_pos_enc", L.ptr(b["viewdirs"]), B, 0, 4, L.ptr(venc), L.stream())
    raw_g = torch.empty((B * S, 4), device="cuda")
    h_g, bot_g, hv_g = train._forward_level(P, enc, venc, S, raw_g)
    # fp64 reference activations from the same encodings
    x = enc.double()
    for i in range(8):
        W, bb = P[i]
        if i == 5:
            x = torch.cat([x, enc.double()], -1)
        x = torch.relu(x @ W.double().T + bb.double())
        hf, hg = h_f[i].double(), h_g[i].double()
        flips_f = ((hf > 0) != (x > 0)).sum().item()
        flips_g = ((hg > 0) != (x > 0)).sum().item()
        ef = (hf - x).abs().max().item() / x.abs().max().item()
        eg = (hg - x).abs().max().item() / x.abs().max().item()
        idx = ((hf > 0) != (x > 0)).nonzero()
        sample = [(int(r), int(c), float(hf[r, c]), float(x[r, c])) for r, c in idx[:3].tolist()]
        print(f"level {level} h{i}: fused err {ef:.2e} flips {flips_f} | gemm err {eg:.2e} flips {flips_g} {sample}")
