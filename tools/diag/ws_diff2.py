"""Localise the rgb-only difference between the weight-streamed and LDS-ring render MLPs
(sigma agreed bit for bit: the trunk is identical): rerun both with parts of the view path
neutralised -- enc_dir columns of views_linear.0 zeroed (is it pos_enc(viewdirs)?), viewdirs = 0,
bottleneck weights zeroed (bottleneck = its bias) -- and count differing rgb values each time.

    python tools/diag/ws_diff2.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "articulated-object-nerf_amd")]
from aonerf import _lib as L  # noqa: E402
from aonerf.model import NeRF  # noqa: E402
from aonerf.synthetic import init_like_reference  # noqa: E402

B, S = 1000, 65
g = torch.Generator().manual_seed(B + S)
o = (torch.randn(B, 3, generator=g) * 0.1 + torch.tensor([0.0, -3.5, 2.0])).cuda()
d = torch.nn.functional.normalize(torch.randn(B, 3, generator=g), dim=-1).cuda()
t = torch.sort(torch.rand(B, S, generator=g) * 4 + 2, dim=-1).values.cuda()
lib = L.lib()


def count(mlp, vd):
    outs = []
    for df in (0, 1):
        lib.aon_mlp_set_dataflow(df)
        outs.append(mlp.forward_rays(o, d, vd, t, 0).cpu())
    lib.aon_mlp_set_dataflow(0)
    diff = (outs[0] - outs[1]).abs()
    return int((diff[:, :3] > 0).sum()), int((diff[:, 3] > 0).sum()), float(diff.max())


base = init_like_reference(NeRF()).cuda().fine_mlp
print("baseline:                         rgb / sigma differing, max:", count(base, d), flush=True)
with torch.no_grad():
    m = init_like_reference(NeRF()).cuda().fine_mlp
    m.views_linear[0].weight[:, 256:] = 0
    print("enc_dir columns of views_linear.0 = 0:", count(m, d), flush=True)
    print("viewdirs = 0:                       ", count(base, torch.zeros_like(d)), flush=True)
    m = init_like_reference(NeRF()).cuda().fine_mlp
    m.bottleneck_layer.weight.zero_()
    print("bottleneck weights = 0:             ", count(m, d), flush=True)
    m = init_like_reference(NeRF()).cuda().fine_mlp
    m.views_linear[0].weight[:, :256] = 0
    print("bottleneck columns of views_linear.0 = 0:", count(m, d), flush=True)
