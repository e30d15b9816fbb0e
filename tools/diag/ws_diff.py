"""Where the weight-streamed render MLP (mlp_ws.hip) and the LDS-ring one (mlp_f16x3.hip) differ:
indices, position in the 128-sample workgroup, channel, both values and an fp64 evaluation of the
same sample at the kernels' fp16x3 operands' exact values (oracle, CPU).

    python tools/diag/ws_diff.py [--rays 1000] [--samples 65]
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "articulated-object-nerf_amd")]
from aonerf import _lib as L  # noqa: E402
from aonerf.model import NeRF  # noqa: E402
from aonerf.synthetic import init_like_reference  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rays", type=int, default=1000)
ap.add_argument("--samples", type=int, default=65)
ap.add_argument("--art", action="store_true")
a = ap.parse_args()
B, S = a.rays, a.samples
g = torch.Generator().manual_seed(B + S)
o = (torch.randn(B, 3, generator=g) * 0.1 + torch.tensor([0.0, -3.5, 2.0])).cuda()
d = torch.nn.functional.normalize(torch.randn(B, 3, generator=g), dim=-1).cuda()
t = torch.sort(torch.rand(B, S, generator=g) * 4 + 2, dim=-1).values.cuda()
lib = L.lib()
if a.art:
    from aonerf.model_autodecoder import NeRF_AE_Art
    from aonerf.synthetic import art_latents

    net = init_like_reference(NeRF_AE_Art()).cuda()
    lat = art_latents(0, device="cuda")
    mlp = net.fine_mlp

    def run():
        return mlp.forward_rays(o, d, d, t, lat)
else:
    mlp = init_like_reference(NeRF()).cuda().fine_mlp

    def run():
        return mlp.forward_rays(o, d, d, t, 0)
outs = []
for df in (0, 1, 0, 1):
    lib.aon_mlp_set_dataflow(df)
    outs.append(run().cpu())
lib.aon_mlp_set_dataflow(0)
print("streamed run-to-run equal:", torch.equal(outs[0], outs[2]), " ws run-to-run equal:",
      torch.equal(outs[1], outs[3]))
if not a.art:  # the fused TRAINING forward (same epilogue arithmetic, fp32 kept tensors) on the same rows
    from aonerf import train

    P = [(m.weight.detach(), m.bias.detach()) for m in mlp._layers()]
    raw_t = torch.empty((B * S, 4), device="cuda")
    h, bot, hv = train._forward_level_fused(P, o, d, d, t, raw_t)
    raw_t = raw_t.cpu()
    print("train-forward raw == streamed:", torch.equal(raw_t, outs[0]), " == ws:", torch.equal(raw_t, outs[1]),
          " max |train - ws|", (raw_t - outs[1]).abs().max().item())
a0, a1 = outs[0].numpy(), outs[1].numpy()
diff = np.abs(a0 - a1)
bad = np.argwhere(diff > 0)
print(f"{len(bad)} of {a0.size} values differ, max {diff.max():.3e}")
rows = np.unique(bad[:, 0])
print("rows:", len(rows), "channels:", np.bincount(bad[:, 1], minlength=4).tolist())
print("row % 128 histogram (16-sample tiles):", np.bincount((rows % 128) // 16, minlength=8).tolist())
print("row // 128 (workgroups):", np.unique(rows // 128)[:20].tolist(), "of", (a0.shape[0] + 127) // 128)
for r, ch in bad[:12]:
    print(f"  row {r} (wg {r // 128}, slot {r % 128}) ch {ch}: streamed {a0[r, ch]:.9g} ws {a1[r, ch]:.9g}")
