"""Diagnostics: trace one ray of the 'a' frame fixture through every stage, GPU vs oracle."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "articulated-object-nerf_amd")]
from oracle import nerf_oracle as O  # noqa: E402
from oracle import weights as W  # noqa: E402
from aonerf import helper, _lib as L  # noqa: E402
from aonerf.model import NeRF  # noqa: E402
from aonerf.ray_utils import frame_rays  # noqa: E402

ray_id = int(sys.argv[1]) if len(sys.argv) > 1 else 354
g = dict(np.load(os.path.join(ROOT, "tests/golden/render_frame.npz")))
H, Wd, nc, chunk = (int(x) for x in g["a_hw"])
sd = W.nerf_state_dict(0)
params = O.split_state_dict(sd)
net = NeRF().cuda()
net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
c2w = torch.from_numpy(g["a_c2w"])
rays_g = frame_rays(c2w, H, Wd, float(g["a_focal"]))
dirs = O.get_ray_directions(H, Wd, float(g["a_focal"]))
o, v, d = O.get_rays(dirs, c2w, True)
print("ray dir diff", (rays_g["rays_d"].cpu() - d).abs().max().item())
sel = [ray_id]
rc = {"rays_o": o[sel], "rays_d": d[sel], "viewdirs": v[sel]}
rg = {k: x[sel].contiguous() for k, x in rays_g.items()}
ret_o, inter_o = O.nerf_forward(params, rc, False, True, 2.0, 6.0, return_intermediates=True)
ret_g = net(rg, False, True, 2.0, 6.0, return_weights=True)
print("fine rgb gpu", ret_g[1][0].cpu().numpy(), "oracle", ret_o[1][0].numpy(), "golden", g["a_comp_rgb"][ray_id])
# coarse level
tc, _ = helper.sample_along_rays(rg["rays_o"], rg["rays_d"], 64, 2.0, 6.0, False, False)
print("coarse t diff", (tc.cpu() - inter_o[0]["t_vals"]).abs().max().item())
wg = ret_g[0][3].cpu()
print("coarse w diff", (wg - inter_o[0]["weights"]).abs().max().item())
# fine t: gpu pdf on gpu weights vs oracle pdf on gpu weights vs oracle pdf on oracle weights
mids = 0.5 * (tc[..., 1:] + tc[..., :-1])
tf_g, _ = helper.sample_pdf(mids, ret_g[0][3][..., 1:-1], rg["rays_o"], rg["rays_d"], tc, 128, False)
tf_o_gw, _ = O.sample_pdf(mids.cpu(), wg[..., 1:-1], o[sel], d[sel], tc.cpu(), 128, False)
tf_o = inter_o[1]["t_vals"]
print("fine t: gpu-pdf(gpu w) vs oracle-pdf(gpu w)", (tf_g.cpu() - tf_o_gw).abs().max().item())
print("fine t: oracle-pdf(gpu w) vs oracle", (tf_o_gw - tf_o).abs().max().item())
diff = (tf_o_gw - tf_o).abs()[0]
k = int(diff.argmax())
print("  worst sample", k, "t gpu-w", tf_o_gw[0, k].item(), "t oracle", tf_o[0, k].item())
w_o = inter_o[0]["weights"][0]
print("  coarse weights (oracle) near:", w_o.numpy()[max(0, k // 3 - 4): k // 3 + 4])
# MLP on identical fine t
raw_g = net.fine_mlp.forward_rays(rg["rays_o"], rg["rays_d"], rg["viewdirs"], tf_o.cuda().contiguous())
xyz = O.cast_rays(tf_o, o[sel], d[sel])
rr, rs = O.mlp_forward(params[1], O.pos_enc(xyz, 0, 10), O.pos_enc(v[sel], 0, 4))
print("fine raw on oracle t: rgb diff", (raw_g[:, :3].cpu() - rr[0]).abs().max().item(),
      "sigma diff", (raw_g[:, 3].cpu() - rs[0, :, 0]).abs().max().item())
print("oracle fine raw sigma range", rs.min().item(), rs.max().item())
