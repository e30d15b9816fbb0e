"""Render-batch API of the reference's Lightning system (models/vanilla_nerf/model.py:295-348)
and the synthetic SAPIEN cameras used by the benches (datasets/sapien_multi.py:29-72)."""
import math
from collections import defaultdict

import numpy as np
import torch

from . import interface
from .ray_utils import frame_rays

# The reference splits every image into hparams.chunk = 3840-ray pieces (opt.py:103) only to
# bound activation memory on a 11 GB card; on a 288 GB MI355X a whole 640x480 frame is one
# launch per stage.  Outputs do not depend on the chunking (the per-chunk depth clamp of
# helper.py:183 is an identity), so `chunk` only bounds the rays per launch.
DEFAULT_CHUNK = 1 << 21


def _chunks(B, chunk):
    chunk = max(int(chunk or DEFAULT_CHUNK), 1)
    for i in range(0, B, chunk):
        yield i, min(i + chunk, B)


@torch.no_grad()
def render_rays(model, batch, chunk, white_bkgd, near, far):
    """LitNeRF.render_rays (model.py:295-321): fine-level comp_rgb/acc/depth over all rays and
    psnr_legacy against batch['target'] (returned as 'psnr' instead of being logged)."""
    B = batch["rays_o"].shape[0]
    ret = defaultdict(list)
    for i, j in _chunks(B, chunk):
        sub = {k: batch[k][i:j] for k in ("rays_o", "rays_d", "viewdirs")}
        fine = model(sub, False, white_bkgd, near, far)[1]
        ret["comp_rgb"].append(fine[0])
        ret["acc"].append(fine[1])
        ret["depth"].append(fine[2])
    out = {k: torch.cat(v, 0) for k, v in ret.items()}
    if "target" in batch:
        out["psnr"] = interface.psnr_legacy(out["comp_rgb"], batch["target"]).mean()
    return out


@torch.no_grad()
def render_rays_test(model, batch, chunk, white_bkgd, near, far):
    """LitNeRF.render_rays_test (model.py:323-348) -> {target, instance_mask, rgb}."""
    out = render_rays(model, {k: v for k, v in batch.items() if k != "target"}, chunk, white_bkgd,
                      near, far)
    test_output = {"rgb": out["comp_rgb"]}
    for k in ("target", "instance_mask"):
        if k in batch:
            test_output[k] = batch[k]
    return test_output


@torch.no_grad()
def render_frame(model, c2w, H, W, focal, near=2.0, far=6.0, white_bkgd=True, p0=0, n=None,
                 chunk=None, timers=None):
    """Fused ray generation + two-level render of pixels [p0, p0+n) of an H x W frame.
    Returns (n, 5) = [rgb(3), depth, acc] per pixel (the payload of the frame gather)."""
    n = H * W - p0 if n is None else n
    rays = frame_rays(c2w, H, W, focal, p0, n)
    out = torch.empty((n, 5), device=rays["rays_o"].device)
    for i, j in _chunks(n, chunk):
        sub = {k: v[i:j] for k, v in rays.items()}
        fine = model(sub, False, white_bkgd, near, far, timers=timers)[1]
        out[i:j, 0:3] = fine[0]
        out[i:j, 3] = fine[2]
        out[i:j, 4] = fine[1]
    return out


# ----------------------------------------------------------------------------- cameras
def create_spheric_poses(radius=4.0, n=40, phi=-30.0):
    """datasets/sapien_multi.py:29-72 -> (n, 4, 4) float32 camera-to-world matrices."""

    def trans_t(t):
        return np.array([[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 1, t], [0, 0, 0, 1]], np.float32)

    def rot_phi(p):
        c, s = np.cos(p), np.sin(p)
        return np.array([[1, 0, 0, 0], [0, c, -s, 0], [0, s, c, 0], [0, 0, 0, 1]], np.float32)

    def rot_theta(th):
        c, s = np.cos(th), np.sin(th)
        return np.array([[c, 0, -s, 0], [0, 1, 0, 0], [s, 0, c, 0], [0, 0, 0, 1]], np.float32)

    flip = np.array([[-1, 0, 0, 0], [0, 0, 1, 0], [0, 1, 0, 0], [0, 0, 0, 1]], np.float32)
    out = []
    for angle in np.linspace(-180, 180, n + 1)[:-1]:
        m = torch.from_numpy(trans_t(radius))
        m = torch.from_numpy(rot_phi(phi / 180.0 * np.pi)) @ m
        m = torch.from_numpy(rot_theta(angle / 180.0 * np.pi)) @ m
        out.append(torch.from_numpy(flip) @ m)
    return torch.stack(out, 0)


def sapien_focal(H, fovy_deg=35.0):
    """SAPIEN pinhole (datagen/data_gen.py:60-67): focal = 0.5*H / tan(0.5*fovy)."""
    return 0.5 * H / math.tan(0.5 * math.radians(fovy_deg))
