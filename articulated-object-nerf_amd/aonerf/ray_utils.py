"""Drop-in for ``get_ray_directions`` / ``get_rays`` of the reference
(datasets/ray_utils.py:71-90, 118-159), on the MI355X, plus a fused frame/tile generator."""
import torch

from . import _lib as L


def _c2w_host(c2w):
    c = torch.as_tensor(c2w, dtype=torch.float32).detach().cpu()[:3, :4].contiguous()
    return (L.ctypes.c_float * 12)(*c.reshape(-1).tolist())


def get_ray_directions(H, W, focal, device="cuda"):
    """reference ray_utils.py:71-90 -> (H, W, 3) camera-space directions (no +0.5 centring)."""
    dirs = torch.empty((H, W, 3), device=device)
    L.require_gpu(dirs)
    L.call("aon_ray_directions", H, W, float(focal), L.ptr(dirs), L.stream(dirs.device))
    return dirs


def get_rays(directions, c2w, output_view_dirs=False, output_radii=False):
    """reference ray_utils.py:118-159.

    Returns (rays_o, rays_d) or, with ``output_view_dirs``, (rays_o, viewdirs, rays_d) where --
    as in the reference, whose ``viewdirs`` aliases ``rays_d`` and is normalised in place --
    both direction outputs are the same unit vectors; ``output_radii`` appends radii (H*W,).
    """
    L.require_gpu(directions)
    directions = L.contig(directions)
    n = directions.numel() // 3
    dev = directions.device
    rays_o = torch.empty((n, 3), device=dev)
    rays_d = torch.empty((n, 3), device=dev)
    radii = None
    H = W = 0
    if output_radii:
        if directions.dim() != 3:
            raise ValueError("output_radii needs an (H, W, 3) direction grid")
        H, W = directions.shape[:2]
        radii = torch.empty((n,), device=dev)
    L.call("aon_get_rays", L.ptr(directions), n, _c2w_host(c2w), L.ptr(rays_o), L.ptr(rays_d), None,
           H, W, L.ptr(radii), L.stream(dev))
    if output_view_dirs:
        out = (rays_o, rays_d, rays_d)
        return out + (radii,) if output_radii else out
    return rays_o, rays_d


def frame_rays(c2w, H, W, focal, p0=0, n=None, device="cuda"):
    """get_ray_directions + get_rays(output_view_dirs=True) fused, for pixels [p0, p0+n) of the
    row-major H x W frame -> dict(rays_o, rays_d, viewdirs) (the dataset's ray dict,
    datasets/sapien.py:152-154)."""
    n = H * W - p0 if n is None else n
    rays_o = torch.empty((n, 3), device=device)
    rays_d = torch.empty((n, 3), device=device)
    L.require_gpu(rays_o)
    L.call("aon_frame_rays", H, W, float(focal), _c2w_host(c2w), p0, n, L.ptr(rays_o),
           L.ptr(rays_d), None, L.stream(rays_o.device))
    return {"rays_o": rays_o, "rays_d": rays_d, "viewdirs": rays_d}
