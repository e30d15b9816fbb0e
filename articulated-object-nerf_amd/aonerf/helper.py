"""Drop-in for ``models/vanilla_nerf/helper.py`` of the reference, running on the MI355X.

Same function names, argument meaning and return tuples as the reference; the work happens in
the HIP kernels of libaonerf.so (include/aonerf.h).  Extensions over the reference signatures
are keyword-only extras (``u=...``) that inject the uniforms the reference draws with
torch.rand (helper.py:126, :227) so randomized mode is testable.

The only host-side arithmetic is the 1-D sample schedule (S floats): it is built with the very
torch CPU ops the reference uses (helper.py:116-125, :229) because torch's CPU linspace is not a
closed formula (vectorised blocks round differently), then cached on the device.
"""
import numpy as np
import torch

from . import _lib as L


# ----------------------------------------------------------------------------- metrics
def img2mse(x, y):
    """reference helper.py:17-18."""
    return torch.mean((x - y) ** 2)


def mse2psnr(x):
    """reference helper.py:21-22."""
    return -10.0 * torch.log(x) / np.log(10)


def cast_rays(t_vals, origins, directions):
    """reference helper.py:25-26 (elementwise; fused into every kernel that needs xyz)."""
    return origins[..., None, :] + t_vals[..., None] * directions[..., None, :]


# ----------------------------------------------------------------------------- schedules
_sched_cache = {}


def coarse_schedule(num_samples, near, far, lindisp, device):
    """(t, lower, upper) of helper.py:116-125 as device tensors, built with torch CPU ops."""
    key = (int(num_samples), float(near), float(far), bool(lindisp), str(device))
    if key not in _sched_cache:
        t = torch.linspace(0.0, 1.0, num_samples + 1)
        if lindisp:
            t = 1.0 / (1.0 / near * (1.0 - t) + 1.0 / far * t)
        else:
            t = near * (1.0 - t) + far * t
        mids = 0.5 * (t[..., 1:] + t[..., :-1])
        upper = torch.cat([mids, t[..., -1:]], -1)
        lower = torch.cat([t[..., :1], mids], -1)
        _sched_cache[key] = tuple(x.to(device) for x in (t, lower, upper))
    return _sched_cache[key]


def eval_u(num_samples, device, float_min_eps=2 ** -32):
    """u of helper.py:229 (its last entry rounds to exactly 1.0 in fp32)."""
    key = ("u", int(num_samples), float(float_min_eps), str(device))
    if key not in _sched_cache:
        _sched_cache[key] = torch.linspace(0.0, 1.0 - float_min_eps, num_samples).to(device)
    return _sched_cache[key]


# ----------------------------------------------------------------------------- sampling
def sample_along_rays(rays_o, rays_d, num_samples, near, far, randomized, lindisp, *, u=None,
                      want_coords=True):
    """reference helper.py:106-133 -> (t_vals (B, S+1), coords (B, S+1, 3))."""
    L.require_gpu(rays_o, rays_d, u)
    rays_o, rays_d = L.contig(rays_o), L.contig(rays_d)
    B, S = rays_o.shape[0], num_samples + 1
    dev = rays_o.device
    t_sched, lower, upper = coarse_schedule(num_samples, near, far, lindisp, dev)
    if randomized and u is None:
        u = torch.rand((B, S), device=dev)
    u = L.contig(u) if randomized else None
    base = lower if randomized else t_sched  # eval mode: the schedule itself (helper.py:129)
    if u is not None and tuple(u.shape) != (B, S):
        raise ValueError(f"u must be ({B}, {S})")
    t_vals = torch.empty((B, S), device=dev)
    coords = torch.empty((B, S, 3), device=dev) if want_coords else None
    L.call("aon_sample_along_rays", L.ptr(rays_o), L.ptr(rays_d), B, S, L.ptr(base), L.ptr(upper),
           L.ptr(u), L.ptr(t_vals), L.ptr(coords), L.stream(dev))
    return t_vals, coords


def pos_enc(x, min_deg, max_deg):
    """reference helper.py:136-140 -> (..., 3 + 6*(max_deg-min_deg))."""
    L.require_gpu(x)
    if x.shape[-1] != 3:
        raise ValueError("pos_enc expects (..., 3) inputs")
    x = L.contig(x)
    n = x.numel() // 3
    out = torch.empty(list(x.shape[:-1]) + [3 + 6 * (max_deg - min_deg)], device=x.device)
    L.call("aon_pos_enc", L.ptr(x), n, min_deg, max_deg, L.ptr(out), L.stream(x.device))
    return out


# ----------------------------------------------------------------------------- composite
def volumetric_rendering(rgb, density, t_vals, dirs, white_bkgd, nocs=None):
    """reference helper.py:157-195 -> (comp_rgb, acc, weights, depth | comp_nocs)."""
    L.require_gpu(rgb, density, t_vals, dirs)
    B, S = t_vals.shape
    if tuple(rgb.shape) != (B, S, 3) or tuple(density.shape) != (B, S, 1) or dirs.shape[-1] != 3:
        raise ValueError("volumetric_rendering: shape mismatch")
    rgb, density, t_vals, dirs = (L.contig(x) for x in (rgb, density, t_vals, dirs))
    comp = torch.empty((B, 3), device=rgb.device)
    acc = torch.empty((B,), device=rgb.device)
    w = torch.empty((B, S), device=rgb.device)
    depth = torch.empty((B,), device=rgb.device)
    L.call("aon_composite_fwd", L.ptr(rgb), 3, L.ptr(density), 1, L.ptr(t_vals), L.ptr(dirs), B, S,
           int(bool(white_bkgd)), L.ACT_NONE, L.ptr(comp), L.ptr(acc), L.ptr(w), L.ptr(depth),
           L.stream(rgb.device))
    if nocs is not None:
        return comp, acc, w, (w[..., None] * nocs).sum(dim=-2)
    return comp, acc, w, depth


# ----------------------------------------------------------------------------- pdf sampling
def _pdf_call(bins, weights, num_samples, randomized, u, t_merge, origins, directions,
              float_min_eps=2 ** -32):
    L.require_gpu(bins, weights, u, t_merge, origins, directions)
    B, nb = bins.shape
    if tuple(weights.shape) != (B, nb - 1):
        raise ValueError("weights must be (B, nbins - 1)")
    dev = bins.device
    bins = L.contig(bins)
    if weights.stride(-1) != 1:
        weights = weights.contiguous()
    if randomized:
        u = torch.rand((B, num_samples), device=dev) if u is None else L.contig(u)
        if tuple(u.shape) != (B, num_samples):
            raise ValueError(f"u must be ({B}, {num_samples})")
        u_stride = num_samples
    else:
        u, u_stride = eval_u(num_samples, dev, float_min_eps), 0
    Nt = 0
    if t_merge is not None:
        t_merge = L.contig(t_merge)
        Nt = t_merge.shape[-1]
    out = torch.empty((B, Nt + num_samples), device=dev)
    xyz = None
    if origins is not None:
        origins, directions = L.contig(origins), L.contig(directions)
        xyz = torch.empty((B, Nt + num_samples, 3), device=dev)
    L.call("aon_sample_pdf", L.ptr(bins), bins.stride(0), L.ptr(weights), weights.stride(0), B, nb,
           num_samples, L.ptr(u), u_stride, L.ptr(t_merge), Nt, L.ptr(origins), L.ptr(directions),
           L.ptr(out), L.ptr(xyz), L.stream(dev))
    return out, xyz


def sorted_piecewise_constant_pdf(bins, weights, num_samples, randomized, float_min_eps=2 ** -32,
                                  *, u=None):
    """reference helper.py:203-243 -> samples (B, num_samples) (unsorted when randomized)."""
    if randomized:
        # the reference returns the samples in u order; sort indices come from the kernel's
        # sorted output, so recover u-order by evaluating without a merge on sorted u
        L.require_gpu(u)
        B = bins.shape[0]
        if u is None:
            u = torch.rand((B, num_samples), device=bins.device)
        us, order = torch.sort(L.contig(u), dim=-1)
        s, _ = _pdf_call(bins, weights, num_samples, True, us, None, None, None)
        out = torch.empty_like(s)
        out.scatter_(-1, order, s)  # samples are monotone in u: sorted u <-> sorted samples
        return out
    s, _ = _pdf_call(bins, weights, num_samples, False, None, None, None, None, float_min_eps)
    return s


def sample_pdf(bins, weights, origins, directions, t_vals, num_samples, randomized, *, u=None):
    """reference helper.py:246-252 -> (sorted t_vals (B, Nt+Ns), coords (B, Nt+Ns, 3))."""
    return _pdf_call(bins.detach(), weights.detach(), num_samples, randomized, u, t_vals.detach(),
                     origins, directions)
