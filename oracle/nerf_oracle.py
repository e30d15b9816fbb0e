"""CPU restatement (torch fp32, CPU only) of the reference's volumetric-render hot path.

TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py.  Every function cites the reference
file:line it restates (paths relative to DJNing/articulated-object-nerf).  Pinned against
golden vectors generated from the reference itself (tests/golden/make_golden.py,
tests/test_oracle_golden.py).

Numerical notes that the HIP kernels reproduce (measured on torch 2.10 CPU):
  * torch CPU ``cumsum``/``cumprod`` accumulate fp32 inputs in fp64 and round every prefix;
  * ``torch.linspace`` on CPU mixes a symmetric scalar formula with a vectorised arange, so
    the 1-D sample schedules (helper.py:116, :229) are built on the host with torch itself
    and handed to the device as tables;
  * ``x + 0.5*np.pi`` in pos_enc is an fp32 add of 1.5707964f (helper.py:139).
"""
import math

import numpy as np
import torch


# ----------------------------------------------------------------------------- rays
def create_spheric_poses(radius=4.0, n=40, phi=-30.0):
    """reference datasets/sapien_multi.py:29-72 -> (n, 4, 4) float32 c2w."""

    def trans_t(t):
        return torch.tensor([[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 1, t], [0, 0, 0, 1]],
                            dtype=torch.float32)

    def rot_phi(p):
        c, s = np.cos(p), np.sin(p)
        return torch.tensor([[1, 0, 0, 0], [0, c, -s, 0], [0, s, c, 0], [0, 0, 0, 1]],
                            dtype=torch.float32)

    def rot_theta(th):
        c, s = np.cos(th), np.sin(th)
        return torch.tensor([[c, 0, -s, 0], [0, 1, 0, 0], [s, 0, c, 0], [0, 0, 0, 1]],
                            dtype=torch.float32)

    flip = torch.tensor([[-1, 0, 0, 0], [0, 0, 1, 0], [0, 1, 0, 0], [0, 0, 0, 1]],
                        dtype=torch.float32)
    poses = []
    for angle in np.linspace(-180, 180, n + 1)[:-1]:
        c2w = trans_t(radius)
        c2w = rot_phi(phi / 180.0 * np.pi) @ c2w
        c2w = rot_theta(angle / 180.0 * np.pi) @ c2w
        poses.append(flip @ c2w)
    return torch.stack(poses, 0)


def get_ray_directions(H, W, focal):
    """reference datasets/ray_utils.py:71-90 (kornia create_meshgrid, no +0.5 centring)."""
    x = torch.linspace(0, W - 1, W)
    y = torch.linspace(0, H - 1, H)
    i, j = torch.meshgrid(x, y, indexing="xy")  # i: column (H,W), j: row (H,W)
    return torch.stack([(i - W / 2) / focal, -(j - H / 2) / focal, -torch.ones_like(i)], -1)


def get_rays(directions, c2w, output_view_dirs=False, output_radii=False):
    """reference datasets/ray_utils.py:118-159.

    With ``output_view_dirs`` the reference normalises ``viewdirs`` in place and it aliases
    ``rays_d`` (ray_utils.py:145-147), so both returned direction tensors are unit vectors.
    """
    rays_d = directions @ c2w[:, :3].T
    rays_o = c2w[:, 3].expand(rays_d.shape)
    radius = None
    if output_radii:
        rd = directions @ c2w[:, :3].T
        dx = torch.sqrt(torch.sum((rd[:-1, :, :] - rd[1:, :, :]) ** 2, dim=-1))
        dx = torch.cat([dx, dx[-2:-1, :]], dim=0)
        radius = (dx[..., None] * 2 / torch.sqrt(torch.tensor(12, dtype=torch.int8))).reshape(-1)
    rays_d = rays_d / torch.norm(rays_d, dim=-1, keepdim=True)
    rays_o = rays_o.reshape(-1, 3)
    rays_d = rays_d.reshape(-1, 3)
    if output_view_dirs:
        if output_radii:
            return rays_o, rays_d, rays_d.clone(), radius
        return rays_o, rays_d, rays_d.clone()
    return rays_o, rays_d


def get_rays_fma(directions, c2w):
    """get_rays(..., output_view_dirs=True) with the (n,3)@(3,3) product and the row norm as
    forward fma chains -- what torch CPU computes for reference ray_utils.py:118-147 in the build
    container (MKL on Intel AVX-512; measured equal element for element on the 640x480 frame and
    on the golden frames), emulated exactly enough in fp64 (a*b is exact in fp64; one rounding of
    the sum before the fp32 one).  The reference's ray generation is machine-dependent at one ulp:
    torch on the GPU box's AMD CPU rounds ~3% of these elements differently (tools/diag/
    parity_scale.py), so the attribution uses this as one more valid implementation of a2."""
    M = c2w[:3, :3].double()
    d = directions.reshape(-1, 3).double()

    def r32(x):
        return x.float().double()

    cols = []
    for k in range(3):
        acc = r32(d[:, 0] * M[k, 0])
        acc = r32(d[:, 1] * M[k, 1] + acc)
        cols.append(r32(d[:, 2] * M[k, 2] + acc))
    r = torch.stack(cols, -1)
    s = r32(r[:, 0] * r[:, 0])
    s = r32(r[:, 1] * r[:, 1] + s)
    s = r32(r[:, 2] * r[:, 2] + s)
    n = r32(torch.sqrt(s))
    rays_d = (r / n[:, None]).float()
    rays_o = c2w[:3, 3].float().expand(rays_d.shape).contiguous()
    return rays_o, rays_d, rays_d.clone()


def focal_from_fovy(H, fovy_deg=35.0):
    """SAPIEN camera (datagen/data_gen.py:60-67): fy = 0.5*H/tan(0.5*fovy)."""
    return 0.5 * H / math.tan(0.5 * math.radians(fovy_deg))


# ----------------------------------------------------------------------------- sampling
def coarse_schedule(num_samples, near, far, lindisp=False):
    """The 1-D schedule of reference helper.py:116-125 -> (t, lower, upper), each (S+1,)."""
    t = torch.linspace(0.0, 1.0, num_samples + 1)
    if lindisp:
        t = 1.0 / (1.0 / near * (1.0 - t) + 1.0 / far * t)
    else:
        t = near * (1.0 - t) + far * t
    mids = 0.5 * (t[..., 1:] + t[..., :-1])
    upper = torch.cat([mids, t[..., -1:]], -1)
    lower = torch.cat([t[..., :1], mids], -1)
    return t, lower, upper


def cast_rays(t_vals, origins, directions):
    """reference helper.py:25-26."""
    return origins[..., None, :] + t_vals[..., None] * directions[..., None, :]


def sample_along_rays(rays_o, rays_d, num_samples, near, far, randomized, lindisp, u=None):
    """reference helper.py:106-133; ``u`` (B, S+1) replaces torch.rand at helper.py:126."""
    B = rays_o.shape[0]
    t, lower, upper = coarse_schedule(num_samples, near, far, lindisp)
    if randomized:
        if u is None:
            u = torch.rand((B, num_samples + 1))
        t_vals = lower + (upper - lower) * u
    else:
        t_vals = torch.broadcast_to(t, (B, num_samples + 1))
    return t_vals, cast_rays(t_vals, rays_o, rays_d)


def pos_enc(x, min_deg, max_deg):
    """reference helper.py:136-140: [x, sin(x*2^d) (d-major, xyz-minor), sin(x*2^d + pi/2)]."""
    scales = torch.tensor([2 ** i for i in range(min_deg, max_deg)]).type_as(x)
    xb = torch.reshape(x[..., None, :] * scales[:, None], list(x.shape[:-1]) + [-1])
    return torch.cat([x, torch.sin(torch.cat([xb, xb + 0.5 * np.pi], dim=-1))], dim=-1)


def fine_u(num_samples, batch_shape, randomized, u=None):
    """The u of reference helper.py:226-230 (eval: linspace(0, 1-2^-32) whose last entry is 1.0)."""
    if randomized:
        return torch.rand(list(batch_shape) + [num_samples]) if u is None else u
    u = torch.linspace(0.0, 1.0 - 2 ** -32, num_samples)
    return torch.broadcast_to(u, list(batch_shape) + [num_samples])


def _pdf_bins(weights, num_samples, randomized, u=None):
    """helper.py:207-229: eps padding, pdf, the 64-entry CDF [0, fmin(1, cumsum), 1], the u
    schedule, and for every u the bin index searchsorted(cdf, u, right=True)."""
    eps = 1e-5
    weight_sum = weights.sum(dim=-1, keepdim=True)
    padding = torch.fmax(torch.zeros_like(weight_sum), eps - weight_sum)
    weights = weights + padding / weights.shape[-1]
    weight_sum = weight_sum + padding
    pdf = weights / weight_sum
    cdf = torch.fmin(torch.ones_like(pdf[..., :-1]), torch.cumsum(pdf[..., :-1], dim=-1))
    zeros = torch.zeros(list(cdf.shape[:-1]) + [1])
    ones = torch.ones(list(cdf.shape[:-1]) + [1])
    cdf = torch.cat([zeros, cdf, ones], dim=-1)
    u = fine_u(num_samples, cdf.shape[:-1], randomized, u).contiguous()
    idx = torch.searchsorted(cdf.contiguous(), u, right=True)
    return cdf, u, idx


def pdf_bin_index(weights, num_samples, randomized, u=None):
    """The CDF bin every fine-sample u of helper.py:203-243 falls in, (..., num_samples) int64:
    two weight vectors whose bin indices differ place some fine sample in a different bin
    (test attribution of inverse-CDF flips)."""
    return _pdf_bins(weights, num_samples, randomized, u)[2]


def sorted_piecewise_constant_pdf(bins, weights, num_samples, randomized, u=None):
    """reference helper.py:203-243, restated with a per-ray searchsorted.

    The reference's mask form (mask = u >= cdf; bin0 = max over masked bins, bin1 = min over
    unmasked, first/last fallbacks) equals ``idx = searchsorted(cdf, u, right=True)``,
    ``i0 = clamp(idx-1, 0, n-1)``, ``i1 = clamp(idx, max=n-1)`` -- pinned bit-exactly by the
    golden vectors (including zero-weight plateaus and u == cdf ties).
    """
    cdf, u, idx = _pdf_bins(weights, num_samples, randomized, u)
    n = cdf.shape[-1]
    i0 = torch.clamp(idx - 1, 0, n - 1)
    i1 = torch.clamp(idx, max=n - 1)
    bin0, bin1 = torch.gather(bins, -1, i0), torch.gather(bins, -1, i1)
    cdf0, cdf1 = torch.gather(cdf, -1, i0), torch.gather(cdf, -1, i1)
    t = torch.clip(torch.nan_to_num((u - cdf0) / (cdf1 - cdf0), 0), 0, 1)
    return bin0 + t * (bin1 - bin0)


def sample_pdf(bins, weights, origins, directions, t_vals, num_samples, randomized, u=None):
    """reference helper.py:246-252 (sorted merge of coarse t and the pdf samples)."""
    t_samples = sorted_piecewise_constant_pdf(bins, weights, num_samples, randomized, u).detach()
    t_vals = torch.sort(torch.cat([t_vals, t_samples], dim=-1), dim=-1).values
    return t_vals, cast_rays(t_vals, origins, directions)


# ----------------------------------------------------------------------------- MLP
def mlp_forward(p, x, condition, netdepth=8, skip_layer=4, netdepth_condition=1):
    """reference models/vanilla_nerf/model.py:95-120 with ``p`` = {layer.weight/bias: tensor}.

    x: (B, S, C) encoded points; condition: (B, Cv) encoded view directions.
    Returns raw_rgb (B, S, 3), raw_density (B, S, 1).
    """
    S, C = x.shape[1:]
    x = x.reshape(-1, C)
    inputs = x
    for idx in range(netdepth):
        x = torch.relu(x @ p[f"pts_linears.{idx}.weight"].T + p[f"pts_linears.{idx}.bias"])
        if idx % skip_layer == 0 and idx > 0:
            x = torch.cat([x, inputs], dim=-1)
    raw_density = (x @ p["density_layer.weight"].T + p["density_layer.bias"]).reshape(-1, S, 1)
    bottleneck = x @ p["bottleneck_layer.weight"].T + p["bottleneck_layer.bias"]
    cond = torch.tile(condition[:, None, :], (1, S, 1)).reshape(-1, condition.shape[-1])
    x = torch.cat([bottleneck, cond], dim=-1)
    for idx in range(netdepth_condition):
        x = torch.relu(x @ p[f"views_linear.{idx}.weight"].T + p[f"views_linear.{idx}.bias"])
    raw_rgb = (x @ p["rgb_layer.weight"].T + p["rgb_layer.bias"]).reshape(-1, S, 3)
    return raw_rgb, raw_density


# ----------------------------------------------------------------------------- composite
def volumetric_rendering(rgb, density, t_vals, dirs, white_bkgd):
    """reference helper.py:157-195 -> (comp_rgb, acc, weights, depth)."""
    eps = 1e-10
    dists = torch.cat([t_vals[..., 1:] - t_vals[..., :-1],
                       torch.ones(t_vals[..., :1].shape) * 1e10], dim=-1)
    dists = dists * torch.norm(dirs[..., None, :], dim=-1)
    alpha = 1.0 - torch.exp(-density[..., 0] * dists)
    trans = torch.cat([torch.ones_like(alpha[..., :1]),
                       torch.cumprod(1.0 - alpha[..., :-1] + eps, dim=-1)], dim=-1)
    weights = alpha * trans
    comp_rgb = (weights[..., None] * rgb).sum(dim=-2)
    depth = (weights * t_vals).sum(dim=-1)
    depth = torch.nan_to_num(depth, float("inf"))
    depth = torch.clamp(depth, torch.min(depth), torch.max(depth))
    acc = weights.sum(dim=-1)
    if white_bkgd:
        comp_rgb = comp_rgb + (1.0 - acc[..., None])
    return comp_rgb, acc, weights, depth


# ----------------------------------------------------------------------------- NeRF
def split_state_dict(sd):
    """{coarse_mlp.x: t, fine_mlp.x: t} -> (coarse params, fine params) as torch tensors."""
    out = ({}, {})
    for k, v in sd.items():
        level, name = k.split(".", 1)
        out[0 if level == "coarse_mlp" else 1][name] = torch.as_tensor(v)
    return out


def nerf_forward(params, rays, randomized, white_bkgd, near, far, num_coarse_samples=64,
                 num_fine_samples=128, min_deg_point=0, max_deg_point=10, deg_view=4,
                 lindisp=False, u_coarse=None, u_fine=None, return_intermediates=False):
    """reference models/vanilla_nerf/model.py:147-199 (two-level coarse/fine loop).

    params: (coarse, fine) dicts as from :func:`split_state_dict`.
    Returns [(rgb, acc, depth)_coarse, (rgb, acc, depth)_fine] (+ per-level intermediates).
    """
    ret, inter = [], []
    weights = t_vals = None
    for level in range(2):
        if level == 0:
            t_vals, samples = sample_along_rays(rays["rays_o"], rays["rays_d"], num_coarse_samples,
                                                near, far, randomized, lindisp, u_coarse)
        else:
            t_mids = 0.5 * (t_vals[..., 1:] + t_vals[..., :-1])
            t_vals, samples = sample_pdf(t_mids, weights[..., 1:-1], rays["rays_o"],
                                         rays["rays_d"], t_vals, num_fine_samples, randomized,
                                         u_fine)
        enc = pos_enc(samples, min_deg_point, max_deg_point)
        venc = pos_enc(rays["viewdirs"], 0, deg_view)
        raw_rgb, raw_sigma = mlp_forward(params[level], enc, venc)
        rgb = torch.sigmoid(raw_rgb)
        sigma = torch.relu(raw_sigma)
        comp_rgb, acc, weights, depth = volumetric_rendering(rgb, sigma, t_vals, rays["rays_d"],
                                                             white_bkgd)
        ret.append((comp_rgb, acc, depth))
        inter.append(dict(t_vals=t_vals, raw_rgb=raw_rgb, raw_sigma=raw_sigma, weights=weights))
    return (ret, inter) if return_intermediates else ret


def render_level(params, rays, t_vals, level, white_bkgd, min_deg_point=0, max_deg_point=10,
                 deg_view=4):
    """One level of model.py:175-197 on GIVEN sample positions t_vals (teacher forcing):
    cast_rays -> pos_enc -> MLP -> sigmoid/relu -> volumetric_rendering."""
    samples = cast_rays(t_vals, rays["rays_o"], rays["rays_d"])
    raw_rgb, raw_sigma = mlp_forward(params[level], pos_enc(samples, min_deg_point, max_deg_point),
                                     pos_enc(rays["viewdirs"], 0, deg_view))
    return volumetric_rendering(torch.sigmoid(raw_rgb), torch.relu(raw_sigma), t_vals,
                                rays["rays_d"], white_bkgd)


def render_rays(params, batch, chunk, white_bkgd, near, far, **kw):
    """reference models/vanilla_nerf/model.py:295-321 (chunk loop, fine outputs concatenated)."""
    B = batch["rays_o"].shape[0]
    out = {"comp_rgb": [], "acc": [], "depth": []}
    for i in range(0, B, chunk):
        sub = {k: v[i:i + chunk] for k, v in batch.items()}
        fine = nerf_forward(params, sub, False, white_bkgd, near, far, **kw)[1]
        out["comp_rgb"].append(fine[0])
        out["acc"].append(fine[1])
        out["depth"].append(fine[2])
    return {k: torch.cat(v, 0) for k, v in out.items()}


# ----------------------------------------------------------------------------- articulated
def _lin(p, name, x):
    """nn.Linear's own call (F.linear: one addmm on 2-D input)."""
    return torch.nn.functional.linear(x, p[f"{name}.weight"], p[f"{name}.bias"])


def _pos_enc_args_fp32(x, min_deg, max_deg):
    """The fp32 arguments of pos_enc's sin (helper.py:136-140) at fp32 points x (R, 3):
    x 2^d (exact) and x 2^d + 0.5 pi (one fp32 add of 1.5707964f, as the reference's fp32
    tensor arithmetic rounds it) -> (R, 6 (max_deg - min_deg)) fp32."""
    x = x.float()
    scales = torch.tensor([2 ** i for i in range(min_deg, max_deg)], dtype=torch.float32)
    xb = torch.reshape(x[..., None, :] * scales[:, None], list(x.shape[:-1]) + [-1])
    return torch.cat([xb, xb + 0.5 * np.pi], dim=-1)


def pos_enc_at(x_value, x_graph, min_deg, max_deg):
    """pos_enc (helper.py:136-140) whose VALUE is evaluated at the fp32 points x_value (the
    sin arguments rounded exactly as the reference's fp32 arithmetic rounds them, the sin itself
    in x_graph's dtype) and whose GRADIENT flows into x_graph: d/dx sin(a) = cos(a) 2^d at those
    same arguments.  x_graph's value is not used (straight-through: teacher forcing at a given
    x' while autograd still reaches the parameters that produced x_graph)."""
    dt = x_graph.dtype
    args = _pos_enc_args_fp32(x_value, min_deg, max_deg).to(dt)
    delta = x_graph - x_graph.detach()  # zero, carries the gradient
    scales = torch.tensor([2 ** i for i in range(min_deg, max_deg)], dtype=dt)
    db = torch.reshape(delta[..., None, :] * scales[:, None], list(delta.shape[:-1]) + [-1])
    return torch.cat([x_value.to(dt) + delta, torch.sin(args + torch.cat([db, db], dim=-1))], dim=-1)


def art_mlp_forward(p, pos, condition, latents, netdepth=8, skip_layer=4, netdepth_deformation=4,
                    netdepth_condition=4, min_deg_point=0, max_deg_point=10, xp_fixed=None,
                    return_xp=False, record=None):
    """reference models/vanilla_nerf/model_autodecoder.py:168-239 (deformation_mlp=True,
    enc_after=True, embed_deg=False).

    pos: (B, S, 3) sample positions; condition: (B, 27) encoded view directions;
    latents: {density (1,128), color (1,128), articulation (1,32)} repeated over all rows
    (model_autodecoder.py:186-194).  Returns raw_rgb (B, S, 3), raw_density (B, S, 1).

    Test hooks (not the reference's arithmetic): ``xp_fixed`` (B*S, 3) fp32 teacher-forces the
    deformed points x' (pos_enc evaluated at those fp32 points, gradients straight through to
    the deformation MLP, :func:`pos_enc_at`); ``return_xp`` also returns this call's x';
    ``record`` (a dict) receives the intermediates in :func:`art_mlp_forward_kept`'s layout.
    """
    rec = record if record is not None else {}
    S = pos.shape[1]
    pos = pos.reshape(-1, 3)
    BN = pos.shape[0]
    shape = latents["density"].repeat(BN, 1)
    app = latents["color"].repeat(BN, 1)
    art = latents["articulation"].repeat(BN, 1)
    rec.update(xyz=pos, hd=[], h=[], hv=[])
    x = torch.cat([pos, shape, art], -1)
    for idx in range(netdepth_deformation):  # model_autodecoder.py:200-203
        x = torch.relu(_lin(p, f"deformations_linear.{idx}", x))
        rec["hd"].append(x)
    x = _lin(p, "deformation_layer", x) + pos  # :205
    xp = rec["xp"] = x
    if xp_fixed is None:
        x = pos_enc(x, min_deg_point, max_deg_point)  # :207-212 (enc_after)
    else:
        x = pos_enc_at(xp_fixed, x, min_deg_point, max_deg_point)
    rec["enc"] = x
    x = torch.cat([x, shape], -1)
    inputs = x
    for idx in range(netdepth):  # :216-220
        x = torch.relu(_lin(p, f"pts_linears.{idx}", x))
        rec["h"].append(x)
        if idx % skip_layer == 0 and idx > 0:
            x = torch.cat([x, inputs], dim=-1)
    raw_density = _lin(p, "density_layer", x).reshape(-1, S, 1)
    bottleneck = rec["bot"] = _lin(p, "bottleneck_layer", x)
    cond = torch.tile(condition[:, None, :], (1, S, 1)).reshape(-1, condition.shape[-1])
    x = torch.cat([bottleneck, cond, app], dim=-1)  # :229-231
    for idx in range(netdepth_condition):
        x = torch.relu(_lin(p, f"views_linear.{idx}", x))
        rec["hv"].append(x)
    raw_rgb = _lin(p, "rgb_layer", x).reshape(-1, S, 3)
    if return_xp:
        return raw_rgb, raw_density, xp
    return raw_rgb, raw_density


def art_mlp_forward_kept(p, kept, condition, latents, S, min_deg_point=0, max_deg_point=10):
    """Stage isolation of the articulated MLP's BACKWARD (model_autodecoder.py:168-239): the
    forward of :func:`art_mlp_forward` whose every intermediate VALUE is the one a GPU forward
    kept -- ``kept`` = {xyz (R,3), hd (4,R,wd), xp (R,3) = x', enc (R,63) = pos_enc(x'),
    h (8,R,256), bot (R,256), hv (4,R,wc)}, ReLU' taken from the sign of the kept activation --
    while autograd runs through this function's own linear maps in the parameters' dtype.  Its
    backward from a given d raw is therefore the exact (e.g. fp64) backward at the GPU's own
    forward values: nothing the forward computed differently (x', hence sin(2^9 x')) can be
    amplified.  pos_enc's derivative is cos at the fp32 arguments of x' (:func:`pos_enc_at`).
    condition: (B, 27) encoded view directions.  Returns raw_rgb (R, 3), raw_density (R, 1)."""
    dt = p["rgb_layer.weight"].dtype
    K = {k: (v.to(dt) if torch.is_tensor(v) else [x.to(dt) for x in v]) for k, v in kept.items()}
    R = K["xyz"].shape[0]

    def forced(value, z):
        return value + (z - z.detach())

    def relu_kept(value, z):
        return forced(value, z * (value > 0).to(dt))

    shape = latents["density"].repeat(R, 1)
    app = latents["color"].repeat(R, 1)
    art = latents["articulation"].repeat(R, 1)
    x = torch.cat([K["xyz"], shape, art], -1)
    for idx in range(len(K["hd"])):
        x = relu_kept(K["hd"][idx], _lin(p, f"deformations_linear.{idx}", x))
    xp = forced(K["xp"], _lin(p, "deformation_layer", x) + K["xyz"])
    enc = forced(K["enc"], pos_enc_at(kept["xp"], xp, min_deg_point, max_deg_point))
    x = torch.cat([enc, shape], -1)
    inputs = x
    for idx in range(len(K["h"])):
        x = relu_kept(K["h"][idx], _lin(p, f"pts_linears.{idx}", x))
        if idx % 4 == 0 and idx > 0:
            x = torch.cat([x, inputs], dim=-1)
    raw_density = _lin(p, "density_layer", x)
    bot = forced(K["bot"], _lin(p, "bottleneck_layer", x))
    cond = torch.tile(condition.to(dt)[:, None, :], (1, S, 1)).reshape(-1, condition.shape[-1])
    x = torch.cat([bot, cond, app], dim=-1)
    for idx in range(len(K["hv"])):
        x = relu_kept(K["hv"][idx], _lin(p, f"views_linear.{idx}", x))
    raw_rgb = _lin(p, "rgb_layer", x)
    return raw_rgb, raw_density


def art_activations(raw_rgb, raw_sigma, rgb_padding=0.001, density_bias=-1.0):
    """NeRF_AE_Art.forward (model_autodecoder.py:321-323): padded sigmoid, softplus(raw - 1)."""
    rgb = torch.sigmoid(raw_rgb) * (1 + 2 * rgb_padding) - rgb_padding
    sigma = torch.nn.functional.softplus(raw_sigma + density_bias)
    return rgb, sigma


def art_nerf_forward(params, rays, randomized, white_bkgd, near, far, latents,
                     num_coarse_samples=64, num_fine_samples=128, deg_view=4, lindisp=False,
                     u_coarse=None, u_fine=None, return_intermediates=False):
    """reference NeRF_AE_Art.forward (model_autodecoder.py:278-337), enc_after=True."""
    ret, inter = [], []
    weights = t_vals = None
    for level in range(2):
        if level == 0:
            t_vals, samples = sample_along_rays(rays["rays_o"], rays["rays_d"], num_coarse_samples,
                                                near, far, randomized, lindisp, u_coarse)
        else:
            t_mids = 0.5 * (t_vals[..., 1:] + t_vals[..., :-1])
            t_vals, samples = sample_pdf(t_mids, weights[..., 1:-1], rays["rays_o"],
                                         rays["rays_d"], t_vals, num_fine_samples, randomized,
                                         u_fine)
        venc = pos_enc(rays["viewdirs"], 0, deg_view)
        raw_rgb, raw_sigma = art_mlp_forward(params[level], samples, venc, latents)
        rgb, sigma = art_activations(raw_rgb, raw_sigma)
        comp_rgb, acc, weights, depth = volumetric_rendering(rgb, sigma, t_vals, rays["rays_d"],
                                                             white_bkgd)
        ret.append((comp_rgb, acc, depth))
        inter.append(dict(t_vals=t_vals, raw_rgb=raw_rgb, raw_sigma=raw_sigma, weights=weights))
    return (ret, inter) if return_intermediates else ret


def art_render_level(params, rays, t_vals, level, white_bkgd, latents, deg_view=4, xp_fixed=None,
                     return_xp=False):
    """One NeRF_AE_Art level on GIVEN sample positions (teacher forcing); ``xp_fixed`` /
    ``return_xp`` as in :func:`art_mlp_forward` (x' appended to the returned tuple)."""
    samples = cast_rays(t_vals, rays["rays_o"], rays["rays_d"])
    out = art_mlp_forward(params[level], samples, pos_enc(rays["viewdirs"], 0, deg_view), latents,
                          xp_fixed=xp_fixed, return_xp=return_xp)
    rgb, sigma = art_activations(out[0], out[1])
    res = volumetric_rendering(rgb, sigma, t_vals, rays["rays_d"], white_bkgd)
    return res + (out[2],) if return_xp else res


def code_library_latents(tables, instance_id, articulation_id):
    """CodeLibraryArticulated.forward, training branch (reference models/code_library.py:36-53):
    rows of the three embedding tables -> {density, color (1, 128), articulation (1, 32)}."""
    iid = torch.as_tensor([instance_id])
    aid = torch.as_tensor([articulation_id])
    return {"density": torch.nn.functional.embedding(iid, tables["embedding_instance_shape.weight"]),
            "color": torch.nn.functional.embedding(iid, tables["embedding_instance_appearance.weight"]),
            "articulation": torch.nn.functional.embedding(
                aid, tables["embedding_instance_articulation.weight"])}


def latent_reg_loss(latents):
    """The latent-code regulariser of LitNeRF_AutoDecoder.training_step (reference
    models/vanilla_nerf/model_autodecoder.py:456-466): 1e-4 * sum of mean column norms."""
    return 1e-4 * (torch.mean(torch.norm(latents["density"], dim=0))
                   + torch.mean(torch.norm(latents["color"], dim=0))
                   + torch.mean(torch.norm(latents["articulation"], dim=0)))


def art_training_loss(params, tables, rays, target, instance_id, articulation_id, randomized,
                      white_bkgd, near, far, u_coarse=None, u_fine=None):
    """LitNeRF_AutoDecoder.training_step (model_autodecoder.py:395-477): loss = mse(fine) +
    mse(coarse) + the latent regulariser; returns (loss, loss0, loss1, reg)."""
    latents = code_library_latents(tables, instance_id, articulation_id)
    ret = art_nerf_forward(params, rays, randomized, white_bkgd, near, far, latents,
                           u_coarse=u_coarse, u_fine=u_fine)
    loss0 = img2mse(ret[0][0], target)
    loss1 = img2mse(ret[1][0], target)
    reg = latent_reg_loss(latents)
    loss = loss1 + loss0
    loss = loss + reg
    return loss, loss0, loss1, reg


# ----------------------------------------------------------------------------- metrics
def img2mse(x, y):
    """reference helper.py:17-18."""
    return torch.mean((x - y) ** 2)


def mse2psnr(x):
    """reference helper.py:21-22."""
    return -10.0 * torch.log(x) / np.log(10)


def psnr_each(preds, gts):
    """reference models/interface.py:54-62 (clip both to [0,1])."""
    return torch.stack([mse2psnr(torch.mean((torch.clip(p, 0, 1) - torch.clip(g, 0, 1)) ** 2))
                        for p, g in zip(preds, gts)])


def psnr_legacy(pred, gt):
    """reference models/interface.py:72-74 (no clipping)."""
    return -10 * torch.log10(torch.mean((pred - gt) ** 2))
