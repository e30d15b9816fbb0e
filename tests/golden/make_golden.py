"""Generate the golden vectors for the hot path by running the REFERENCE itself.

Runs only in the build container (needs /root/reference); its outputs (tests/golden/*.npz) are
the committed fixtures that travel to the GPU box.  Inputs are synthetic (no datasets offline):
SAPIEN-style spherical poses (datasets/sapien_multi.py:29-72), fovy-35 focal
(datagen/data_gen.py:64), near=2/far=6 (datasets/sapien.py:72-73), and NeRF weights regenerated
from numpy PCG64 by oracle/weights.py (their sha256 is stored with every fixture).

    python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)

import _refimport  # noqa: E402
from oracle import weights as W  # noqa: E402
from oracle.attribution import TRANSCENDENTAL_VARIANTS  # noqa: E402

helper, model, ray_utils, sapien_multi = _refimport.load()
torch.set_num_threads(8)


class RandQueue:
    """Replace torch.rand with recorded uniforms (reference helper.py:126, :227)."""

    def __init__(self, seed):
        self.rng = np.random.Generator(np.random.PCG64(seed))
        self.drawn = []
        self._orig = torch.rand

    def __call__(self, *size, **kw):
        if len(size) == 1 and isinstance(size[0], (list, tuple, torch.Size)):
            size = tuple(size[0])
        u = torch.from_numpy(self.rng.random(size, dtype=np.float32))
        self.drawn.append(u.numpy().copy())
        return u

    def __enter__(self):
        torch.rand = self
        return self

    def __exit__(self, *a):
        torch.rand = self._orig


# Re-associations of the reference's fp32 GEMMs (nn.Linear) used to measure the reference's own
# sensitivity envelope: the fine level re-samples along the coarse CDF, so an ulp-level change
# of the MLP outputs moves some fine samples by delta-cdf / pdf.  The GPU end-to-end gate lets a
# ray exceed 1e-4 only where the reference itself moves that much (tests/test_gpu_parity.py).
_LINEAR_VARIANTS = {
    "fp64": lambda m, x: (x.double() @ m.weight.double().T + m.bias.double()).float(),
    "ksplit": lambda m, x: (x[..., : m.weight.shape[1] // 2] @ m.weight[:, : m.weight.shape[1] // 2].T
                            + x[..., m.weight.shape[1] // 2:] @ m.weight[:, m.weight.shape[1] // 2:].T)
                           + m.bias,
}


def envelope(run):
    """max over equally valid fp32 implementations of the reference of |run() - run()| per output
    key: its GEMMs re-associated or in fp64, and (round 5) its torch.sin (pos_enc, helper.py:139)
    and torch.exp (alpha, helper.py:168) correctly rounded or moved by a seeded +-1 ulp
    (oracle/attribution.py TRANSCENDENTAL_VARIANTS)."""
    base = run()
    env = {k: np.zeros_like(v) for k, v in base.items()}
    orig = torch.nn.Linear.forward
    try:
        for fn in _LINEAR_VARIANTS.values():
            torch.nn.Linear.forward = fn
            out = run()
            for k in env:
                env[k] = np.maximum(env[k], np.abs(out[k] - base[k]))
    finally:
        torch.nn.Linear.forward = orig
    for ctx in TRANSCENDENTAL_VARIANTS.values():
        with ctx():
            out = run()
        for k in env:
            env[k] = np.maximum(env[k], np.abs(out[k] - base[k]))
    keep = ("rgb", "acc", "depth", "weights")
    return {f"env_{k}": v for k, v in env.items() if k.endswith(keep) and "raw" not in k}


def make_nerf(seed=0, **kw):
    net = model.NeRF(**kw)
    sd = W.nerf_state_dict(seed)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    net.eval()
    return net, W.digest(sd)


def frame_rays(H, W_, pose_idx=5, radius=4.0):
    focal = 0.5 * H / np.tan(0.5 * np.deg2rad(35.0))
    c2w = sapien_multi.create_spheric_poses(radius)[pose_idx][:3, :4]
    dirs = ray_utils.get_ray_directions(H, W_, focal)
    rays_o, viewdirs, rays_d = ray_utils.get_rays(dirs, c2w, output_view_dirs=True)
    return dict(rays_o=rays_o.contiguous(), rays_d=rays_d.contiguous(),
                viewdirs=viewdirs.contiguous()), c2w, focal, dirs


def capture_forward(net, rays, randomized, white_bkgd, near=2.0, far=6.0, extra=()):
    """Run reference NeRF.forward and record per-level intermediates via module hooks
    (``extra``: further positional arguments, e.g. NeRF_AE_Art's latents)."""
    rec = {"t": [], "raw_rgb": [], "raw_sigma": [], "weights": [], "bins": [], "wpdf": []}
    orig_vr, orig_pdf = helper.volumetric_rendering, helper.sample_pdf

    def vr(rgb, density, t_vals, dirs, white_bkgd, nocs=None):
        out = orig_vr(rgb, density, t_vals, dirs, white_bkgd, nocs)
        rec["t"].append(t_vals.detach().clone())
        rec["weights"].append(out[2].detach().clone())
        return out

    def pdf(bins, weights, *a, **k):
        rec["bins"].append(bins.detach().clone())
        rec["wpdf"].append(weights.detach().clone())
        return orig_pdf(bins, weights, *a, **k)

    def hook(mod, inp, out):
        rec["raw_rgb"].append(out[0].detach().clone())
        rec["raw_sigma"].append(out[1].detach().clone())  # returns None: output untouched

    hooks = [mlp.register_forward_hook(hook) for mlp in (net.coarse_mlp, net.fine_mlp)]
    helper.volumetric_rendering, helper.sample_pdf = vr, pdf
    try:
        with torch.no_grad():
            ret = net(rays, randomized, white_bkgd, near, far, *extra)
    finally:
        helper.volumetric_rendering, helper.sample_pdf = orig_vr, orig_pdf
        for h in hooks:
            h.remove()
    return ret, rec


def level_arrays(ret, rec):
    out = {}
    for lv, name in enumerate(("coarse", "fine")):
        out[f"{name}_rgb"] = ret[lv][0].numpy()
        out[f"{name}_acc"] = ret[lv][1].numpy()
        out[f"{name}_depth"] = ret[lv][2].numpy()
        out[f"{name}_t"] = rec["t"][lv].numpy()
        out[f"{name}_raw_rgb"] = rec["raw_rgb"][lv].numpy()
        out[f"{name}_raw_sigma"] = rec["raw_sigma"][lv].numpy()
        out[f"{name}_weights"] = rec["weights"][lv].numpy()
    return out


def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    print(f"{name}: {os.path.getsize(path) / 1e3:.1f} kB  keys={sorted(arrays)}")


def case_rays():
    """get_ray_directions / get_rays (ray_utils.py:71-159) on a 48x64 frame + radii."""
    out = {}
    for k, (H, W_, pose) in enumerate(((48, 64, 5), (30, 40, 17))):
        rays, c2w, focal, dirs = frame_rays(H, W_, pose)
        _, _, _, radii = ray_utils.get_rays(dirs, c2w, output_view_dirs=True, output_radii=True)
        o2, d2 = ray_utils.get_rays(dirs, c2w)
        out.update({f"c2w{k}": c2w.numpy(), f"hwf{k}": np.array([H, W_, focal]),
                    f"dirs{k}": dirs.numpy(), f"rays_o{k}": rays["rays_o"].numpy(),
                    f"rays_d{k}": rays["rays_d"].numpy(), f"viewdirs{k}": rays["viewdirs"].numpy(),
                    f"radii{k}": radii.numpy(), f"plain_o{k}": o2.numpy(), f"plain_d{k}": d2.numpy()})
    out["poses"] = sapien_multi.create_spheric_poses(4.0).numpy()
    save("rays.npz", **out)


def case_forward_eval():
    """NeRF.forward, randomized=False, white background, 64c+128f (config C2 semantics)."""
    net, dig = make_nerf(0)
    rays, c2w, focal, _ = frame_rays(24, 32, 5)
    sel = torch.arange(0, 24 * 32, 3)  # 256 rays spread over the frame
    rays = {k: v[sel].contiguous() for k, v in rays.items()}
    ret, rec = capture_forward(net, rays, False, True)
    env = envelope(lambda: level_arrays(*capture_forward(net, rays, False, True)))
    save("forward_eval.npz", digest=np.array(dig), **{k: v.numpy() for k, v in rays.items()},
         bins=rec["bins"][0].numpy(), wpdf=rec["wpdf"][0].numpy(), **level_arrays(ret, rec), **env)


def case_forward_random():
    """NeRF.forward, randomized=True with recorded uniforms, black background."""
    net, dig = make_nerf(0)
    rays, _, _, _ = frame_rays(16, 16, 11)
    rays = {k: v[:128].contiguous() for k, v in rays.items()}
    with RandQueue(1) as rq:
        ret, rec = capture_forward(net, rays, True, False)
    assert len(rq.drawn) == 2, len(rq.drawn)

    def rerun():
        with RandQueue(1):
            return level_arrays(*capture_forward(net, rays, True, False))

    save("forward_random.npz", digest=np.array(dig), **{k: v.numpy() for k, v in rays.items()},
         u_coarse=rq.drawn[0], u_fine=rq.drawn[1], **level_arrays(ret, rec), **envelope(rerun))


def case_render_frame():
    """LitNeRF.render_rays chunk loop (model.py:295-321): 20x24 frame, chunk 100 (ragged tail)
    and config C1 (64x64, num_coarse_samples=32) fine outputs."""
    out = {}
    for tag, (H, W_, nc, chunk) in (("a", (20, 24, 64, 100)), ("c1", (64, 64, 32, 3840))):
        net, dig = make_nerf(0, num_coarse_samples=nc)
        rays, c2w, focal, _ = frame_rays(H, W_, 7)

        def run():
            res = {"comp_rgb": [], "acc": [], "depth": []}
            with torch.no_grad():
                for i in range(0, H * W_, chunk):
                    sub = {k: v[i:i + chunk] for k, v in rays.items()}
                    fine = net(sub, False, True, 2.0, 6.0)[1]
                    for j, k in enumerate(("comp_rgb", "acc", "depth")):
                        res[k].append(fine[j])
            return {k: torch.cat(v).numpy() for k, v in res.items()}

        out.update({f"{tag}_hw": np.array([H, W_, nc, chunk]), f"{tag}_c2w": c2w.numpy(),
                    f"{tag}_focal": np.array(focal), f"{tag}_digest": np.array(dig)})
        out.update({f"{tag}_{k}": v for k, v in run().items()})
        out.update({f"{tag}_{k}": v for k, v in envelope(run).items()})
    save("render_frame.npz", **out)


def case_pdf_edges():
    """sorted_piecewise_constant_pdf / sample_pdf edge cases (helper.py:203-252)."""
    rng = np.random.Generator(np.random.PCG64(7))
    B, nb = 12, 64
    bins = np.sort(rng.uniform(2, 6, size=(B, nb)).astype(np.float32), -1)
    w = rng.uniform(0, 1, size=(B, nb - 1)).astype(np.float32)
    w[0] = 0.0                          # all-zero -> padding branch
    w[1, 10:40] = 0.0                   # plateau inside
    w[2] = 0.0; w[2, 5] = 1.0           # single spike -> cdf hits 1.0 early
    w[3] = 1e-9                         # tiny total below eps
    w[4, :] = 1.0                       # uniform -> u == cdf ties on the linspace grid
    w[5, -5:] = 0.0                     # zero tail
    w[6] = 0.0; w[6, -1] = 3.0          # mass only in the last bin
    w[7, ::2] = 0.0                     # alternating zeros
    out = {"bins": bins, "weights": w}
    for tag, randomized in (("eval", False), ("rand", True)):
        for ns in (128, 16):
            with RandQueue(3) as rq:
                s = helper.sorted_piecewise_constant_pdf(torch.from_numpy(bins), torch.from_numpy(w),
                                                         ns, randomized)
            out[f"{tag}{ns}_samples"] = s.numpy()
            if randomized:
                out[f"{tag}{ns}_u"] = rq.drawn[0]
    # u forced exactly onto cdf knots (ties) via a custom u table, uniform weights
    t_c = np.sort(rng.uniform(2, 6, size=(B, nb + 1)).astype(np.float32), -1)
    o = rng.normal(size=(B, 3)).astype(np.float32)
    d = rng.normal(size=(B, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=-1, keepdims=True)
    with RandQueue(4) as rq:
        tv, xyz = helper.sample_pdf(torch.from_numpy(bins), torch.from_numpy(w), torch.from_numpy(o),
                                    torch.from_numpy(d), torch.from_numpy(t_c), 128, True)
    out.update(sp_tc=t_c, sp_o=o, sp_d=d, sp_u=rq.drawn[0], sp_t=tv.numpy(), sp_xyz=xyz.numpy())
    tv, xyz = helper.sample_pdf(torch.from_numpy(bins), torch.from_numpy(w), torch.from_numpy(o),
                                torch.from_numpy(d), torch.from_numpy(t_c), 128, False)
    out.update(spe_t=tv.numpy(), spe_xyz=xyz.numpy())
    save("pdf_edges.npz", **out)


def case_composite_edges():
    """volumetric_rendering (helper.py:157-195) on crafted densities."""
    rng = np.random.Generator(np.random.PCG64(9))
    B, S = 16, 65
    t = np.sort(rng.uniform(2, 6, size=(B, S)).astype(np.float32), -1)
    rgb = rng.uniform(0, 1, size=(B, S, 3)).astype(np.float32)
    sig = rng.uniform(0, 2, size=(B, S, 1)).astype(np.float32)
    sig[0] = 0.0                        # empty ray -> acc 0, background
    sig[1, :, 0] = 1e4                  # opaque at the first sample
    sig[2, :-1] = 0.0                   # only the last (1e10 interval) sample
    sig[3, -1] = 0.0                    # last sample empty
    sig[4] = 1e-12                      # tiny densities against 1e10 last interval
    t[5, 10] = t[5, 11]                 # zero-length interval
    d = rng.normal(size=(B, 3)).astype(np.float32)
    d[:8] /= np.linalg.norm(d[:8], axis=-1, keepdims=True)  # half unit, half not
    out = {"t": t, "rgb": rgb, "sigma": sig, "dirs": d}
    for wb in (False, True):
        r = helper.volumetric_rendering(torch.from_numpy(rgb), torch.from_numpy(sig),
                                        torch.from_numpy(t), torch.from_numpy(d), wb)
        for k, v in zip(("comp_rgb", "acc", "weights", "depth"), r):
            out[f"wb{int(wb)}_{k}"] = v.numpy()
    save("composite_edges.npz", **out)


def case_pos_enc():
    """pos_enc (helper.py:136-140) including |x|~10 (args up to 2^9*10)."""
    rng = np.random.Generator(np.random.PCG64(11))
    x = rng.uniform(-10, 10, size=(64, 3)).astype(np.float32)
    x[0] = 0.0
    x[1] = [1e-7, -3.1415927, 10.0]
    v = rng.normal(size=(32, 3)).astype(np.float32)
    v /= np.linalg.norm(v, axis=-1, keepdims=True)
    save("pos_enc.npz", x=x, enc_x=helper.pos_enc(torch.from_numpy(x), 0, 10).numpy(),
         v=v, enc_v=helper.pos_enc(torch.from_numpy(v), 0, 4).numpy())


def case_train_step():
    """LitNeRF.training_step loss (model.py:256-282) + autograd grads, randomized with recorded
    uniforms (config C5 semantics at 64 rays)."""
    net, dig = make_nerf(0)
    net.train()
    rays, _, _, _ = frame_rays(16, 16, 3)
    sel = torch.arange(0, 256, 4)
    rays = {k: v[sel].contiguous() for k, v in rays.items()}
    rng = np.random.Generator(np.random.PCG64(3))
    target = torch.from_numpy(rng.uniform(0, 1, size=(64, 3)).astype(np.float32))
    with RandQueue(2) as rq:
        ret = net(rays, True, True, 2.0, 6.0)
    loss0 = helper.img2mse(ret[0][0], target)
    loss1 = helper.img2mse(ret[1][0], target)
    loss = loss1 + loss0
    loss.backward()
    keep = ("bias", "density_layer.weight", "rgb_layer.weight", "fine_mlp.pts_linears.0.weight",
            "fine_mlp.views_linear.0.weight")
    grads = {f"grad::{k}": p.grad.numpy().copy() for k, p in net.named_parameters()
             if any(k.endswith(s) for s in keep)}
    save("train_step.npz", digest=np.array(dig), **{k: v.numpy() for k, v in rays.items()},
         target=target.numpy(), u_coarse=rq.drawn[0], u_fine=rq.drawn[1],
         loss=np.array(loss.item(), dtype=np.float32), loss0=np.array(loss0.item(), np.float32),
         loss1=np.array(loss1.item(), np.float32),
         psnr0=helper.mse2psnr(loss0).detach().numpy(), **grads)


def case_articulated():
    """NeRF_AE_Art.forward (model_autodecoder.py:278-337) with fixed latents (CodeLibrary
    rows): eval on 256 rays of a 240x320 (config C3) view, and randomized with recorded
    uniforms on 128 rays; per-level outputs + intermediates + re-association envelope."""
    mad = _refimport.load_articulated()
    net = mad.NeRF_AE_Art()
    sd = W.art_state_dict(0)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    net.eval()
    lat = {k: torch.from_numpy(v) for k, v in W.art_latents(0).items()}
    rays, c2w, focal, _ = frame_rays(240, 320, pose_idx=11)
    out = {"digest": np.array(W.digest(sd))}
    for tag, sel, randomized in (("eval", torch.arange(0, 76800, 300), False),
                                 ("rand", torch.arange(17, 76800, 600), True)):
        r = {k: v[sel].contiguous() for k, v in rays.items()}

        def run():
            if randomized:
                with RandQueue(11) as rq:
                    ret, rec = capture_forward(net, r, True, True, extra=(lat,))
                run.drawn = rq.drawn
            else:
                ret, rec = capture_forward(net, r, False, True, extra=(lat,))
            return level_arrays(ret, rec)

        arrays = run()
        env = envelope(run)
        for k, v in {**{kk: r[kk].numpy() for kk in r}, **arrays, **env}.items():
            out[f"{tag}_{k}"] = v
        if randomized:
            out[f"{tag}_u_coarse"], out[f"{tag}_u_fine"] = run.drawn[0], run.drawn[1]
    for k, v in W.art_latents(0).items():
        out[f"latent_{k}"] = v
    save("articulated.npz", **out)


def case_art_train_step():
    """LitNeRF_AutoDecoder.training_step (model_autodecoder.py:395-477) run as the reference's
    own method on a stand-in ``self`` (code library, NeRF_AE_Art, near/far, a recording
    ``log``): loss = mse(fine) + mse(coarse) + 1e-4 latent regulariser, randomized with recorded
    uniforms, 64 rays of a 240x320 view; autograd gradients of the MLPs and of the code
    library's embedding tables."""
    import types

    mad = _refimport.load_articulated()
    from models.code_library import CodeLibraryArticulated

    net = mad.NeRF_AE_Art()
    sd = W.art_state_dict(0)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    net.train()
    lib = CodeLibraryArticulated(types.SimpleNamespace(N_max_objs=151, N_obj_code_length=128))
    tables = W.code_library_state_dict(0)
    lib.load_state_dict({k: torch.from_numpy(v) for k, v in tables.items()})
    logs = {}
    fake = types.SimpleNamespace(
        code_library=lib, model=net, white_bkgd=True, randomized=True, near=2.0, far=6.0,
        log=lambda k, v, **kw: logs.__setitem__(k, float(v)),
        optimizers=lambda: types.SimpleNamespace(param_groups=[{"lr": 5e-4}]))
    rays, _, _, _ = frame_rays(240, 320, pose_idx=23)
    sel = torch.arange(101, 76800, 1200)
    rays = {k: v[sel].contiguous() for k, v in rays.items()}
    rng = np.random.Generator(np.random.PCG64(5))
    target = torch.from_numpy(rng.uniform(0, 1, size=(64, 3)).astype(np.float32))
    iid, aid = 7, 3
    batch = {k: v[None] for k, v in rays.items()}
    batch.update(target=target[None], instance_id=torch.tensor([iid]),
                 articulation_id=torch.tensor([aid]), deg=torch.tensor([0.25]))
    with RandQueue(13) as rq:
        loss = mad.LitNeRF_AutoDecoder.training_step(fake, batch, 0)
    assert len(rq.drawn) == 2, len(rq.drawn)
    loss.backward()
    heavy = ("fine_mlp.deformations_linear.0.weight", "fine_mlp.pts_linears.0.weight",
             "fine_mlp.pts_linears.5.weight", "fine_mlp.views_linear.0.weight",
             "coarse_mlp.deformations_linear.0.weight")
    light = ("bias", "deformation_layer.weight", "density_layer.weight", "rgb_layer.weight")
    grads = {f"grad::{k}": p.grad.numpy().copy() for k, p in net.named_parameters()
             if k in heavy or any(k.endswith(s) for s in light)}
    for k, p in lib.named_parameters():
        row = iid if "articulation" not in k else aid
        assert np.count_nonzero(p.grad.numpy().any(axis=1)) == 1  # one row touched
        grads[f"grad::{k}"] = p.grad.numpy()[row].copy()
    save("art_train_step.npz", digest=np.array(W.digest(sd)), **{k: v.numpy() for k, v in rays.items()},
         target=target.numpy(), instance_id=np.array(iid), articulation_id=np.array(aid),
         u_coarse=rq.drawn[0], u_fine=rq.drawn[1], loss=np.array(loss.item(), dtype=np.float32),
         reg=np.array(logs["train/loss/reg"], np.float32), psnr0=np.array(logs["train/psnr0"], np.float32),
         psnr1=np.array(logs["train/psnr1"], np.float32),
         art_interp=lib.get_interpolated_articulations(2, "cpu").detach().numpy(), **grads)


def _write_png(path, arr, mode):
    from PIL import Image

    os.makedirs(os.path.dirname(path), exist_ok=True)
    Image.fromarray(arr, mode).save(path)


def make_mini_datasets(root):
    """Tiny synthetic datasets in the reference's two layouts (data files, committed):
    sapien_mini/{train,val}/{rgb/r_<i>.png (RGBA 40x30), transforms.json} (sapien.py) and
    multi_mini/inst1/train/deg0/{rgb (RGB), seg (L)}/r_<i>.png + transforms.json (sapien_multi)."""
    rng = np.random.Generator(np.random.PCG64(21))
    poses = sapien_multi.create_spheric_poses(4.0)
    for split, n in (("train", 3), ("val", 2)):
        frames = {}
        for i in range(n):
            img = rng.integers(0, 256, size=(30, 40, 4), dtype=np.uint8)
            img[:8, :, 3] = 0          # fully transparent rows
            img[-6:, :, 3] = 255       # opaque rows
            _write_png(os.path.join(root, "sapien_mini", split, "rgb", f"r_{i}.png"), img, "RGBA")
            frames[f"r_{i}"] = np.asarray(poses[3 + 7 * i + (split == "val")]).tolist()
        with open(os.path.join(root, "sapien_mini", split, "transforms.json"), "w") as f:
            json.dump({"camera_angle_x": 0.6911112070083618, "frames": frames}, f)
    base = os.path.join(root, "multi_mini", "inst1", "train", "deg0")
    frames = {}
    for i in range(2):
        img = rng.integers(0, 256, size=(30, 40, 3), dtype=np.uint8)
        seg = np.zeros((30, 40), dtype=np.uint8)
        seg[6:22, 9 + 5 * i:30 + 5 * i] = 3
        _write_png(os.path.join(base, "rgb", f"r_{i}.png"), img, "RGB")
        _write_png(os.path.join(base, "seg", f"r_{i}.png"), seg, "L")
        frames[f"r_{i}"] = np.asarray(poses[11 + 5 * i]).tolist()
    with open(os.path.join(base, "transforms.json"), "w") as f:
        json.dump({"camera_angle_x": 0.6911112070083618, "frames": frames}, f)


def case_datasets():
    """Reference SapienDataset (train buffers, val samples) and SapienDatasetMulti read_data +
    get_ray_batch (recorded pixel indices) on the mini datasets, img_wh (32, 24) (LANCZOS
    resize from 40x30)."""
    sapien, smulti = _refimport.load_datasets()
    root = os.path.join(HERE, "data")
    make_mini_datasets(root)
    out = {}
    ds = sapien.SapienDataset(os.path.join(root, "sapien_mini"), "train", img_wh=(32, 24),
                              white_back=True)
    files = [f for f in os.listdir(os.path.join(root, "sapien_mini", "train", "rgb"))]
    out["train_files"] = np.array(files)  # the reference's (listdir) image order
    out["train_focal"] = np.array(ds.focal)
    out["train_rays"] = ds.all_rays.numpy()
    out["train_rays_d"] = ds.all_rays_d.numpy()
    out["train_rgbs"] = ds.all_rgbs.numpy()
    dv = sapien.SapienDataset(os.path.join(root, "sapien_mini"), "val", img_wh=(32, 24),
                              white_back=True)
    for i in range(2):
        smp = dv[i] if i == 0 else dv.__getitem__(i)
        for k in ("rays_o", "rays_d", "viewdirs", "instance_mask", "target"):
            out[f"val{i}_{k}"] = smp[k].numpy()
    m = object.__new__(smulti.SapienDatasetMulti)
    m.root_dir, m.split, m.img_wh, m.white_back = os.path.join(root, "multi_mini"), "train", (32, 24), True
    m.img_transform = lambda x: x
    rays_o, view_dirs, rays_d, img, seg = m.read_data("inst1", "deg0", 1)
    pix = torch.from_numpy(np.random.Generator(np.random.PCG64(5)).integers(0, 768, 97)).long()
    orig = torch.randint
    torch.randint = lambda *a, **k: pix
    try:
        rays, rd, vd, _, rgbs, msk = m.get_ray_batch(rays_o, view_dirs, rays_d, img, seg, 97)
    finally:
        torch.randint = orig
    out["multi_files"] = np.array(os.listdir(os.path.join(root, "multi_mini", "inst1", "train",
                                                          "deg0", "rgb")))
    out["multi_pix"] = pix.numpy()
    out["multi_rays_o"], out["multi_rays_d"], out["multi_viewdirs"] = rays.numpy(), rd.numpy(), vd.numpy()
    out["multi_rgbs"], out["multi_mask"] = rgbs.numpy(), msk.numpy()
    save("datasets.npz", **out)


LIGHTNING_META = {"epoch": 7, "global_step": 1234, "pytorch-lightning_version": "1.5.10"}


def lightning_checkpoints():
    """The two Lightning checkpoint layouts the reference evaluates from (run.py:156-163):
    LitNeRF (self.model = NeRF, model.py:218) and LitNeRF_AutoDecoder (self.model = NeRF_AE_Art,
    self.code_library = CodeLibraryArticulated, model_autodecoder.py:356-357), with PCG64 weights
    (oracle/weights.py) and the keys of the reference modules' own state_dict()."""
    net, _ = make_nerf(0)
    mad = _refimport.load_articulated()
    art = mad.NeRF_AE_Art()
    art.load_state_dict({k: torch.from_numpy(v) for k, v in W.art_state_dict(0).items()})
    lib = {k: torch.from_numpy(v) for k, v in W.code_library_state_dict(0).items()}
    van = {"model." + k: v for k, v in net.state_dict().items()}
    artsd = {"model." + k: v for k, v in art.state_dict().items()}
    artsd.update({"code_library." + k: v for k, v in lib.items()})
    return {"vanilla": dict(LIGHTNING_META, state_dict=van, optimizer_states=[], lr_schedulers=[]),
            "articulated": dict(LIGHTNING_META, state_dict=artsd, optimizer_states=[],
                                lr_schedulers=[])}


CKPT_CASES = (("vanilla", "model", []), ("vanilla", "model", ["coarse_mlp"]),
              ("articulated", "model", []), ("articulated", "code_library", []),
              ("articulated", "model", ["fine_mlp.views_linear"]))


def case_checkpoint():
    """The reference's own utils.extract_model_state_dict (utils/__init__.py:117-132) applied to
    the checkpoints of lightning_checkpoints(): per case the extracted keys in order, their
    shapes and the sha256 of every tensor's bytes -> checkpoint_manifest.json (the checkpoint
    files themselves, ~10 MB, are regenerated by tests/test_checkpoint.py from the same PCG64
    weights and compared against this manifest)."""
    import hashlib
    import tempfile

    ref_utils = sys.modules["utils"]  # imported by the reference's model.py (utils.train_helper)
    cks = lightning_checkpoints()
    out = {"meta": LIGHTNING_META, "layouts": {}, "cases": []}
    with tempfile.TemporaryDirectory() as tmp:
        for name, ck in cks.items():
            path = os.path.join(tmp, f"{name}.ckpt")
            torch.save(ck, path)
            out["layouts"][name] = [[k, list(v.shape)] for k, v in ck["state_dict"].items()]
        for name, model_name, ignore in CKPT_CASES:
            ext = ref_utils.extract_model_state_dict(os.path.join(tmp, f"{name}.ckpt"), model_name,
                                                     list(ignore))
            out["cases"].append({
                "checkpoint": name, "model_name": model_name, "prefixes_to_ignore": list(ignore),
                "keys": list(ext), "shapes": [list(v.shape) for v in ext.values()],
                "sha256": [hashlib.sha256(v.contiguous().numpy().tobytes()).hexdigest()
                           for v in ext.values()]})
        # load_ckpt into a fresh reference NeRF: its state_dict afterwards
        fresh = model.NeRF()
        ref_utils.load_ckpt(fresh, os.path.join(tmp, "vanilla.ckpt"))
        out["load_ckpt_vanilla_sha256"] = {
            k: hashlib.sha256(v.contiguous().numpy().tobytes()).hexdigest()
            for k, v in fresh.state_dict().items()}
    path = os.path.join(HERE, "checkpoint_manifest.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=0)
    print(f"checkpoint_manifest.json: {os.path.getsize(path) / 1e3:.1f} kB")


if __name__ == "__main__":
    if len(sys.argv) > 1:  # e.g. `make_golden.py case_art_train_step`
        for name in sys.argv[1:]:
            globals()[name]()
        sys.exit(0)
    case_rays()
    case_forward_eval()
    case_forward_random()
    case_render_frame()
    case_pdf_edges()
    case_composite_edges()
    case_pos_enc()
    case_train_step()
    case_articulated()
    case_datasets()
    case_art_train_step()
    case_checkpoint()
