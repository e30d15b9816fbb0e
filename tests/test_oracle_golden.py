"""Pin the CPU oracle (oracle/nerf_oracle.py) against golden vectors produced by the reference.

The oracle is what every GPU parity test compares against, so it must reproduce the reference
on all committed fixtures first.  Tolerances: 0 (bit-exact) where the op sequence is identical,
1e-6 where only the fp32 GEMM blocking differs.
"""
import numpy as np
import torch

from oracle import nerf_oracle as O
from oracle import weights as W


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a))


def _params(digest):
    sd = W.nerf_state_dict(0)
    assert W.digest(sd) == str(digest), "regenerated weights drifted from the fixtures"
    return O.split_state_dict(sd)


def test_poses_and_rays(golden):
    g = golden("rays.npz")
    assert np.array_equal(O.create_spheric_poses(4.0).numpy(), g["poses"])
    for k in (0, 1):
        H, Wd, f = g[f"hwf{k}"]
        dirs = O.get_ray_directions(int(H), int(Wd), float(f))
        assert np.array_equal(dirs.numpy(), g[f"dirs{k}"])
        o, v, d, radii = O.get_rays(dirs, _t(g[f"c2w{k}"]), True, True)
        np.testing.assert_array_equal(o.numpy(), g[f"rays_o{k}"])
        np.testing.assert_allclose(d.numpy(), g[f"rays_d{k}"], rtol=0, atol=1e-7)
        np.testing.assert_allclose(v.numpy(), g[f"viewdirs{k}"], rtol=0, atol=1e-7)
        np.testing.assert_allclose(radii.numpy(), g[f"radii{k}"], rtol=0, atol=1e-7)
        o2, d2 = O.get_rays(dirs, _t(g[f"c2w{k}"]))
        np.testing.assert_allclose(d2.numpy(), g[f"plain_d{k}"], rtol=0, atol=1e-7)


def test_pos_enc(golden):
    g = golden("pos_enc.npz")
    assert np.array_equal(O.pos_enc(_t(g["x"]), 0, 10).numpy(), g["enc_x"])
    assert np.array_equal(O.pos_enc(_t(g["v"]), 0, 4).numpy(), g["enc_v"])


def test_composite(golden):
    g = golden("composite_edges.npz")
    for wb in (0, 1):
        out = O.volumetric_rendering(_t(g["rgb"]), _t(g["sigma"]), _t(g["t"]), _t(g["dirs"]), bool(wb))
        for k, v in zip(("comp_rgb", "acc", "weights", "depth"), out):
            np.testing.assert_allclose(v.numpy(), g[f"wb{wb}_{k}"], rtol=0, atol=1e-7, err_msg=k)


def test_pdf_edges_bit_exact(golden):
    g = golden("pdf_edges.npz")
    bins, w = _t(g["bins"]), _t(g["weights"])
    for ns in (128, 16):
        s = O.sorted_piecewise_constant_pdf(bins, w, ns, False)
        assert np.array_equal(s.numpy(), g[f"eval{ns}_samples"])
        s = O.sorted_piecewise_constant_pdf(bins, w, ns, True, u=_t(g[f"rand{ns}_u"]))
        assert np.array_equal(s.numpy(), g[f"rand{ns}_samples"])
    t, xyz = O.sample_pdf(bins, w, _t(g["sp_o"]), _t(g["sp_d"]), _t(g["sp_tc"]), 128, True,
                          u=_t(g["sp_u"]))
    assert np.array_equal(t.numpy(), g["sp_t"])
    assert np.array_equal(xyz.numpy(), g["sp_xyz"])
    t, xyz = O.sample_pdf(bins, w, _t(g["sp_o"]), _t(g["sp_d"]), _t(g["sp_tc"]), 128, False)
    assert np.array_equal(t.numpy(), g["spe_t"])


def _check_forward(g, randomized, white):
    params = _params(g["digest"])
    rays = {k: _t(g[k]) for k in ("rays_o", "rays_d", "viewdirs")}
    kw = {}
    if randomized:
        kw = dict(u_coarse=_t(g["u_coarse"]), u_fine=_t(g["u_fine"]))
    ret, inter = O.nerf_forward(params, rays, randomized, white, 2.0, 6.0,
                                return_intermediates=True, **kw)
    for lv, name in enumerate(("coarse", "fine")):
        np.testing.assert_allclose(inter[lv]["t_vals"].numpy(), g[f"{name}_t"], rtol=0, atol=1e-6)
        np.testing.assert_allclose(inter[lv]["raw_sigma"].numpy(), g[f"{name}_raw_sigma"], rtol=0,
                                   atol=1e-5)
        np.testing.assert_allclose(inter[lv]["raw_rgb"].numpy(), g[f"{name}_raw_rgb"], rtol=0, atol=1e-5)
        np.testing.assert_allclose(inter[lv]["weights"].numpy(), g[f"{name}_weights"], rtol=0, atol=1e-5)
        for j, k in enumerate(("rgb", "acc", "depth")):
            np.testing.assert_allclose(ret[lv][j].numpy(), g[f"{name}_{k}"], rtol=0, atol=1e-5,
                                       err_msg=f"{name}_{k}")


def test_forward_eval(golden):
    _check_forward(golden("forward_eval.npz"), False, True)


def test_forward_random(golden):
    _check_forward(golden("forward_random.npz"), True, False)


def test_render_frame_chunks(golden):
    g = golden("render_frame.npz")
    for tag in ("a", "c1"):
        H, Wd, nc, chunk = (int(x) for x in g[f"{tag}_hw"])
        params = _params(g[f"{tag}_digest"])
        dirs = O.get_ray_directions(H, Wd, float(g[f"{tag}_focal"]))
        o, v, d = O.get_rays(dirs, _t(g[f"{tag}_c2w"]), True)
        out = O.render_rays(params, dict(rays_o=o, rays_d=d, viewdirs=v), chunk, True, 2.0, 6.0,
                            num_coarse_samples=nc)
        for k in ("comp_rgb", "acc", "depth"):
            np.testing.assert_allclose(out[k].numpy(), g[f"{tag}_{k}"], rtol=0, atol=1e-5, err_msg=k)


def test_train_step_loss(golden):
    g = golden("train_step.npz")
    params = _params(g["digest"])
    for p in params:
        for v in p.values():
            v.requires_grad_(True)
    rays = {k: _t(g[k]) for k in ("rays_o", "rays_d", "viewdirs")}
    ret = O.nerf_forward(params, rays, True, True, 2.0, 6.0, u_coarse=_t(g["u_coarse"]),
                         u_fine=_t(g["u_fine"]))
    target = _t(g["target"])
    loss = O.img2mse(ret[1][0], target) + O.img2mse(ret[0][0], target)
    loss.backward()
    np.testing.assert_allclose(loss.item(), g["loss"], rtol=1e-6)
    for key in g:
        if key.startswith("grad::"):
            level, name = key[6:].split(".", 1)
            got = params[0 if level == "coarse_mlp" else 1][name].grad.numpy()
            np.testing.assert_allclose(got, g[key], rtol=1e-4, atol=1e-6, err_msg=key)


def test_articulated(golden):
    """NeRF_AE_Art (model_autodecoder.py:278-337): oracle vs the reference's outputs, eval and
    randomized (recorded uniforms)."""
    g = golden("articulated.npz")
    sd = W.art_state_dict(0)
    assert W.digest(sd) == str(g["digest"])
    params = O.split_state_dict(sd)
    lat = {k: _t(g[f"latent_{k}"]) for k in ("density", "color", "articulation")}
    for tag, randomized in (("eval", False), ("rand", True)):
        rays = {k: _t(g[f"{tag}_{k}"]) for k in ("rays_o", "rays_d", "viewdirs")}
        kw = dict(u_coarse=_t(g[f"{tag}_u_coarse"]), u_fine=_t(g[f"{tag}_u_fine"])) if randomized else {}
        ret, inter = O.art_nerf_forward(params, rays, randomized, True, 2.0, 6.0, lat,
                                        return_intermediates=True, **kw)
        for lv, name in enumerate(("coarse", "fine")):
            np.testing.assert_array_equal(inter[lv]["t_vals"].numpy(), g[f"{tag}_{name}_t"])
            for j, k in enumerate(("rgb", "acc", "depth")):
                np.testing.assert_allclose(ret[lv][j].numpy(), g[f"{tag}_{name}_{k}"], rtol=0,
                                           atol=1e-6, err_msg=f"{tag} {name} {k}")
            np.testing.assert_allclose(inter[lv]["raw_rgb"].numpy(), g[f"{tag}_{name}_raw_rgb"],
                                       rtol=0, atol=1e-6)


def test_art_train_step(golden):
    """LitNeRF_AutoDecoder.training_step (model_autodecoder.py:395-477): the oracle's loss
    (incl. the latent regulariser) and autograd gradients of both MLPs and of the code
    library's embedding rows vs the reference run on the same weights / uniforms."""
    g = golden("art_train_step.npz")
    sd = W.art_state_dict(0)
    assert W.digest(sd) == str(g["digest"])
    params = O.split_state_dict(sd)
    for p in params:
        for v in p.values():
            v.requires_grad_(True)
    tables = {k: _t(v).requires_grad_(True) for k, v in W.code_library_state_dict(0).items()}
    rays = {k: _t(g[k]) for k in ("rays_o", "rays_d", "viewdirs")}
    loss, loss0, loss1, reg = O.art_training_loss(
        params, tables, rays, _t(g["target"]), int(g["instance_id"]), int(g["articulation_id"]),
        True, True, 2.0, 6.0, u_coarse=_t(g["u_coarse"]), u_fine=_t(g["u_fine"]))
    loss.backward()
    np.testing.assert_allclose(loss.item(), g["loss"], rtol=1e-6)
    np.testing.assert_allclose(reg.item(), g["reg"], rtol=1e-6)
    np.testing.assert_allclose(O.mse2psnr(loss0).item(), g["psnr0"], rtol=1e-6)
    for key in g:
        if not key.startswith("grad::"):
            continue
        name = key[6:]
        if name.startswith("embedding"):
            row = int(g["articulation_id"] if "articulation" in name else g["instance_id"])
            got = tables[name].grad.numpy()[row]
        else:
            level, pname = name.split(".", 1)
            got = params[0 if level == "coarse_mlp" else 1][pname].grad.numpy()
        np.testing.assert_allclose(got, g[key], rtol=1e-4, atol=1e-6, err_msg=key)
