"""The articulated bf16 training mode (BASELINE config C5's "bf16" on LitNeRF_AutoDecoder;
NeRF_AE_Art(train_precision="bf16")): the backward chain and the weight-gradient GEMMs are bf16
throughout (aon_mlp_art_bwd_bf16, aon_gemm mma_bf16), kept activations and gradients bf16;
compositing, the loss, their backward, the latent terms and Adam stay fp32 on fp32 master
weights.  The forward (aon_mlp_art_fwd_train_bf16), the deformation MLP always fp16x3 (x' = delta
+ xyz feeds pos_enc's sin(2^9 x'), model_autodecoder.py:205-212), every later layer
(TrainNumerics.art_forward, a per-model setting):
  "f16_acts" (default): two fp16 MFMAs per product, the weights' exact hi / lo split and the
    activations rounded once to fp16 -- 8x finer than the bf16 copies the backward reads;
  "f16x3": fp16x3 throughout, only the stores bf16;
  "f16_weights": two fp16 MFMAs, the weights rounded to fp16, the activations exact;
  "bf16_trunk": the trunk, heads and view branch one bf16 MFMA per product (the mixed stream);
  "bf16_view": the view branch only bf16.
The articulated step's gradients are ill-conditioned in the forward values
(test_gpu_art_train.test_art_train_step_c5_4096_rays): a bf16 trunk's 2^-9 forward rounding alone
moves the deformation gradients to cosine 0.987 against the fp32 oracle, while the bf16 backward
stage-isolated at our own forward values is at cosine >= 0.9999 (tools/diag/art_bf16_diag.py,
profiles/r03/art_bf16/diag.log); the fp16 forwards sit at 0.9992 (activations) and 0.9989
(weights).

Gated as the vanilla bf16 mode (test_gpu_train_bf16.py): the C5 step's loss against the fp32
oracle within 3e-3, every gradient's cosine against it >= 0.999 and max-rel <= 0.05 (the default
and the fp16x3 forward); training step by step against the fp32 reference, teacher-forced, in
tests/test_gpu_teacher_forced.py (the free-running trajectories of rounds 3-5 were chaotic
quantities: oracle/trajectory.py).  The forward itself is pinned exactly where it is fp16x3.
"""
import numpy as np
import pytest
import torch

from oracle import nerf_oracle as O
from oracle import weights as W
from test_gpu_art_train import L_contig, _make, rel_err

pytestmark = pytest.mark.gpu


# the bf16 mode's forward numerics (TrainNumerics.art_forward): fp16x3 throughout, fp16
# activations (the default) or fp16 weights past the deformation MLP, the trunk bf16, or the view
# branch bf16
FWD_MODES = ["f16x3_fwd", "f16x", "f16w", "bf16_trunk", "bf16_view"]
ART_FORWARD = {"f16x3_fwd": "f16x3", "f16x": "f16_acts", "f16w": "f16_weights",
               "bf16_trunk": "bf16_trunk", "bf16_view": "bf16_view"}


def _level_inputs(seed=12, n=1024, **numerics):
    from test_gpu_train import c5_batch

    net, lib = _make(0, **numerics)
    batch, u_c, u_f = c5_batch(n=n, seed=seed)
    batch["instance_id"] = torch.tensor([7], device="cuda")
    batch["articulation_id"] = torch.tensor([3], device="cuda")
    return net, lib, batch, u_c, u_f


@pytest.mark.parametrize("mode", FWD_MODES)
@pytest.mark.parametrize("level", [0, 1], ids=["coarse", "fine"])
def test_art_bf16_forward(level, mode):
    """One level's training forward, f16x3 mode vs bf16 mode at the same t and the same
    (fp16x3-path) latent folds -- the kernels, not the folds, under test.  The deformation MLP
    is the fp16x3 kernel's in both, so x', pos_enc(x'), the points and the deformation layers'
    ReLU' bits are bit-identical, hd is exactly bf16(f16x3 hd) and the tiled 128-column enc_bf
    exactly bf16(pos_enc(x')) with zero padding.  The fp16x3 forward: everything
    is -- h / bot / hv exactly bf16 of the f16x3 values, raw and all ReLU' bits identical.
    True: the bf16 trunk's h / bot / hv and raw within bf16 distance of the fp64 oracle at our
    x' (gate 2e-2 of each tensor's max).  bf16_view: the trunk and bottleneck exactly as in the
    fp16x3 forward (h / bot and their ReLU' bits), the view branch's hv and raw within bf16
    distance of the fp64 oracle."""
    from aonerf import tiles, train_art

    trunk = mode != "f16x3_fwd"
    net, lib, batch, u_c, u_f = _level_inputs()
    latents = lib(batch)
    with torch.no_grad():
        ret = net(batch, True, True, 2.0, 6.0, {k: v.detach() for k, v in latents.items()},
                  u_coarse=u_c, u_fine=u_f, return_intermediates=True)
        t = ret[level][3]["t_vals"].contiguous()
        B, S = t.shape
        R = B * S
        mlp = net.fine_mlp if level else net.coarse_mlp
        geo = train_art._Geo(mlp)
        P = [(m.weight.detach(), m.bias.detach()) for m in train_art.art_layers(mlp)]
        lat = tuple(L_contig(latents[k]) for k in ("density", "color", "articulation"))
        out = {}
        enc_bf = torch.full((tiles.rows(R), 128), 7.0, device="cuda", dtype=torch.bfloat16)
        for bf in (False, True):
            raw = torch.empty((R, 4), device="cuda")
            masks = torch.empty((16, tiles.rows(R), 8), dtype=torch.int32, device="cuda")
            kept = train_art._forward_level_fused(geo, P, lat, batch["rays_o"], batch["rays_d"],
                                                  batch["viewdirs"], t, raw, None, masks, bf16=bf,
                                                  enc_bf=enc_bf if bf else None,
                                                  art_forward=ART_FORWARD[mode],
                                                  exact_folds=False)
            out[bf] = (kept, raw, masks)
        torch.cuda.synchronize()
    (xyz32, hd32, enc32, h32, bot32, hv32), raw32, m32 = out[False]
    (xyzbf, hdbf, encbf, hbf, botbf, hvbf), rawbf, mbf = out[True]
    assert hdbf.dtype == hbf.dtype == botbf.dtype == hvbf.dtype == torch.bfloat16
    # pos_enc(x'): the fp16x3 forward keeps it tiled (NR, 64), the bf16 one columns 0..15
    e32 = tiles.untile(enc32, R)
    assert encbf.shape == (tiles.rows(R), 16) and not e32[:, 63].any()
    assert torch.equal(xyzbf, xyz32) and torch.equal(tiles.untile(encbf, R), e32[:, :16])
    # the all-GEMM backward's row-major pos_enc(x') recomputed from the bf16 forward's x'
    # (aon_pos_enc, the kernel's own pos_enc_feature): bit-identical to what fp16x3 keeps
    assert torch.equal(train_art.enc_rows(geo, encbf, R), e32[:, :63])
    assert torch.equal(hdbf, hd32.to(torch.bfloat16))
    assert torch.equal(mbf[:4], m32[:4])  # ReLU' bits of hd0..3
    # the tiled bf16 copy of pos_enc(x') for the enc-column weight gradients
    eb = tiles.untile(enc_bf, R)
    assert torch.equal(eb[:, :63], e32[:, :63].to(torch.bfloat16)) and not eb[:, 63:].float().any()
    if not trunk:
        assert torch.equal(rawbf, raw32) and torch.equal(mbf, m32)
        for a, b in ((hbf, h32), (botbf, bot32), (hvbf, hv32)):
            assert torch.equal(a, b.to(torch.bfloat16))
        return
    if mode == "bf16_view":  # everything through the bottleneck is the fp16x3 forward's
        assert torch.equal(mbf[:12], m32[:12])
        for a, b in ((hbf, h32), (botbf, bot32)):
            assert torch.equal(a, b.to(torch.bfloat16))
    # the bf16 part against the fp64 oracle at our x'
    rec = {}
    names = ("density", "color", "articulation")
    p64 = {k[len("fine_mlp." if level else "coarse_mlp."):]: torch.from_numpy(v).double()
           for k, v in W.art_state_dict(0).items() if k.startswith("fine_mlp." if level else "coarse_mlp.")}
    venc = torch.empty((B, 27), device="cuda")
    from aonerf import _lib as L

    L.call("aon_pos_enc", L.ptr(batch["viewdirs"]), B, 0, 4, L.ptr(venc), L.stream())
    with torch.no_grad():
        samples = O.cast_rays(t.cpu().double(), batch["rays_o"].cpu().double(), batch["rays_d"].cpu().double())
        rgb64, sig64 = O.art_mlp_forward(p64, samples, venc.cpu().double(),
                                         {k: x.cpu().double() for k, x in zip(names, lat)},
                                         xp_fixed=tiles.untile(encbf, R)[:, :3].cpu(), record=rec)
    errs = {}
    for i in range(8):
        errs[f"h{i}"] = rel_err(tiles.untile(hbf[i], R).float().cpu(), rec["h"][i])
    errs["bot"] = rel_err(tiles.untile(botbf, R).float().cpu(), rec["bot"])
    for i in range(4):
        errs[f"hv{i}"] = rel_err(tiles.untile(hvbf[i], R).float().cpu(), rec["hv"][i])
    errs["raw_rgb"] = rel_err(rawbf[:, :3].cpu(), rgb64.reshape(-1, 3))
    errs["raw_sigma"] = rel_err(rawbf[:, 3].cpu(), sig64.reshape(-1))
    print(f"level {level} {mode} forward vs fp64 at our x':",
          {k: f"{v:.1e}" for k, v in errs.items()})
    if mode in ("f16w", "f16x"):  # bf16 storage (2^-9 of a value) + one fp16 rounding
        assert max(errs.values()) < 4e-3, errs
    assert max(errs.values()) < 2e-2, errs


@pytest.mark.parametrize("mode", FWD_MODES)
def test_art_bf16_train_step_c5(mode):
    """One C5 step of the articulated auto-decoder (4,096 rays, randomized, injected uniforms) in
    the bf16 mode: the loss against the fp32 oracle at our sample positions within 3e-3 relative,
    every MLP parameter's and latent code's gradient against the fp32 oracle (teacher-forced at
    our t) with cosine >= 0.999 and within 0.05 of its max (measured: cosine >= 0.99984, max-rel
    <= 2.1e-2 with the fp16x3 forward, 0.99919 / 0.049 with the default fp16-activation forward;
    the f16x3 mode meets 1e-3 -- or x'-attributed -- in
    test_gpu_art_train.test_art_train_step_c5_4096_rays).  "f16_weights" (not the default):
    cosine >= 0.998, max-rel <= 0.1 (measured 0.99886 / 0.074).  "bf16_trunk" (the bf16 trunk
    forward, not the default) is held to what its forward rounding allows: cosine >= 0.98,
    max-rel <= 0.3 (measured 0.987 / 0.21, the deformation gradients; the heads and view branch
    0.9994 / 0.07).  "bf16_view" (the view branch bf16, not the default either: it saves
    0.23 ms of the 10.1 ms step) likewise: cosine >= 0.995, max-rel <= 0.15 (measured 0.9968 /
    0.10, again the deformation gradients -- the view branch's bf16 rounding reaches them through
    the bottleneck's gradient)."""
    from aonerf import train_art

    min_cos, max_rel = {"bf16_trunk": (0.98, 0.3), "bf16_view": (0.995, 0.15),
                        "f16w": (0.998, 0.1)}.get(mode, (0.999, 0.05))
    net, lib, batch, u_c, u_f = _level_inputs(n=4096, precision="bf16",
                                              art_forward=ART_FORWARD[mode])
    latents = lib(batch)
    ret = net(batch, True, True, 2.0, 6.0, latents, u_coarse=u_c, u_fine=u_f,
              return_intermediates=True)
    target = batch["target"]
    loss = train_art.img2mse(ret[1][0], target) + train_art.img2mse(ret[0][0], target)
    for x in latents.values():
        x.retain_grad()
    loss.backward()
    torch.cuda.synchronize()
    rays = {k: batch[k].cpu() for k in ("rays_o", "rays_d", "viewdirs")}
    params = [{k: v.requires_grad_(True) for k, v in p.items()}
              for p in O.split_state_dict(W.art_state_dict(0))]
    lat = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in latents.items()}
    tgt = target.cpu()
    ref_loss = 0.0
    for level in range(2):
        t = ret[level][3]["t_vals"].cpu()
        comp = O.art_render_level(params, rays, t, level, True, lat)[0]
        ref_loss = ref_loss + O.img2mse(comp, tgt)
    ref_loss.backward()
    print(f"C5 art bf16 loss gpu {loss.item():.6f}  fp32 oracle on our t {ref_loss.item():.6f}")
    np.testing.assert_allclose(loss.item(), ref_loss.item(), rtol=3e-3)
    want = {f"{pre}{n}": v.grad.double().numpy()
            for lv, pre in ((0, "coarse_mlp."), (1, "fine_mlp.")) for n, v in params[lv].items()}
    want.update({f"latent {k}": v.grad.double().numpy() for k, v in lat.items()})
    ours = {n: p.grad.double().cpu().numpy() for n, p in net.named_parameters()}
    ours.update({f"latent {k}": v.grad.double().cpu().numpy() for k, v in latents.items()})
    worst_e, worst_c, bad = 0.0, 1.0, []
    for name, w in want.items():
        got = ours[name].reshape(w.shape)
        e = rel_err(got, w)
        cos = float((got * w).sum() / (np.linalg.norm(got) * np.linalg.norm(w) + 1e-300))
        worst_e, worst_c = max(worst_e, e), min(worst_c, cos)
        if e > 1e-2 or cos < 0.9999:
            print(f"  {name:45s} max-rel {e:.2e}  cosine {cos:.6f}")
        if not (e < max_rel and cos >= min_cos):
            bad.append((name, e, cos))
    print(f"C5 art bf16 grads vs fp32 oracle: worst max-rel {worst_e:.2e}, worst cosine {worst_c:.6f}")
    assert not bad, bad


_LAYERS = (["deformations_linear.%d" % i for i in range(4)] + ["deformation_layer"]
           + ["pts_linears.%d" % i for i in range(8)] + ["density_layer", "bottleneck_layer"]
           + ["views_linear.%d" % i for i in range(4)] + ["rgb_layer"])


@pytest.mark.parametrize("level", [0, 1], ids=["coarse", "fine"])
def test_art_bf16_backward_stage_isolated(level):
    """The bf16 backward (aon_mlp_art_bwd_bf16 + the mma_bf16 weight-gradient GEMMs) on its own:
    the fp64 oracle's autograd forced to OUR kept forward values (oracle.art_mlp_forward_kept,
    the bf16 trunk forward's bf16 activations) with OUR d raw (the compositing backward of the C5
    loss), every parameter's and latent code's gradient within 3e-2 of its max and cosine
    >= 0.9999 (measured <= 1.9e-2 / >= 0.99990 at 4,096 rays): what separates the bf16-trunk
    step from the fp32 oracle is its forward rounding, not the backward kernels."""
    from aonerf import _lib as L
    from aonerf import tiles, train_art

    net, lib, batch, u_c, u_f = _level_inputs(n=1024)
    latents = lib(batch)
    with torch.no_grad():
        ret = net(batch, True, True, 2.0, 6.0, {k: v.detach() for k, v in latents.items()},
                  u_coarse=u_c, u_fine=u_f, return_intermediates=True)
    lat_t = tuple(L_contig(latents[k]) for k in ("density", "color", "articulation"))
    mlp = net.fine_mlp if level else net.coarse_mlp
    t = ret[level][3]["t_vals"].contiguous()
    B, S = t.shape
    R = B * S
    geo = train_art._Geo(mlp)
    P = [(m.weight.detach(), m.bias.detach()) for m in train_art.art_layers(mlp)]
    raw = torch.empty((R, 4), device="cuda")
    masks = torch.empty((16, tiles.rows(R), 8), dtype=torch.int32, device="cuda")
    xyz, hd, enc, h, bot, hv, enc_bf = train_art._forward_level_fused(
        geo, P, lat_t, batch["rays_o"], batch["rays_d"], batch["viewdirs"], t, raw, None, masks,
        bf16=True, return_enc_bf=True, art_forward="bf16_trunk")
    venc = torch.empty((B, 27), device="cuda")
    L.call("aon_pos_enc", L.ptr(batch["viewdirs"]), B, 0, 4, L.ptr(venc), L.stream())
    comp = torch.empty((B, 3), device="cuda")
    acc = torch.empty((B,), device="cuda")
    wts = torch.empty((B, S), device="cuda")
    depth = torch.empty((B,), device="cuda")
    L.call("aon_composite_fwd", L.ptr(raw), 4, L.ptr(raw[:, 3:]), 4, L.ptr(t), L.ptr(batch["rays_d"]),
           B, S, 1, L.ACT_ARTIC, L.ptr(comp), L.ptr(acc), L.ptr(wts), L.ptr(depth), L.stream())
    g_rgb = (2.0 * (comp - batch["target"]) / (3 * B)).contiguous()
    draw = torch.empty((R, 4), device="cuda")
    L.call("aon_composite_bwd", L.ptr(raw), 4, L.ptr(raw[:, 3:]), 4, L.ptr(t), L.ptr(batch["rays_d"]),
           B, S, 1, L.ACT_ARTIC, L.ptr(g_rgb), None, None, L.ptr(draw), L.ptr(draw[:, 3:]), 4,
           L.stream())
    G = [(torch.empty_like(w), torch.empty_like(b)) for w, b in P]
    dlat = tuple(torch.empty_like(x) for x in lat_t)
    train_art._backward_level_fused(geo, P, G, lat_t, dlat, xyz, enc, venc, S, hd, h, bot, hv,
                                    draw, masks, True, enc_bf)
    torch.cuda.synchronize()
    assert h[0].dtype == torch.bfloat16
    rm = [torch.stack([tiles.untile(x, R).float() for x in tt]).cpu() for tt in (hd, h, hv)]
    enc_c = train_art.enc_rows(geo, enc, R).cpu()
    kept = {"xyz": xyz.cpu(), "hd": list(rm[0]), "xp": enc_c[:, :3].clone(), "enc": enc_c,
            "h": list(rm[1]), "bot": tiles.untile(bot, R).float().cpu(), "hv": list(rm[2])}
    pre = "fine_mlp." if level else "coarse_mlp."
    p64 = {k[len(pre):]: torch.from_numpy(v).double().requires_grad_(True)
           for k, v in W.art_state_dict(0).items() if k.startswith(pre)}
    names = ("density", "color", "articulation")
    l64 = {k: x.cpu().double().requires_grad_(True) for k, x in zip(names, lat_t)}
    r_rgb, r_sig = O.art_mlp_forward_kept(p64, kept, venc.cpu(), l64, S)
    d64 = draw.cpu().double()
    torch.autograd.backward([r_rgb, r_sig], [d64[:, :3], d64[:, 3:]])
    pairs = []
    for (dw, db), name in zip(G, _LAYERS):
        pairs += [(name + ".weight", dw, p64[name + ".weight"].grad),
                  (name + ".bias", db, p64[name + ".bias"].grad)]
    pairs += [("latent " + k, d, l64[k].grad) for d, k in zip(dlat, names)]
    worst_e, worst_c, bad = 0.0, 1.0, []
    for name, got, want in pairs:
        g_ = got.double().cpu().numpy().reshape(-1)
        w_ = want.numpy().reshape(-1)
        e = rel_err(g_, w_)
        cos = float(g_ @ w_ / (np.linalg.norm(g_) * np.linalg.norm(w_) + 1e-300))
        worst_e, worst_c = max(worst_e, e), min(worst_c, cos)
        if not (e <= 3e-2 and cos >= 0.9999):
            bad.append((name, e, cos))
    print(f"level {level} bf16 backward stage-isolated: worst max-rel {worst_e:.2e}, "
          f"worst cosine {worst_c:.6f}")
    assert not bad, bad
