"""GPU parity of the articulated training path (reference LitNeRF_AutoDecoder.training_step,
models/vanilla_nerf/model_autodecoder.py:395-477): the pos_enc backward and the latent
regulariser kernels against torch autograd through the CPU oracle, the whole training step
(loss, both MLPs' gradients, the code-library rows' gradients) against the reference's golden
vectors, teacher-forced per-level gradients, and an Adam step over all 83 parameter tensors.

Tolerances: pos_enc backward 1e-5 of each tensor's gradient scale (fp32 sin' = cos at the same
fp32 arguments, ulp-level differences of cosf at |arg| <= 5120); regulariser 1e-6 relative;
loss rtol 1e-5.  Gradients:
  * stage-isolated (test_art_backward_stage_isolated): the backward kernels on the GPU
    forward's own kept tensors vs the fp64 oracle backward at those same values, every tensor
    within 1e-4 of its max -- the gate that sees a kernel error well below the reference's own
    fp32 noise;
  * C5-size stage isolation per level (test_art_c5_level_stage_isolated): forward values 1e-5,
    d raw 1e-5 / 1e-4, backward 1e-4, each against fp64 at our own inputs;
  * x'- and mask-forced at C5's size: the fp64 oracle at our deformed points and our ReLU'
    pattern, 1e-4 of each tensor's max; our ReLU' flips against fp64 at most twice the fp32
    oracle's (the x'-forced distance alone, ~1e-3, is a lottery of those flips);
  * free-running (the deformation gradients pass through sin(2^9 x'), so the reference's own
    fp32 evaluation sits up to ~1e-2 from fp64): vs the reference's golden gradients within
    max(4 x its fp32-vs-fp64 spread, 1e-4); teacher-forced vs the fp32 oracle within
    max(2 x that tensor's own spread, 1e-3) -- at C5's size a tensor outside it must be
    attributed to the last bits of x' (x'-forced gate held, our x' no less accurate than the
    reference's fp32 x'); measured values printed.
"""
import numpy as np
import pytest
import torch

from oracle import nerf_oracle as O
from oracle import weights as W

pytestmark = pytest.mark.gpu


def cuda(a):
    return torch.as_tensor(np.ascontiguousarray(a)).cuda()


def rel_err(got, want):
    got, want = np.asarray(got, np.float64), np.asarray(want, np.float64)
    scale = np.abs(want).max() if want.size else 1.0
    return float(np.abs(got - want).max() / max(scale, 1e-30)) if want.size else 0.0


@pytest.mark.parametrize("n,L", [(1000, 10), (37, 4), (1, 10)])
def test_pos_enc_backward(n, L):
    from aonerf import _lib

    gen = torch.Generator().manual_seed(n + L)
    x = (torch.rand(n, 3, generator=gen) - 0.5) * 20
    x[0] = torch.tensor([0.0, -3.1415927, 10.0])
    g = torch.randn(n, 3 + 6 * L, generator=gen)
    xr = x.clone().requires_grad_(True)
    O.pos_enc(xr, 0, L).backward(g)
    enc = torch.empty((n, 3 + 6 * L), device="cuda")
    xd, gd = x.cuda(), g.cuda()
    _lib.call("aon_pos_enc", _lib.ptr(xd), n, 0, L, _lib.ptr(enc), _lib.stream())
    dx = torch.full((n, 3), 0.5, device="cuda")
    # identity channels of the encoding as the points (ldx = 3 + 6L), accumulate into dx
    _lib.call("aon_pos_enc_bwd", _lib.ptr(enc), 3 + 6 * L, _lib.ptr(gd), 3 + 6 * L, n, 0, L, 1,
              _lib.ptr(dx), 3, _lib.stream())
    got = dx.cpu().numpy() - 0.5
    e = rel_err(got, xr.grad.numpy())
    print(f"pos_enc backward n={n} L={L}: max rel err {e:.2e}")
    assert e < 1e-5


def test_latent_reg():
    from aonerf.train_art import LatentReg

    lat = {k: cuda(v) for k, v in W.art_latents(3).items()}
    lat["density"][0, 5] = 0.0  # zero entry: torch's norm backward gives 0
    codes = [lat[k].clone().requires_grad_(True) for k in ("density", "color", "articulation")]
    loss = LatentReg.apply(*codes)
    loss.backward()
    ref_codes = [lat[k].cpu().clone().requires_grad_(True) for k in ("density", "color", "articulation")]
    ref = O.latent_reg_loss(dict(zip(("density", "color", "articulation"), ref_codes)))
    ref.backward()
    np.testing.assert_allclose(loss.item(), ref.item(), rtol=1e-6)
    for c, r in zip(codes, ref_codes):
        np.testing.assert_allclose(c.grad.cpu().numpy(), r.grad.numpy(), rtol=1e-6, atol=0)


@pytest.fixture(params=[(True, True), (False, False), (True, False), (False, True)],
                ids=["fused", "gemm", "fused_fwd_gemm_bwd", "gemm_fwd_fused_bwd"])
def art_fwd_mode(request):
    """Articulated training forward on the fused kernel with activation stores
    (aon_mlp_art_fwd_train) or layer by layer on aon_gemm; input gradients in the fused chain
    (aon_mlp_art_bwd) or as GEMMs + aon_pos_enc_bwd.  The mixed pairs convert pos_enc(x')
    between the fused kernels' tiled copy and the GEMMs' row-major one (train_art.enc_rows /
    _enc_tiled).  The model's TrainNumerics."""
    fwd, bwd = request.param
    return dict(fused_forward=fwd, fused_backward=bwd)


def test_fused_art_train_forward_activations():
    """aon_mlp_art_fwd_train's kept tensors and raw outputs (with noise) against the
    layer-by-layer GEMM forward on a ragged batch: the points bit-exact, the deformation layers
    ~1e-6 of each tensor's range (both f16x3), pos_enc(x') and the layers after it within the
    sin(2^9 x') amplification of that (measured ~4e-5)."""
    from aonerf import tiles, train_art
    from aonerf import _lib as L

    net, _ = _make(0)
    mlp = net.fine_mlp
    geo = train_art._Geo(mlp)
    gen = torch.Generator().manual_seed(4)
    B, S = 37, 65
    o = (torch.rand(B, 3, generator=gen) - 0.5).cuda()
    d = torch.nn.functional.normalize(torch.randn(B, 3, generator=gen), dim=-1).cuda()
    t = (2.0 + 4.0 * torch.rand(B, S, generator=gen)).sort(-1).values.cuda()
    noise = torch.rand(B * S, generator=gen).cuda()
    lat = tuple(cuda(v) for v in W.art_latents(1).values())
    P = [(m.weight.detach(), m.bias.detach()) for m in train_art.art_layers(mlp)]
    raw_f = torch.empty((B * S, 4), device="cuda")
    R = B * S
    masks = torch.empty((16, tiles.rows(R), 8), dtype=torch.int32, device="cuda")
    xyz_f, hd_t, enc_f, h_t, bot_t, hv_t = train_art._forward_level_fused(geo, P, lat, o, d, d, t,
                                                                         raw_f, noise, masks)
    # kept tensors are tiled (aonerf/tiles.py; 2,405 rows: a partial last block)
    hd_f, h_f, hv_f = ([tiles.untile(x, R) for x in tt] for tt in (hd_t, h_t, hv_t))
    bot_f = tiles.untile(bot_t, R)
    enc_f = train_art.enc_rows(geo, enc_f, R)  # tiled (NR, 64), column 63 zero
    # the ReLU' bits written by the forward == those built from its stored activations
    rebuilt = train_art.relu_masks(list(hd_f) + list(h_f) + list(hv_f), R)
    for i in range(16):
        assert torch.equal(tiles.untile_masks(masks[i], R), tiles.untile_masks(rebuilt[i], R)), i
    xyz = torch.empty((B * S, 3), device="cuda")
    L.call("aon_cast_rays", L.ptr(o), L.ptr(d), L.ptr(t), B, S, None, 0, L.ptr(xyz), 0, 0, None,
           L.stream())
    venc = torch.empty((B, 27), device="cuda")
    L.call("aon_pos_enc", L.ptr(d), B, 0, 4, L.ptr(venc), L.stream())
    raw_g = torch.empty((B * S, 4), device="cuda")
    hd_g, enc_g, h_g, bot_g, hv_g = train_art._forward_level(geo, P, lat, xyz, venc, S, raw_g, noise)
    np.testing.assert_array_equal(xyz_f.cpu().numpy(), xyz.cpu().numpy())
    pairs = ([(f"hd{i}", hd_f[i], hd_g[i]) for i in range(4)] + [("enc", enc_f, enc_g)]
             + [(f"h{i}", h_f[i], h_g[i]) for i in range(8)]
             + [("bot", bot_f, bot_g)] + [(f"hv{i}", hv_f[i], hv_g[i]) for i in range(4)]
             + [("raw", raw_f, raw_g)])
    for name, a, b in pairs:
        e = rel_err(a.cpu().numpy(), b.cpu().numpy())
        print(f"  fused vs gemm forward {name}: max rel err {e:.2e}")
        # enc carries sin(2^9 x'): a 1e-7 change of x' (the two deformation evaluations differ
        # by that) moves it by ~1e-4, and everything after it inherits that
        assert e < (2e-5 if name.startswith("hd") else 5e-4), name


def test_fused_art_backward_chain():
    """aon_mlp_art_bwd (+ the weight-gradient GEMMs) against the all-GEMM backward on the same
    kept activations and d raw (ragged batch): every parameter and latent gradient within
    2e-5 of its tensor's max (two f16x3 evaluations of the same products).  The fused chain
    reads the forward's tiled tensors in place, the GEMM backward their row-major copies."""
    from aonerf import tiles, train_art

    net, _ = _make(0)
    mlp = net.fine_mlp
    geo = train_art._Geo(mlp)
    gen = torch.Generator().manual_seed(6)
    B, S = 29, 65
    R = B * S
    o = (torch.rand(B, 3, generator=gen) - 0.5).cuda()
    d = torch.nn.functional.normalize(torch.randn(B, 3, generator=gen), dim=-1).cuda()
    t = (2.0 + 4.0 * torch.rand(B, S, generator=gen)).sort(-1).values.cuda()
    lat = tuple(cuda(v) for v in W.art_latents(2).values())
    P = [(m.weight.detach(), m.bias.detach()) for m in train_art.art_layers(mlp)]
    raw = torch.empty((R, 4), device="cuda")
    xyz, hd, enc, h, bot, hv = train_art._forward_level_fused(geo, P, lat, o, d, d, t, raw)
    venc = torch.empty((B, 27), device="cuda")
    L = train_art.L
    L.call("aon_pos_enc", L.ptr(d), B, 0, 4, L.ptr(venc), L.stream())
    draw = (torch.randn(R, 4, generator=gen) * 1e-3).cuda()
    out = {}
    rm = [torch.stack([tiles.untile(x, R) for x in tt]) for tt in (hd, h, hv)]
    kept = {"fused": (hd, h, bot, hv),
            "gemm": (rm[0], rm[1], tiles.untile(bot, R), rm[2])}
    for mode, fn in (("fused", train_art._backward_level_fused), ("gemm", train_art._backward_level)):
        G = [(torch.empty_like(w), torch.empty_like(b)) for w, b in P]
        dlat = tuple(torch.empty_like(x) for x in lat)
        khd, kh, kbot, khv = kept[mode]
        fn(geo, P, G, lat, dlat, xyz, enc, venc, S, khd, kh, kbot, khv, draw)
        out[mode] = [g for pair in G for g in pair] + list(dlat)
    names = [f"{i}.{k}" for i in range(20) for k in ("w", "b")] + ["shape", "app", "art"]
    worst = 0.0
    for name, a, b in zip(names, out["fused"], out["gemm"]):
        e = rel_err(a.cpu().numpy(), b.cpu().numpy())
        worst = max(worst, e)
        assert e < 2e-5, (name, e)
    print(f"fused vs GEMM articulated backward: worst max-rel err {worst:.2e}")


_ART_NAMES = ([f"deformations_linear.{i}" for i in range(4)] + ["deformation_layer"]
              + [f"pts_linears.{i}" for i in range(8)] + ["density_layer", "bottleneck_layer"]
              + [f"views_linear.{i}" for i in range(4)] + ["rgb_layer"])  # train_art.art_layers order


@pytest.mark.parametrize("B,S,level,scale", [(29, 65, 1, 1e-3), (128, 193, 1, 1e-4),
                                             (4096, 65, 0, 1e-4)],
                         ids=["ragged", "fine193", "c5_coarse_4096"])
@pytest.mark.parametrize("bwd", ["fused", "gemm"])
def test_art_backward_stage_isolated(B, S, level, scale, bwd):
    """Stage isolation of the articulated backward (model_autodecoder.py:168-239): the GPU
    forward's own kept tensors -- the points, the deformation activations, x', pos_enc(x'), the
    trunk / bottleneck / view activations and their ReLU' bits -- and a fixed d raw go through
    (a) aon_mlp_art_bwd + the weight-gradient aon_gemm's (``fused``) or the all-GEMM backward
    + aon_pos_enc_bwd (``gemm``), and (b) the oracle's fp64 autograd evaluated at exactly those
    forward values (oracle.art_mlp_forward_kept; pos_enc's derivative cos at the fp32
    arguments of the GPU's x').  Nothing the forward computed differently is amplified, so every
    weight, bias and latent-code gradient must agree within 1e-4 of its tensor's max (f16x3
    operands carry ~22 bits; measured values printed).  The last case is config C5's coarse
    level at its size (4,096 rays)."""
    from aonerf import tiles, train_art

    net, _ = _make(0)
    mlp = net.fine_mlp if level else net.coarse_mlp
    geo = train_art._Geo(mlp)
    gen = torch.Generator().manual_seed(B + S)
    R = B * S
    o = (torch.rand(B, 3, generator=gen) - 0.5).cuda()
    d = torch.nn.functional.normalize(torch.randn(B, 3, generator=gen), dim=-1).cuda()
    t = (2.0 + 4.0 * torch.rand(B, S, generator=gen)).sort(-1).values.cuda()
    lat = tuple(cuda(v) for v in W.art_latents(2).values())
    layers = train_art.art_layers(mlp)
    P = [(m.weight.detach(), m.bias.detach()) for m in layers]
    raw = torch.empty((R, 4), device="cuda")
    masks = torch.empty((16, tiles.rows(R), 8), dtype=torch.int32, device="cuda")
    xyz, hd, enc, h, bot, hv = train_art._forward_level_fused(geo, P, lat, o, d, d, t, raw, None,
                                                              masks)
    L = train_art.L
    venc = torch.empty((B, 27), device="cuda")
    L.call("aon_pos_enc", L.ptr(d), B, 0, 4, L.ptr(venc), L.stream())
    draw = (torch.randn(R, 4, generator=gen) * scale).cuda()
    G = [(torch.empty_like(w), torch.empty_like(b)) for w, b in P]
    dlat = tuple(torch.empty_like(x) for x in lat)
    rm = [torch.stack([tiles.untile(x, R) for x in tt]) for tt in (hd, h, hv)]
    bot_rm = tiles.untile(bot, R)
    if bwd == "fused":
        train_art._backward_level_fused(geo, P, G, lat, dlat, xyz, enc, venc, S, hd, h, bot, hv,
                                        draw, masks, True)
    else:
        train_art._backward_level(geo, P, G, lat, dlat, xyz, enc, venc, S, rm[0], rm[1], bot_rm,
                                  rm[2], draw)
    torch.cuda.synchronize()
    # fp64 oracle backward at the GPU's own forward values
    sd = W.art_state_dict(0)
    pre = "fine_mlp." if level else "coarse_mlp."
    p64 = {k[len(pre):]: torch.from_numpy(v).double().requires_grad_(True)
           for k, v in sd.items() if k.startswith(pre)}
    names = ("density", "color", "articulation")
    l64 = {k: x.cpu().double().requires_grad_(True) for k, x in zip(names, lat)}
    enc_c = train_art.enc_rows(geo, enc, R).cpu()
    kept = {"xyz": xyz.cpu(), "hd": list(rm[0].cpu()), "xp": enc_c[:, :3].clone(), "enc": enc_c,
            "h": list(rm[1].cpu()), "bot": bot_rm.cpu(), "hv": list(rm[2].cpu())}
    r_rgb, r_sig = O.art_mlp_forward_kept(p64, kept, venc.cpu(), l64, S)
    d64 = draw.cpu().double()
    torch.autograd.backward([r_rgb, r_sig], [d64[:, :3], d64[:, 3:]])
    worst, worst_name = 0.0, ""
    for (dw, db), name in zip(G, _ART_NAMES):
        for got, key in ((dw, f"{name}.weight"), (db, f"{name}.bias")):
            e = rel_err(got.cpu().numpy(), p64[key].grad.numpy())
            if e > worst:
                worst, worst_name = e, key
            assert e <= 1e-4, (key, e)
    for got, k in zip(dlat, names):
        e = rel_err(got.cpu().numpy(), l64[k].grad.numpy().reshape(got.shape))
        if e > worst:
            worst, worst_name = e, f"latent {k}"
        assert e <= 1e-4, (k, e)
    print(f"articulated backward ({bwd}, B={B}, S={S}) vs fp64 at the GPU's forward values: "
          f"worst {worst:.2e} ({worst_name})")


@pytest.mark.parametrize("level", [0, 1], ids=["coarse", "fine"])
def test_art_c5_level_stage_isolated(level):
    """Config C5's articulated step at its size, one level, every kernel stage-isolated against
    fp64 at OUR forward values (nothing amplified by sin(2^9 x')):
      (ii)  the fused training forward's kept tensors (deformation activations, pos_enc(x'),
            trunk, bottleneck, view branch) and raw outputs against the fp64 forward at our x'
            (oracle.art_mlp_forward, xp_fixed): within 1e-5 of each tensor's max (measured <= 7e-7);
      (iii) our compositing backward's d raw (the C5 loss's gradient) against fp64 autograd of
            the compositor on the fp64 raw: rgb 1e-5, sigma 1e-4 (measured 1.3e-6 / 1.4e-5: dL/dsigma
            is a difference of transmittance-weighted sums);
      (i)   aon_mlp_art_bwd + the weight GEMMs on our kept tensors with THAT d raw against the fp64
            backward at the same values (oracle.art_mlp_forward_kept): 1e-4 (measured <= 3.5e-6)."""
    from aonerf import tiles, train_art
    from test_gpu_train import c5_batch

    L = train_art.L
    net, lib = _make(0)
    batch, u_c, u_f = c5_batch(seed=12)
    batch["instance_id"] = torch.tensor([7], device="cuda")
    batch["articulation_id"] = torch.tensor([3], device="cuda")
    latents = {k: v.detach() for k, v in lib(batch).items()}
    with torch.no_grad():
        ret = net(batch, True, True, 2.0, 6.0, latents, u_coarse=u_c, u_fine=u_f,
                  return_intermediates=True)
    t = ret[level][3]["t_vals"].contiguous()
    B, S = t.shape
    R = B * S
    mlp = net.fine_mlp if level else net.coarse_mlp
    geo = train_art._Geo(mlp)
    P = [(m.weight.detach(), m.bias.detach()) for m in train_art.art_layers(mlp)]
    names = ("density", "color", "articulation")
    lat = tuple(latents[k].reshape(1, -1).contiguous() for k in names)
    raw = torch.empty((R, 4), device="cuda")
    masks = torch.empty((16, tiles.rows(R), 8), dtype=torch.int32, device="cuda")
    xyz, hd, enc, h, bot, hv = train_art._forward_level_fused(
        geo, P, lat, batch["rays_o"], batch["rays_d"], batch["viewdirs"], t, raw, None, masks)
    venc = torch.empty((B, 27), device="cuda")
    L.call("aon_pos_enc", L.ptr(batch["viewdirs"]), B, 0, 4, L.ptr(venc), L.stream())
    comp = torch.empty((B, 3), device="cuda")
    acc = torch.empty((B,), device="cuda")
    wts = torch.empty((B, S), device="cuda")
    depth = torch.empty((B,), device="cuda")
    L.call("aon_composite_fwd", L.ptr(raw), 4, L.ptr(raw[:, 3:]), 4, L.ptr(t), L.ptr(batch["rays_d"]),
           B, S, 1, L.ACT_ARTIC, L.ptr(comp), L.ptr(acc), L.ptr(wts), L.ptr(depth), L.stream())
    loss = torch.empty((), device="cuda")
    g_rgb = torch.empty((B, 3), device="cuda")
    L.call("aon_mse", L.ptr(comp), L.ptr(batch["target"]), 3 * B, 1.0, L.ptr(loss), L.ptr(g_rgb),
           L.stream())
    draw = torch.empty((R, 4), device="cuda")
    L.call("aon_composite_bwd", L.ptr(raw), 4, L.ptr(raw[:, 3:]), 4, L.ptr(t), L.ptr(batch["rays_d"]),
           B, S, 1, L.ACT_ARTIC, L.ptr(g_rgb), None, None, L.ptr(draw), L.ptr(draw[:, 3:]), 4,
           L.stream())
    G = [(torch.empty_like(w), torch.empty_like(b)) for w, b in P]
    dlat = tuple(torch.empty_like(x) for x in lat)
    train_art._backward_level_fused(geo, P, G, lat, dlat, xyz, enc, venc, S, hd, h, bot, hv, draw,
                                    masks, True)
    torch.cuda.synchronize()
    rm = [torch.stack([tiles.untile(x, R) for x in tt]).cpu() for tt in (hd, h, hv)]
    enc_c = train_art.enc_rows(geo, enc, R).cpu()
    kept = {"xyz": xyz.cpu(), "hd": list(rm[0]), "xp": enc_c[:, :3].clone(), "enc": enc_c,
            "h": list(rm[1]), "bot": tiles.untile(bot, R).cpu(), "hv": list(rm[2])}
    pre = "fine_mlp." if level else "coarse_mlp."
    sd = W.art_state_dict(0)

    def params64():
        return {k[len(pre):]: torch.from_numpy(v).double().requires_grad_(True)
                for k, v in sd.items() if k.startswith(pre)}

    # (ii) forward values
    rec = {}
    with torch.no_grad():
        samples = O.cast_rays(t.cpu().double(), batch["rays_o"].cpu().double(),
                              batch["rays_d"].cpu().double())
        rgb64, sig64 = O.art_mlp_forward(params64(), samples, venc.cpu().double(),
                                         {k: x.cpu().double() for k, x in zip(names, lat)},
                                         xp_fixed=kept["xp"], record=rec)
    fwd = [(f"hd{i}", kept["hd"][i], rec["hd"][i]) for i in range(4)] + [("enc", kept["enc"], rec["enc"])]
    fwd += [(f"h{i}", kept["h"][i], rec["h"][i]) for i in range(8)] + [("bot", kept["bot"], rec["bot"])]
    fwd += [(f"hv{i}", kept["hv"][i], rec["hv"][i]) for i in range(4)]
    fwd += [("raw_rgb", raw[:, :3].cpu(), rgb64.reshape(-1, 3)), ("raw_sigma", raw[:, 3].cpu(), sig64.reshape(-1))]
    e_fwd = {n: rel_err(a, b) for n, a, b in fwd}
    # (iii) d raw
    rr = torch.cat([rgb64.reshape(-1, 3), sig64.reshape(-1, 1)], -1).reshape(B, S, 4).requires_grad_(True)
    rgb_a, sig_a = O.art_activations(rr[..., :3], rr[..., 3:])
    c64 = O.volumetric_rendering(rgb_a, sig_a, t.cpu().double(), batch["rays_d"].cpu().double(), True)[0]
    O.img2mse(c64, batch["target"].cpu().double()).backward()
    d64 = rr.grad.reshape(-1, 4)
    e_drgb = rel_err(draw[:, :3].cpu(), d64[:, :3])
    e_dsig = rel_err(draw[:, 3].cpu(), d64[:, 3])
    # (i) backward at our values with our d raw
    p64 = params64()
    l64 = {k: x.cpu().double().requires_grad_(True) for k, x in zip(names, lat)}
    r_rgb, r_sig = O.art_mlp_forward_kept(p64, kept, venc.cpu(), l64, S)
    dd = draw.cpu().double()
    torch.autograd.backward([r_rgb, r_sig], [dd[:, :3], dd[:, 3:]])
    e_bwd = {}
    for (dw, db), name in zip(G, _ART_NAMES):
        e_bwd[f"{name}.weight"] = rel_err(dw.cpu(), p64[f"{name}.weight"].grad)
        e_bwd[f"{name}.bias"] = rel_err(db.cpu(), p64[f"{name}.bias"].grad)
    for got, k in zip(dlat, names):
        e_bwd[f"latent {k}"] = rel_err(got.cpu(), l64[k].grad.reshape(got.shape))
    wf = max(e_fwd, key=e_fwd.get)
    wb = max(e_bwd, key=e_bwd.get)
    print(f"C5 articulated level {level} (B={B}, S={S}), stage-isolated vs fp64: forward worst "
          f"{e_fwd[wf]:.2e} ({wf}); d raw rgb {e_drgb:.2e} sigma {e_dsig:.2e}; backward worst "
          f"{e_bwd[wb]:.2e} ({wb})")
    assert e_fwd[wf] <= 1e-5, (wf, e_fwd[wf])
    assert e_drgb <= 1e-5 and e_dsig <= 1e-4, (e_drgb, e_dsig)
    assert e_bwd[wb] <= 1e-4, (wb, e_bwd[wb])


def _make(seed=0, **numerics):
    """NeRF_AE_Art + code library with the oracle's seed weights; ``numerics``: TrainNumerics
    fields."""
    import types

    from aonerf.code_library import CodeLibraryArticulated
    from aonerf.model_autodecoder import NeRF_AE_Art
    from aonerf.numerics import TrainNumerics

    net = NeRF_AE_Art(train_numerics=TrainNumerics(**numerics)).cuda()
    net.load_state_dict({k: torch.from_numpy(v) for k, v in W.art_state_dict(seed).items()})
    lib = CodeLibraryArticulated(types.SimpleNamespace(N_max_objs=151, N_obj_code_length=128)).cuda()
    lib.load_state_dict({k: torch.from_numpy(v) for k, v in W.code_library_state_dict(seed).items()})
    return net, lib


def _batch(g):
    b = {k: cuda(g[k]) for k in ("rays_o", "rays_d", "viewdirs", "target")}
    b["instance_id"] = torch.tensor([int(g["instance_id"])], device="cuda")
    b["articulation_id"] = torch.tensor([int(g["articulation_id"])], device="cuda")
    return b


def _oracle_grads(g, dtype):
    params = [{k: v.to(dtype).requires_grad_(True) for k, v in p.items()}
              for p in O.split_state_dict(W.art_state_dict(0))]
    tables = {k: torch.from_numpy(v).to(dtype).requires_grad_(True)
              for k, v in W.code_library_state_dict(0).items()}
    rays = {k: torch.from_numpy(g[k]).to(dtype) for k in ("rays_o", "rays_d", "viewdirs")}
    loss, *_ = O.art_training_loss(params, tables, rays, torch.from_numpy(g["target"]).to(dtype),
                                   int(g["instance_id"]), int(g["articulation_id"]), True, True,
                                   2.0, 6.0, u_coarse=torch.from_numpy(g["u_coarse"]).to(dtype),
                                   u_fine=torch.from_numpy(g["u_fine"]).to(dtype))
    loss.backward()
    grads = {f"{lv}.{k}": v.grad.double().numpy() for lv, p in zip(("coarse_mlp", "fine_mlp"), params)
             for k, v in p.items()}
    grads.update({k: v.grad.double().numpy() for k, v in tables.items()})
    return grads


def _named_grad(net, lib, name, g):
    if name.startswith("embedding"):
        row = int(g["articulation_id"] if "articulation" in name else g["instance_id"])
        return dict(lib.named_parameters())[name].grad[row].cpu().numpy()
    return dict(net.named_parameters())[name].grad.cpu().numpy()


def test_art_train_step_golden(golden, art_fwd_mode):
    """Loss (incl. the latent regulariser) and the recorded gradients of one
    LitNeRF_AutoDecoder.training_step (randomized, injected uniforms) vs the reference."""
    from aonerf import train_art

    g = golden("art_train_step.npz")
    assert W.digest(W.art_state_dict(0)) == str(g["digest"])
    net, lib = _make(0, **art_fwd_mode)
    loss, logs = train_art.training_step(net, lib, _batch(g), True, True, 2.0, 6.0,
                                         u_coarse=cuda(g["u_coarse"]), u_fine=cuda(g["u_fine"]))
    loss.backward()
    torch.cuda.synchronize()
    print(f"loss gpu {loss.item():.8f} ref {float(g['loss']):.8f}")
    np.testing.assert_allclose(loss.item(), g["loss"], rtol=1e-5)
    np.testing.assert_allclose(logs["reg"].item(), g["reg"], rtol=1e-5)
    np.testing.assert_allclose(logs["psnr0"].item(), g["psnr0"], rtol=1e-5)
    g64 = _oracle_grads(g, torch.float64)
    worst = 0.0
    for key in g:
        if not key.startswith("grad::"):
            continue
        name = key[6:]
        ref = g[key]
        ref64 = g64[name]
        if name.startswith("embedding"):
            ref64 = ref64[int(g["articulation_id"] if "articulation" in name else g["instance_id"])]
        env = rel_err(ref, ref64)
        e = rel_err(_named_grad(net, lib, name, g), ref)
        print(f"  {name:45s} ours {e:.2e}  reference fp32-vs-fp64 envelope {env:.2e}")
        worst = max(worst, e / max(4 * env, 1e-4))
        assert e <= max(4 * env, 1e-4), (key, e, env)
    # the code library's untouched rows get exactly zero gradient
    for name, p in lib.named_parameters():
        row = int(g["articulation_id"] if "articulation" in name else g["instance_id"])
        gr = p.grad.clone()
        gr[row] = 0
        assert not gr.any(), name
    print(f"articulated train-step grads vs reference: worst error / allowance {worst:.2f}")


@pytest.mark.parametrize("loss_scale", [1.0, 1.0 / 64], ids=["64rays", "grad_mag_4096rays"])
def test_art_train_step_chain(golden, art_fwd_mode, loss_scale):
    """Teacher-forced: our level-l sample positions through the oracle's autograd; gradients of
    every MLP parameter and of the three latent codes against the fp32 oracle (the reference's
    arithmetic), each within max(2 x its own distance from the fp64 oracle, 1e-3) of the
    tensor's max.  ``loss_scale``
    1/64 gives the per-row gradient magnitudes of a 4096-ray batch (the mean over 64x more
    rays)."""
    from aonerf import train_art

    g = golden("art_train_step.npz")
    net, lib = _make(0, **art_fwd_mode)
    batch = _batch(g)
    latents = lib(batch)
    ret = net(batch, True, True, 2.0, 6.0, latents, u_coarse=cuda(g["u_coarse"]),
              u_fine=cuda(g["u_fine"]), return_intermediates=True)
    target = batch["target"]
    loss = (train_art.img2mse(ret[1][0], target) + train_art.img2mse(ret[0][0], target)) * loss_scale
    for x in latents.values():
        x.retain_grad()
    loss.backward()
    # the oracle at our sample positions, in fp32 and in fp64: the deformation gradients pass
    # through pos_enc's sin(2^9 x') (model_autodecoder.py:205-212), so a 1e-7 relative change
    # of x' moves them by ~1e-3 -- the reference's own fp32 evaluation is that far from fp64
    ref = {}
    for dtype in (torch.float32, torch.float64):
        rays = {k: torch.from_numpy(g[k]).to(dtype) for k in ("rays_o", "rays_d", "viewdirs")}
        params = [{k: v.to(dtype).requires_grad_(True) for k, v in p.items()}
                  for p in O.split_state_dict(W.art_state_dict(0))]
        lat = {k: v.detach().cpu().to(dtype).requires_grad_(True) for k, v in latents.items()}
        tgt = torch.from_numpy(g["target"]).to(dtype)
        ref_loss = 0.0
        for level in range(2):
            t = ret[level][3]["t_vals"].cpu().to(dtype)
            comp, acc, w, depth = O.art_render_level(params, rays, t, level, True, lat)
            ref_loss = ref_loss + O.img2mse(comp, tgt)
            np.testing.assert_allclose(ret[level][0].detach().cpu().numpy(), comp.detach().numpy(),
                                       rtol=0, atol=1e-5)
        (ref_loss * loss_scale).backward()
        ref[dtype] = {f"{pre}{n}": v.grad.double().numpy() for lv, pre in ((0, "coarse_mlp."), (1, "fine_mlp."))
                      for n, v in params[lv].items()}
        ref[dtype].update({f"latent {k}": v.grad.double().numpy() for k, v in lat.items()})
    ours = {n: p.grad.cpu().numpy() for n, p in net.named_parameters()}
    ours.update({f"latent {k}": v.grad.cpu().numpy() for k, v in latents.items()})
    worst = 0.0
    for name, want in ref[torch.float32].items():
        env = rel_err(want, ref[torch.float64][name])
        e = rel_err(ours[name], want)
        allow = max(2 * env, 1e-3)
        if e > 1e-4 or name.startswith("latent"):
            print(f"  {name:45s} ours {e:.2e}  oracle fp32-vs-fp64 {env:.2e}")
        worst = max(worst, e / allow)
        assert e <= allow, (name, e, env)
    print(f"articulated teacher-forced grads vs fp32 oracle: worst error / allowance {worst:.2f}")


def test_art_adam_all_tensors(golden):
    """configure_optimizers (model_autodecoder.py:599-601): one Adam over the 80 MLP tensors and
    the 3 embedding tables (two aon_adam_step launches) matches torch.optim.Adam."""
    from aonerf import train_art

    g = golden("art_train_step.npz")
    net, lib = _make(0)
    ref_net, ref_lib = _make(0)
    opt = train_art.configure_optimizers(net, lib)
    ref_opt = torch.optim.Adam(list(ref_net.parameters()) + list(ref_lib.parameters()), lr=5e-4,
                               betas=(0.9, 0.999))  # foreach: as on a GPU (test_gpu_train)
    assert len(opt.params) == 83
    kw = dict(u_coarse=cuda(g["u_coarse"]), u_fine=cuda(g["u_fine"]))
    loss, _ = train_art.training_step(net, lib, _batch(g), True, True, 2.0, 6.0, **kw)
    loss.backward()
    for p, q in zip(list(net.parameters()) + list(lib.parameters()),
                    list(ref_net.parameters()) + list(ref_lib.parameters())):
        q.grad = p.grad.clone()
    lr = train_art.learning_rate(1, 1000)
    opt.step(lr=lr)
    for pg in ref_opt.param_groups:
        pg["lr"] = lr
    ref_opt.step()
    for (name, p), q in zip(list(net.named_parameters()) + list(lib.named_parameters()),
                            list(ref_net.parameters()) + list(ref_lib.parameters())):
        d = (p.detach() - q.detach()).abs().max().item()
        assert d <= 1e-6, (name, d)


def test_art_train_step_c5_4096_rays():
    """Config C5 on the articulated auto-decoder at its stated size: one training step on a
    4096-ray batch.  Loss against the oracle on our sample positions (rtol 1e-5) and end to end
    (rtol 1e-4), and every MLP parameter's and latent code's gradient against the oracle on our
    sample positions, twice:

    (A) x'- and mask-forced: the fp64 oracle with pos_enc evaluated at OUR deformed points x'
        (oracle.pos_enc_at; gradients straight through to its own deformation MLP) and with OUR
        ReLU' pattern (oracle.art_mlp_forward_kept on its own fp64 forward values, the units whose
        sign differs from ours set to our side of zero), its own fp64 compositor and loss: every
        parameter's and latent's gradient within 1e-4 of its max.  Forcing x' alone is not enough:
        tools/diag/art_c5_forward_attr.py (profiles/r04/art_attr.log) shows the x'-forced distance
        (~1e-3) is carried entirely by ReLU' flips -- ours 20 / 98 / 35 units of hd / h / hv on
        the fine level, the fp32 oracle's 30 / 137 / 41 -- each a discrete event that the step's
        ill-conditioning (dL/dx' sums 60 terms of up to 2^9 |d enc|) turns into ~1e-3 of a
        deformation gradient, so one evaluation lands 20x closer than another of equal accuracy
        (the fp32 oracle: 7.7e-5 on a fine deformation tensor where ours is 2e-3, 8.6e-3 on a
        coarse one where ours is 1.3e-3; verdict r03's "6x" was one such draw).  With the pattern
        shared the distance drops to <= 2.7e-7 (diagnostic), the backward kernels' own 3.5e-6
        (test_art_c5_level_stage_isolated) on top.  And the flips themselves are gated: ours at
        most max(2 x the fp32 oracle's count, 16) per group and level;
    (B) free-running against the fp32 oracle (the reference's arithmetic): per tensor within
        max(2 x env, 1e-3) of its max, env = the oracle's own fp32-vs-fp64 distance on that
        tensor -- or ATTRIBUTED: the gradients see sin(2^9 x') (model_autodecoder.py:205-212)
        and move chaotically with the last bits of x', so a tensor outside that allowance must
        show (A) within its gate and our x' at most 1.5x as far from the fp64 x' as the fp32
        oracle's (r, measured per level, printed).  An unattributed tensor fails.
    test_art_backward_stage_isolated pins the backward kernels themselves at ~1e-5."""
    from aonerf import train_art
    from test_gpu_train import c5_batch

    net, lib = _make(0)
    batch, u_c, u_f = c5_batch(seed=12)
    batch["instance_id"] = torch.tensor([7], device="cuda")
    batch["articulation_id"] = torch.tensor([3], device="cuda")
    latents = lib(batch)
    ret = net(batch, True, True, 2.0, 6.0, latents, u_coarse=u_c, u_fine=u_f,
              return_intermediates=True)
    target = batch["target"]
    loss = train_art.img2mse(ret[1][0], target) + train_art.img2mse(ret[0][0], target)
    for x in latents.values():
        x.retain_grad()
    loss.backward()
    torch.cuda.synchronize()
    lat_dev = {k: v.detach().cpu() for k, v in latents.items()}
    # our x' per level: the fused forward at the level's t (deterministic: the values the
    # autograd forward saw)
    from aonerf import tiles

    xp_ours, relu_ours = [], []
    with torch.no_grad():
        lat_t = tuple(L_contig(latents[k]) for k in ("density", "color", "articulation"))
        for level, mlp in enumerate((net.coarse_mlp, net.fine_mlp)):
            t = ret[level][3]["t_vals"].contiguous()
            R = t.numel()
            P = [(m.weight.detach(), m.bias.detach()) for m in train_art.art_layers(mlp)]
            raw = torch.empty((R, 4), device="cuda")
            _, hd, enc, h, _, hv = train_art._forward_level_fused(
                train_art._Geo(mlp), P, lat_t, batch["rays_o"], batch["rays_d"], batch["viewdirs"],
                t, raw)
            xp_ours.append(tiles.untile(enc, R)[:, :3].cpu())
            # the ReLU' pattern our forward fed the backward: the sign of each kept activation
            relu_ours.append({grp: [tiles.untile(x, R).cpu() > 0 for x in tt]
                              for grp, tt in (("hd", hd), ("h", h), ("hv", hv))})
            del hd, enc, h, hv
        rays = {k: batch[k].cpu() for k in ("rays_o", "rays_d", "viewdirs")}
        params = O.split_state_dict(W.art_state_dict(0))
        e2e = O.art_nerf_forward(params, rays, True, True, 2.0, 6.0, lat_dev, u_coarse=u_c.cpu(),
                                 u_fine=u_f.cpu())
        tgt = target.cpu()
        ref_e2e = (O.img2mse(e2e[1][0], tgt) + O.img2mse(e2e[0][0], tgt)).item()
    ref, ref_loss, xps = {}, None, {}
    for mode, dtype in (("fp32", torch.float32), ("fp64", torch.float64), ("forced", torch.float64)):
        rays = {k: batch[k].cpu().to(dtype) for k in ("rays_o", "rays_d", "viewdirs")}
        params = [{k: v.to(dtype).requires_grad_(True) for k, v in p.items()}
                  for p in O.split_state_dict(W.art_state_dict(0))]
        lat = {k: v.detach().clone().to(dtype).requires_grad_(True) for k, v in lat_dev.items()}
        tgt = target.cpu().to(dtype)
        lv_loss = 0.0
        for level in range(2):
            t = ret[level][3]["t_vals"].cpu().to(dtype)
            out = O.art_render_level(params, rays, t, level, True, lat, return_xp=True,
                                     xp_fixed=xp_ours[level] if mode.startswith("forced") else None)
            xps[(mode, level)] = out[4].detach().double()
            lv_loss = lv_loss + O.img2mse(out[0], tgt)
        lv_loss.backward()
        if mode == "fp32":
            ref_loss = lv_loss.item()
        ref[mode] = {f"{pre}{n}": v.grad.double().numpy()
                     for lv, pre in ((0, "coarse_mlp."), (1, "fine_mlp.")) for n, v in params[lv].items()}
        ref[mode].update({f"latent {k}": v.grad.double().numpy() for k, v in lat.items()})
        del params, lv_loss
    print(f"C5 art loss gpu {loss.item():.8f}  oracle on our t {ref_loss:.8f}  "
          f"oracle end to end {ref_e2e:.8f}")
    np.testing.assert_allclose(loss.item(), ref_loss, rtol=1e-5)
    np.testing.assert_allclose(loss.item(), ref_e2e, rtol=1e-4)
    ours = {n: p.grad.cpu().numpy() for n, p in net.named_parameters()}
    ours.update({f"latent {k}": v.grad.cpu().numpy() for k, v in latents.items()})
    # x' rounding: ours and the fp32 oracle's, against the fp64 oracle's, per level
    rms = lambda a: float(a.pow(2).mean().sqrt())  # noqa: E731
    ratio = {}
    for level, pre in ((0, "coarse_mlp."), (1, "fine_mlp.")):
        x64 = xps[("fp64", level)]
        e_ours = rms(xp_ours[level].double() - x64)
        e_32 = rms(xps[("fp32", level)] - x64)
        ratio[pre] = e_ours / e_32
        print(f"  level {level}: x' rms error vs fp64  ours {e_ours:.2e}  fp32 oracle {e_32:.2e}  "
              f"r = {e_ours / e_32:.2f}")
    ratio["latent"] = max(ratio.values())
    # (A) the fp64 oracle forced to our x' AND our ReLU' pattern (values its own): the forced fp64
    # forward's kept values, each hidden activation whose sign differs from ours replaced by ours
    # (oracle.art_mlp_forward_kept: ReLU' from the sign), its fp64 backward through its own
    # compositor and loss.  Mask flips are discrete events of the forward's last bits (counted
    # below, ours against the fp32 oracle's); with the pattern shared, what is left is the
    # continuous part, which the step does not amplify.
    names3 = ("density", "color", "articulation")
    l64 = {k: lat_dev[k].double().requires_grad_(True) for k in names3}
    p64 = [{k: v.double().requires_grad_(True) for k, v in p.items()}
           for p in O.split_state_dict(W.art_state_dict(0))]
    o64, d64, v64 = (batch[k].cpu().double() for k in ("rays_o", "rays_d", "viewdirs"))
    venc64 = O.pos_enc(v64, 0, 4)
    loss_m = 0.0
    flips = {}
    for level in range(2):
        t64 = ret[level][3]["t_vals"].cpu().double()
        B_, S_ = t64.shape
        recs = {}
        with torch.no_grad():
            for tag, dt in (("64", torch.float64), ("32", torch.float32)):
                rec = {}
                O.art_mlp_forward({k: v.detach().to(dt) for k, v in p64[level].items()},
                                  O.cast_rays(t64.to(dt), o64.to(dt), d64.to(dt)), venc64.to(dt),
                                  {k: v.detach().to(dt) for k, v in l64.items()},
                                  xp_fixed=xp_ours[level], record=rec)
                recs[tag] = rec
        r64 = recs["64"]
        kept = {"xyz": r64["xyz"], "xp": xp_ours[level], "enc": r64["enc"], "bot": r64["bot"]}
        for grp in ("hd", "h", "hv"):
            # a flipped unit takes 1e-30 (ours > 0: fp64 had it at 0, ~1e-7 from the edge) or 0
            kept[grp] = [torch.where(m == (v > 0), v, torch.where(m, torch.full_like(v, 1e-30),
                                                                 torch.zeros_like(v)))
                         for m, v in zip(relu_ours[level][grp], r64[grp])]
            flips[(level, grp)] = (
                sum(int((m != (v > 0)).sum()) for m, v in zip(relu_ours[level][grp], r64[grp])),
                sum(int(((a > 0) != (v > 0)).sum()) for a, v in zip(recs["32"][grp], r64[grp])))
        del recs
        r_rgb, r_sig = O.art_mlp_forward_kept(p64[level], kept, venc64, l64, S_)
        rgb_a, sig_a = O.art_activations(r_rgb.reshape(B_, S_, 3), r_sig.reshape(B_, S_, 1))
        comp = O.volumetric_rendering(rgb_a, sig_a, t64, d64, True)[0]
        loss_m = loss_m + O.img2mse(comp, target.cpu().double())
        del kept, r_rgb, r_sig
    loss_m.backward()
    ref["masked"] = {f"{pre}{n}": v.grad.double().numpy()
                     for lv, pre in ((0, "coarse_mlp."), (1, "fine_mlp.")) for n, v in p64[lv].items()}
    ref["masked"].update({f"latent {k}": v.grad.double().numpy() for k, v in l64.items()})
    bad_flips = []
    for (level, grp), (fo, f32) in sorted(flips.items()):
        print(f"  level {level} {grp}: ReLU' flips against the forced fp64 forward: ours {fo}, fp32 "
              f"oracle {f32}")
        if fo > max(2 * f32, 16):
            bad_flips.append((level, grp, fo, f32))
    worst_a = worst_b = 0.0
    bad_a, unexplained, attributed = [], [], []
    for name, want in ref["fp32"].items():
        ea = rel_err(ours[name], ref["masked"][name])
        lottery = rel_err(ours[name], ref["forced"][name])
        env = rel_err(want, ref["fp64"][name])
        r = next(v for pre, v in ratio.items() if name.startswith(pre))
        e = rel_err(ours[name], want)
        allow = max(2 * env, 1e-3)
        worst_a = max(worst_a, ea / 1e-4)
        worst_b = max(worst_b, e / allow)
        ok_a = ea <= 1e-4
        if not ok_a:
            bad_a.append((name, ea))
        if e > allow:
            (attributed if ok_a and r <= 1.5 else unexplained).append(name)
        if e > 1e-4 or ea > 1e-5 or not ok_a:
            print(f"  {name:45s} (A) mask-forced {ea:.2e}, unforced {lottery:.2e}  (B) ours {e:.2e}"
                  f"  oracle fp32-vs-fp64 {env:.2e}"
                  f"{'  ATTRIBUTED' if name in attributed else ''}")
    print(f"C5 art grads (4096 rays): (A) x'- and mask-forced worst error / 1e-4 {worst_a:.2f}; (B) "
          f"free-running worst error / allowance {worst_b:.2f}, {len(attributed)} tensor(s) "
          f"outside it attributed to x' rounding")
    assert not bad_flips, bad_flips
    assert not bad_a, bad_a
    assert not unexplained, unexplained


def L_contig(x):
    return x.detach().reshape(1, -1).contiguous()


def test_two_art_precisions_in_one_process():
    """Verdict r05 #5: an f16x3 and a bf16 (default fp16-activation forward) articulated model
    train in one process, interleaved, each bit-equal to its solo run."""
    from aonerf import train_art
    from test_gpu_train import _step_state, c5_batch

    batch, u_c, u_f = c5_batch(n=256, seed=6)
    batch["instance_id"] = torch.tensor([7], device="cuda")
    batch["articulation_id"] = torch.tensor([3], device="cuda")
    solo = {}
    for prec in ("f16x3", "bf16"):
        net, lib = _make(0, precision=prec)
        opt = train_art.configure_optimizers(net, lib)
        solo[prec] = _step_state(net, opt, train_art, batch, u_c, u_f, lib)
    (na, la_), (nb, lb_) = _make(0, precision="f16x3"), _make(0, precision="bf16")
    oa, ob = train_art.configure_optimizers(na, la_), train_art.configure_optimizers(nb, lb_)
    oa.zero_grad()
    ob.zero_grad()
    xa, _ = train_art.training_step(na, la_, batch, True, True, 2.0, 6.0, u_coarse=u_c, u_fine=u_f)
    xb, _ = train_art.training_step(nb, lb_, batch, True, True, 2.0, 6.0, u_coarse=u_c, u_fine=u_f)
    (xa + xb).backward()
    got = {}
    for prec, net, lib, loss in (("f16x3", na, la_, xa), ("bf16", nb, lb_, xb)):
        ps = list(net.parameters()) + list(lib.parameters())
        got[prec] = (loss.detach().cpu(), [p.grad.detach().cpu().clone() for p in ps])
    ob.step()
    oa.step()
    for prec, net, lib in (("f16x3", na, la_), ("bf16", nb, lb_)):
        loss, grads, params = solo[prec]
        assert torch.equal(loss, got[prec][0])
        assert all(torch.equal(x, y) for x, y in zip(grads, got[prec][1]))
        ps = list(net.parameters()) + list(lib.parameters())
        assert all(torch.equal(x, p.detach().cpu()) for x, p in zip(params, ps))
