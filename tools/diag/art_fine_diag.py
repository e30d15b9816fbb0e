"""Diagnostic (GPU): where the articulated fine level's x'-forced gradient differences come from.
On C5's batch (tests/test_gpu_train.c5_batch, seed 12) at the fine level's sample positions:
  (i)   the backward kernels on our own kept tensors with the REAL d raw (compositing backward of
        the C5 loss) vs the fp64 oracle backward at those values (oracle.art_mlp_forward_kept);
  (ii)  our kept forward values (hd, enc, h, bot, hv, raw) vs the fp64 forward at our x';
  (iii) our d raw vs the fp64 oracle's d raw at our x'.
Prints max-relative errors per tensor."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "articulated-object-nerf_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import nerf_oracle as O  # noqa: E402
from oracle import weights as W  # noqa: E402


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def main():
    from test_gpu_art_train import _ART_NAMES, _make
    from test_gpu_train import c5_batch

    from aonerf import tiles, train_art
    L = train_art.L
    torch.set_num_threads(16)
    level = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    net, lib = _make(0)
    batch, u_c, u_f = c5_batch(seed=12)
    batch["instance_id"] = torch.tensor([7], device="cuda")
    batch["articulation_id"] = torch.tensor([3], device="cuda")
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
    lat = tuple(latents[k].detach().reshape(1, -1).contiguous() for k in ("density", "color", "articulation"))
    raw = torch.empty((R, 4), device="cuda")
    masks = torch.empty((16, tiles.rows(R), 8), dtype=torch.int32, device="cuda")
    xyz, hd, enc, h, bot, hv = train_art._forward_level_fused(geo, P, lat, batch["rays_o"], batch["rays_d"],
                                                              batch["viewdirs"], t, raw, None, masks)
    venc = torch.empty((B, 27), device="cuda")
    L.call("aon_pos_enc", L.ptr(batch["viewdirs"]), B, 0, 4, L.ptr(venc), L.stream())
    # our compositing + loss gradient: d comp = 2 (comp - target) / (3 B)
    comp = torch.empty((B, 3), device="cuda")
    acc = torch.empty((B,), device="cuda")
    wts = torch.empty((B, S), device="cuda")
    depth = torch.empty((B,), device="cuda")
    L.call("aon_composite_fwd", L.ptr(raw), 4, L.ptr(raw[:, 3:]), 4, L.ptr(t), L.ptr(batch["rays_d"]),
           B, S, 1, L.ACT_ARTIC, L.ptr(comp), L.ptr(acc), L.ptr(wts), L.ptr(depth), L.stream())
    g_rgb = (2.0 * (comp - batch["target"]) / (3 * B)).contiguous()
    draw = torch.empty((R, 4), device="cuda")
    L.call("aon_composite_bwd", L.ptr(raw), 4, L.ptr(raw[:, 3:]), 4, L.ptr(t), L.ptr(batch["rays_d"]),
           B, S, 1, L.ACT_ARTIC, L.ptr(g_rgb), None, None, L.ptr(draw), L.ptr(draw[:, 3:]), 4, L.stream())
    G = [(torch.empty_like(w), torch.empty_like(b)) for w, b in P]
    dlat = tuple(torch.empty_like(x) for x in lat)
    train_art._backward_level_fused(geo, P, G, lat, dlat, xyz, enc, venc, S, hd, h, bot, hv, draw,
                                    masks, True)
    torch.cuda.synchronize()
    rm = [torch.stack([tiles.untile(x, R) for x in tt]).cpu() for tt in (hd, h, hv)]
    bot_rm = tiles.untile(bot, R).cpu()
    enc_c = train_art.enc_rows(geo, enc, R).cpu()
    kept = {"xyz": xyz.cpu(), "hd": list(rm[0]), "xp": enc_c[:, :3].clone(), "enc": enc_c,
            "h": list(rm[1]), "bot": bot_rm, "hv": list(rm[2])}
    pre = "fine_mlp." if level else "coarse_mlp."
    sd = W.art_state_dict(0)
    names = ("density", "color", "articulation")

    def params64():
        return {k[len(pre):]: torch.from_numpy(v).double().requires_grad_(True)
                for k, v in sd.items() if k.startswith(pre)}

    # (i) stage-isolated with the real d raw
    p64 = params64()
    l64 = {k: x.cpu().double().requires_grad_(True) for k, x in zip(names, lat)}
    r_rgb, r_sig = O.art_mlp_forward_kept(p64, kept, venc.cpu(), l64, S)
    d64 = draw.cpu().double()
    torch.autograd.backward([r_rgb, r_sig], [d64[:, :3], d64[:, 3:]])
    dr = draw.cpu().abs()
    print(f"level {level}: d raw |max| {dr.max():.3e}, median {dr.median():.3e}, "
          f"fraction below max*1e-6 {(dr < dr.max() * 1e-6).float().mean():.3f}")
    worst = []
    for (dw, db), name in zip(G, _ART_NAMES):
        for got, key in ((dw, f"{name}.weight"), (db, f"{name}.bias")):
            worst.append((rel(got.cpu(), p64[key].grad), key))
    for got, k in zip(dlat, names):
        worst.append((rel(got.cpu(), l64[k].grad.reshape(got.shape)), "latent " + k))
    worst.sort(reverse=True)
    print("(i) stage-isolated, real d raw: worst", [(f"{e:.2e}", k) for e, k in worst[:6]])
    # (ii) forward values vs fp64 at our x'
    p64 = params64()
    lat64 = {k: x.cpu().double() for k, x in zip(names, lat)}
    rec = {}
    with torch.no_grad():
        samples = O.cast_rays(t.cpu().double(), batch["rays_o"].cpu().double(), batch["rays_d"].cpu().double())
        rgb64, sig64 = O.art_mlp_forward(p64, samples, venc.cpu().double(), lat64, xp_fixed=kept["xp"],
                                         record=rec)
    print("(ii) forward vs fp64 at our x':",
          {"hd%d" % i: f"{rel(kept['hd'][i], rec['hd'][i]):.1e}" for i in range(4)},
          {"enc": f"{rel(kept['enc'], rec['enc']):.1e}"},
          {"h%d" % i: f"{rel(kept['h'][i], rec['h'][i]):.1e}" for i in range(8)},
          {"bot": f"{rel(kept['bot'], rec['bot']):.1e}"},
          {"hv%d" % i: f"{rel(kept['hv'][i], rec['hv'][i]):.1e}" for i in range(4)},
          {"raw_rgb": f"{rel(raw[:, :3].cpu(), rgb64.reshape(-1, 3)):.1e}",
           "raw_sigma": f"{rel(raw[:, 3].cpu(), sig64.reshape(-1)):.1e}"})
    # (iii) d raw vs fp64 composite backward on the fp64 raw
    rr = torch.cat([rgb64.reshape(-1, 3), sig64.reshape(-1, 1)], -1).reshape(B, S, 4).requires_grad_(True)
    rgbA, sigA = O.art_activations(rr[..., :3], rr[..., 3:])
    c, a, w, dd = O.volumetric_rendering(rgbA, sigA, t.cpu().double(), batch["rays_d"].cpu().double(), True)
    loss = O.img2mse(c, batch["target"].cpu().double())
    loss.backward()
    print(f"(iii) d raw vs fp64: rgb {rel(draw[:, :3].cpu(), rr.grad.reshape(-1, 4)[:, :3]):.2e}  "
          f"sigma {rel(draw[:, 3].cpu(), rr.grad.reshape(-1, 4)[:, 3]):.2e}")


if __name__ == "__main__":
    main()
