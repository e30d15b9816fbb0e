"""Where the articulated C5 step's x'-forced gradient distance comes from (verdict r03 #2,
tests/test_gpu_art_train.py::test_art_train_step_c5_4096_rays (A)).

Per level: the fp64 backward (oracle.art_mlp_forward_kept: autograd through fp64 linear maps
with every intermediate VALUE forced) at several sets of forward values, all at our x':
  K64   the fp64 forward's own values            -> the (A) reference gradients
  K32   the fp32 oracle's forward values         -> the reference arithmetic's distance
  Kours our fused f16x3 forward's kept values    -> our distance (the backward kernels themselves
                                                    add <= 3.5e-6: test_art_c5_level_stage_isolated)
  hybrids: K64 with ONE group (hd / h / bot / hv) replaced by ours -> which forward values
           carry the distance.
Also the forward distances themselves (rms / max of each group vs K64, ours and fp32).
Prints one table per level.  GPU + CPU oracle; ~1-2 min.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "articulated-object-nerf_amd"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import nerf_oracle as O  # noqa: E402
from oracle import weights as W  # noqa: E402


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def rms_rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.sqrt(((a - b) ** 2).mean()) / max(np.abs(b).max(), 1e-30))


def main():
    from aonerf import tiles, train_art
    from test_gpu_art_train import _make
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
    names = ("density", "color", "articulation")
    lat = tuple(latents[k].reshape(1, -1).contiguous() for k in names)
    venc = torch.empty((batch["rays_o"].shape[0], 27), device="cuda")
    L.call("aon_pos_enc", L.ptr(batch["viewdirs"]), venc.shape[0], 0, 4, L.ptr(venc), L.stream())
    tgt64 = batch["target"].cpu().double()
    sd = W.art_state_dict(0)
    levels = [int(x) for x in os.environ.get("ATTR_LEVELS", "0,1").split(",")]
    for level in levels:
        t = ret[level][3]["t_vals"].contiguous()
        B, S = t.shape
        R = B * S
        mlp = net.fine_mlp if level else net.coarse_mlp
        geo = train_art._Geo(mlp)
        P = [(m.weight.detach(), m.bias.detach()) for m in train_art.art_layers(mlp)]
        raw = torch.empty((R, 4), device="cuda")
        with torch.no_grad():
            xyz, hd, enc, h, bot, hv = train_art._forward_level_fused(
                geo, P, lat, batch["rays_o"], batch["rays_d"], batch["viewdirs"], t, raw)
        torch.cuda.synchronize()
        rm = [torch.stack([tiles.untile(x, R) for x in tt]).cpu() for tt in (hd, h, hv)]
        enc_c = train_art.enc_rows(geo, enc, R).cpu()
        ours = {"xyz": xyz.cpu().double(), "hd": [x.double() for x in rm[0]],
                "xp": enc_c[:, :3].clone(), "enc": enc_c.double(),
                "h": [x.double() for x in rm[1]], "bot": tiles.untile(bot, R).cpu().double(),
                "hv": [x.double() for x in rm[2]]}
        pre = "fine_mlp." if level else "coarse_mlp."

        def params(dt, grad=False):
            return {k[len(pre):]: torch.from_numpy(v).to(dt).requires_grad_(grad)
                    for k, v in sd.items() if k.startswith(pre)}

        t64 = t.cpu().double()
        o64, d64 = batch["rays_o"].cpu().double(), batch["rays_d"].cpu().double()
        kept = {}
        raws = {}
        for tag, dt in (("K64", torch.float64), ("K32", torch.float32)):
            rec = {}
            with torch.no_grad():
                samples = O.cast_rays(t.cpu().to(dt), batch["rays_o"].cpu().to(dt),
                                      batch["rays_d"].cpu().to(dt))
                rgb, sig = O.art_mlp_forward(params(dt), samples, venc.cpu().to(dt),
                                             {k: x.cpu().to(dt) for k, x in zip(names, lat)},
                                             xp_fixed=ours["xp"], record=rec)
            kept[tag] = {"xyz": ours["xyz"], "hd": [x.double() for x in rec["hd"]],
                         "xp": ours["xp"], "enc": rec["enc"].double(),
                         "h": [x.double() for x in rec["h"]], "bot": rec["bot"].double(),
                         "hv": [x.double() for x in rec["hv"]]}
            raws[tag] = (rgb.reshape(-1, 3).double(), sig.reshape(-1).double())
        kept["Kours"] = ours
        raws["Kours"] = (raw[:, :3].cpu().double(), raw[:, 3].cpu().double())
        print(f"== level {level} ({'fine' if level else 'coarse'}, {R} samples): forward values "
              f"vs K64 (max rel / rms rel)")
        for g in ("hd", "enc", "h", "bot", "hv", "raw_rgb", "raw_sigma"):
            line = f"   {g:9s}"
            for tag in ("Kours", "K32"):
                if g.startswith("raw"):
                    a, b = raws[tag][0 if g == "raw_rgb" else 1], raws["K64"][0 if g == "raw_rgb" else 1]
                else:
                    a, b = kept[tag][g], kept["K64"][g]
                    if isinstance(a, list):
                        a, b = torch.stack(a), torch.stack(b)
                line += f"  {tag} {rel(a, b):.2e} / {rms_rel(a, b):.2e}"
            print(line)

        def grads_at(k):
            p = params(torch.float64, True)
            lt = {kk: x.cpu().double().requires_grad_(True) for kk, x in zip(names, lat)}
            rgb_raw, sig_raw = O.art_mlp_forward_kept(p, k, venc.cpu().double(), lt, S)
            rgb, sig = O.art_activations(rgb_raw.reshape(B, S, 3), sig_raw.reshape(B, S, 1))
            comp = O.volumetric_rendering(rgb, sig, t64, d64, True)[0]
            loss = O.img2mse(comp, tgt64)
            loss.backward()
            out = {n: v.grad.numpy() for n, v in p.items()}
            out.update({f"latent {n}": v.grad.numpy() for n, v in lt.items()})
            return out

        def with_masks(src):
            # K64's values, but the ReLU' mask (the sign of the kept activation) of `src`: where
            # the two disagree take src's value (one side of zero exactly when the other is not)
            v = dict(kept["K64"])
            for g in ("hd", "h", "hv"):
                v[g] = [torch.where((a > 0) == (b > 0), b, a) for a, b in zip(kept[src][g], kept["K64"][g])]
            return v

        for src in ("Kours", "K32"):
            flips = {g: sum(int(((a > 0) != (b > 0)).sum()) for a, b in zip(kept[src][g], kept["K64"][g]))
                     for g in ("hd", "h", "hv")}
            print(f"   ReLU' flips vs K64, {src}: {flips}")
        variants = {"K64": kept["K64"], "K32": kept["K32"], "Kours": kept["Kours"],
                    "K64.masks_ours": with_masks("Kours"), "K64.masks_32": with_masks("K32")}
        for g in os.environ.get("ATTR_GROUPS", "hd,h,hv").split(","):
            if not g:
                continue
            v = dict(kept["K64"])
            v[g] = kept["Kours"][g]
            variants[f"K64+ours.{g}"] = v
        G = {}
        for tag, k in variants.items():
            G[tag] = grads_at(k)
            print(f"   (backward at {tag} done)", flush=True)
        ref = G["K64"]
        G["Kours-vs-K64.masks_ours"] = G["Kours"]
        tags = [t_ for t_ in G if t_ != "K64"]
        print(f"   gradient distance from the fp64 backward at K64 (max rel of each tensor):")
        print("   " + f"{'tensor':38s}" + "".join(f"{t_[-16:]:>17s}" for t_ in tags))
        worst = {t_: 0.0 for t_ in tags}
        for n in ref:
            row = [rel(G[t_][n], G["K64.masks_ours"][n] if t_ == "Kours-vs-K64.masks_ours" else ref[n])
                   for t_ in tags]
            for t_, e in zip(tags, row):
                worst[t_] = max(worst[t_], e)
            if n.startswith("deformation") or n.startswith("pts_linears.0") or n.startswith("pts_linears.1"):
                print("   " + f"{n:38s}" + "".join(f"{e:17.2e}" for e in row))
        print("   " + f"{'worst':38s}" + "".join(f"{worst[t_]:17.2e}" for t_ in tags))


if __name__ == "__main__":
    main()
