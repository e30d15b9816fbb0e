"""Diagnostic (GPU): the articulated bf16 training mode's gradient error, by source.
On C5's batch (tests/test_gpu_train.c5_batch, seed 12, 4,096 rays), for each forward numerics
(art_forward "bf16_trunk": trunk / heads / view branch bf16; "f16x3": fp16x3 forward, bf16 stores):
  (i)  the whole step's gradients vs the fp32 oracle at our t (worst max-rel and cosine per
       group: deformation, trunk, heads + view, latents);
  (ii) the bf16 backward (chain + dW GEMMs) stage-isolated: the fp64 oracle's autograd forced to
       OUR kept forward values (oracle.art_mlp_forward_kept) with OUR d raw, per level;
  (iii) step time (ms) of train_art.training_step + backward at C5 size.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "articulated-object-nerf_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import nerf_oracle as O  # noqa: E402
from oracle import weights as W  # noqa: E402


def stats(got, want):
    got, want = np.asarray(got, np.float64).reshape(-1), np.asarray(want, np.float64).reshape(-1)
    e = float(np.abs(got - want).max() / max(np.abs(want).max(), 1e-30))
    c = float(got @ want / (np.linalg.norm(got) * np.linalg.norm(want) + 1e-300))
    return e, c


def group(name):
    if "deformation" in name:
        return "deformation"
    if "pts_linears" in name:
        return "trunk"
    if name.startswith("latent"):
        return "latent"
    return "heads+view"


def report(tag, ours, want):
    worst = {}
    for name, w in want.items():
        e, c = stats(ours[name], w)
        g = group(name)
        we, wc = worst.get(g, (0.0, 1.0))
        worst[g] = (max(we, e), min(wc, c))
    print(tag, {g: f"max-rel {e:.2e} cos {c:.6f}" for g, (e, c) in worst.items()}, flush=True)


def main():
    from test_gpu_art_train import L_contig, _make
    from test_gpu_train import c5_batch

    from aonerf import _lib as L
    from aonerf import tiles, train_art
    torch.set_num_threads(16)
    batch, u_c, u_f = c5_batch(seed=12)
    batch["instance_id"] = torch.tensor([7], device="cuda")
    batch["articulation_id"] = torch.tensor([3], device="cuda")
    for trunk in (True, False):
        net, lib = _make(0, precision="bf16", art_forward="bf16_trunk" if trunk else "f16x3")
        latents = lib(batch)
        ret = net(batch, True, True, 2.0, 6.0, latents, u_coarse=u_c, u_fine=u_f,
                  return_intermediates=True)
        loss = train_art.img2mse(ret[1][0], batch["target"]) + train_art.img2mse(ret[0][0], batch["target"])
        for x in latents.values():
            x.retain_grad()
        loss.backward()
        torch.cuda.synchronize()
        rays = {k: batch[k].cpu() for k in ("rays_o", "rays_d", "viewdirs")}
        params = [{k: v.requires_grad_(True) for k, v in p.items()}
                  for p in O.split_state_dict(W.art_state_dict(0))]
        lat = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in latents.items()}
        ref_loss = 0.0
        for level in range(2):
            comp = O.art_render_level(params, rays, ret[level][3]["t_vals"].cpu(), level, True, lat)[0]
            ref_loss = ref_loss + O.img2mse(comp, batch["target"].cpu())
        ref_loss.backward()
        want = {f"{pre}{n}": v.grad for lv, pre in ((0, "coarse_mlp."), (1, "fine_mlp."))
                for n, v in params[lv].items()}
        want.update({f"latent {k}": v.grad for k, v in lat.items()})
        ours = {n: p.grad.cpu() for n, p in net.named_parameters()}
        ours.update({f"latent {k}": v.grad.cpu() for k, v in latents.items()})
        print(f"bf16_trunk={trunk}: loss gpu {loss.item():.7f} fp32 oracle {ref_loss.item():.7f}")
        report(f"  (i) whole step vs fp32 oracle:", ours, want)
        # (ii) stage-isolated backward per level
        lat_t = tuple(L_contig(latents[k]) for k in ("density", "color", "articulation"))
        for level, mlp in enumerate((net.coarse_mlp, net.fine_mlp)):
            t = ret[level][3]["t_vals"].contiguous()
            B, S = t.shape
            R = B * S
            geo = train_art._Geo(mlp)
            P = [(m.weight.detach(), m.bias.detach()) for m in train_art.art_layers(mlp)]
            raw = torch.empty((R, 4), device="cuda")
            masks = torch.empty((16, tiles.rows(R), 8), dtype=torch.int32, device="cuda")
            xyz, hd, enc, h, bot, hv, enc_bf = train_art._forward_level_fused(
                geo, P, lat_t, batch["rays_o"], batch["rays_d"], batch["viewdirs"], t, raw, None,
                masks, bf16=True, return_enc_bf=True)
            venc = torch.empty((B, 27), device="cuda")
            L.call("aon_pos_enc", L.ptr(batch["viewdirs"]), B, 0, 4, L.ptr(venc), L.stream())
            comp = torch.empty((B, 3), device="cuda")
            acc = torch.empty((B,), device="cuda")
            wts = torch.empty((B, S), device="cuda")
            depth = torch.empty((B,), device="cuda")
            L.call("aon_composite_fwd", L.ptr(raw), 4, L.ptr(raw[:, 3:]), 4, L.ptr(t),
                   L.ptr(batch["rays_d"]), B, S, 1, L.ACT_ARTIC, L.ptr(comp), L.ptr(acc),
                   L.ptr(wts), L.ptr(depth), L.stream())
            g_rgb = (2.0 * (comp - batch["target"]) / (3 * B)).contiguous()
            draw = torch.empty((R, 4), device="cuda")
            L.call("aon_composite_bwd", L.ptr(raw), 4, L.ptr(raw[:, 3:]), 4, L.ptr(t),
                   L.ptr(batch["rays_d"]), B, S, 1, L.ACT_ARTIC, L.ptr(g_rgb), None, None,
                   L.ptr(draw), L.ptr(draw[:, 3:]), 4, L.stream())
            G = [(torch.empty_like(w), torch.empty_like(b)) for w, b in P]
            dlat = tuple(torch.empty_like(x) for x in lat_t)
            train_art._backward_level_fused(geo, P, G, lat_t, dlat, xyz, enc, venc, S, hd, h, bot,
                                            hv, draw, masks, True, enc_bf)
            torch.cuda.synchronize()
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
            o2, w2 = {}, {}
            layer_names = [f"{n}" for n in ("deformations_linear.0", "deformations_linear.1",
                                            "deformations_linear.2", "deformations_linear.3",
                                            "deformation_layer")] + \
                [f"pts_linears.{i}" for i in range(8)] + ["density_layer", "bottleneck_layer"] + \
                [f"views_linear.{i}" for i in range(4)] + ["rgb_layer"]
            for (dw, db), name in zip(G, layer_names):
                o2[name + ".weight"], w2[name + ".weight"] = dw.cpu(), p64[name + ".weight"].grad
                o2[name + ".bias"], w2[name + ".bias"] = db.cpu(), p64[name + ".bias"].grad
            for d, k in zip(dlat, names):
                o2["latent " + k], w2["latent " + k] = d.cpu(), l64[k].grad
            report(f"  (ii) level {level} bf16 backward stage-isolated vs fp64 at our forward:", o2, w2)
        # (iii) step time
        opt = train_art.configure_optimizers(net, lib)
        for i in range(8):
            if i == 3:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
            opt.zero_grad()
            ls, _ = train_art.training_step(net, lib, batch, True, True, 2.0, 6.0)
            ls.backward()
            opt.step()
        torch.cuda.synchronize()
        print(f"  (iii) step {1e3 * (time.perf_counter() - t0) / 5:.2f} ms", flush=True)


if __name__ == "__main__":
    main()
