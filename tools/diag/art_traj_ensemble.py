#!/usr/bin/env python3
"""The reference's own spread on the articulated trajectory test's run (CPU, no GPU needed):
test_gpu_art_train_bf16.test_art_bf16_loss_trajectory's 128-ray batch, 20 Adam steps at lr
2e-4 (or --lr / --steps), through the fp32 oracle, the fp64 oracle, and fp32 oracles whose MLP
weights differ from the reference's by one rounding each (x (1 + 2^-24 n), n ~ N(0, 1), seeded)
-- an ensemble of fp32-class evaluations of the same run.  Prints each member's largest
relative distance from the fp32 oracle's loss over the steps (the quantity the test gates)."""
import argparse
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import nerf_oracle as O  # noqa: E402
from oracle import weights as W  # noqa: E402


def batch():
    H, Wd = 48, 64
    focal = 0.5 * H / math.tan(0.5 * math.radians(35.0))
    c2w = torch.as_tensor(O.create_spheric_poses(4.0)[2][:3])
    rays_o, rays_d = O.get_rays(O.get_ray_directions(H, Wd, focal), c2w)[:2]
    rays_o, rays_d = rays_o.reshape(-1, 3), rays_d.reshape(-1, 3)
    sel = torch.arange(0, H * Wd, 24)
    b = {"rays_o": rays_o[sel], "rays_d": rays_d[sel], "viewdirs": rays_d[sel]}
    g = torch.linspace(0.0, 1.0, len(sel))
    b["target"] = torch.stack([g, 1.0 - g, 0.5 + 0.4 * torch.sin(12.0 * g)], -1)
    return b


def trajectory(b, steps, lr, dtype, perturb_seed=None):
    gen = torch.Generator().manual_seed(perturb_seed) if perturb_seed is not None else None

    def leaf(v):
        v = torch.as_tensor(v)
        if gen is not None:
            v = v.double() * (1 + 2.0 ** -24 * torch.randn(v.shape, generator=gen, dtype=torch.float64))
        return v.to(dtype).requires_grad_(True)

    params = [{k: leaf(v) for k, v in p.items()} for p in O.split_state_dict(W.art_state_dict(0))]
    tables = {k: torch.from_numpy(v).to(dtype).requires_grad_(True)
              for k, v in W.code_library_state_dict(0).items()}
    flat = [v for p in params for v in p.values()] + list(tables.values())
    opt = torch.optim.Adam(flat, lr=lr, betas=(0.9, 0.999))
    rc = {k: b[k].to(dtype) for k in ("rays_o", "rays_d", "viewdirs")}
    tgt = b["target"].to(dtype)
    out = []
    for _ in range(steps):
        opt.zero_grad()
        loss = O.art_training_loss(params, tables, rc, tgt, 7, 3, False, True, 2.0, 6.0)[0]
        loss.backward()
        opt.step()
        out.append(loss.item())
    return np.array(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--lr", type=float, default=2e-4)
    ap.add_argument("--seeds", type=int, default=6)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    b = batch()
    ref = trajectory(b, args.steps, args.lr, torch.float32)
    res = {"lr": args.lr, "steps": args.steps, "fp32_final": float(ref[-1])}
    members = {"fp64": trajectory(b, args.steps, args.lr, torch.float64)}
    for s in range(1, args.seeds + 1):
        members[f"fp32 ulp seed {s}"] = trajectory(b, args.steps, args.lr, torch.float32, s)
    for k, v in members.items():
        d = np.abs(v / ref - 1)
        res[k] = {"max_rel": float(d.max()), "at_step": int(d.argmax())}
        print(f"{k:18s} max rel {d.max():.2e} (step {d.argmax()})", flush=True)
    if args.out:
        json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
