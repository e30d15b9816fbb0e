"""Diagnostic (GPU box): the bench frame's parity at scale, ray by ray, for the rays the
attribution leaves unexplained (bench.py cpu_baseline `unattributed`), plus whether the box's
torch CPU reproduces the reference's ray generation as fma chains (the GPU kernel's order,
bit-exact against the golden rays generated in the build container).

    python tools/diag/parity_scale.py [--chunks 16] [--out gpurun_out/parity_scale.json]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "articulated-object-nerf_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import attribution as A  # noqa: E402
from oracle import nerf_oracle as O  # noqa: E402
from oracle import weights as Wt  # noqa: E402

H, W = 480, 640


def fma_chain_rays(dirs, c2w):
    """rays_d as the GPU kernel computes it (forward fma chains, rays.hip), emulated in fp64."""
    M = c2w[:3, :3].double().numpy()
    d = dirs.reshape(-1, 3).double().numpy()

    def r32(x):
        return x.astype(np.float32).astype(np.float64)

    r = np.zeros((d.shape[0], 3))
    for k in range(3):
        acc = r32(d[:, 0] * M[k, 0])
        acc = r32(d[:, 1] * M[k, 1] + acc)
        r[:, k] = r32(d[:, 2] * M[k, 2] + acc)
    s = r32(r[:, 0] * r[:, 0])
    s = r32(r[:, 1] * r[:, 1] + s)
    s = r32(r[:, 2] * r[:, 2] + s)
    n = r32(np.sqrt(s))
    return r, r32(r / n[:, None])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", type=int, default=16)
    ap.add_argument("--out", default="gpurun_out/parity_scale.json")
    args = ap.parse_args()
    from aonerf.model import NeRF
    from aonerf.ray_utils import frame_rays
    from aonerf.render import create_spheric_poses, sapien_focal
    from aonerf.synthetic import init_like_reference

    torch.set_num_threads(16)
    res = {"torch_cpu_capability": torch.backends.cpu.get_cpu_capability()}
    c2w = create_spheric_poses(4.0)[7]
    focal = sapien_focal(H)
    dirs = O.get_ray_directions(H, W, focal)
    ro, rv, rd = O.get_rays(dirs, c2w[:3, :4], True)
    raw_t = (dirs @ c2w[:3, :3].T).reshape(-1, 3).double().numpy()
    raw_f, unit_f = fma_chain_rays(dirs, c2w)
    res["box_torch_matmul_vs_fma_chain_mismatches"] = int((raw_t != raw_f).sum())
    res["box_torch_rays_d_vs_fma_chain_mismatches"] = int((rd.double().numpy() != unit_f).sum())
    net = init_like_reference(NeRF()).cuda()
    gr = frame_rays(c2w, H, W, focal)
    g_rd = gr["rays_d"].cpu().double().numpy()
    res["gpu_rays_d_vs_box_torch_mismatch_rays"] = int((g_rd != rd.double().numpy()).any(-1).sum())
    res["gpu_rays_d_vs_fma_chain_mismatch_rays"] = int((g_rd != unit_f).any(-1).sum())
    n = 3840 * args.chunks
    p0 = (H * W) // 2 - n // 2
    params = O.split_state_dict(Wt.nerf_state_dict(0))
    outs, w_ref = [], []
    for i in range(p0, p0 + n, 3840):
        sl = slice(i, i + 3840)
        ret, inter = O.nerf_forward(params, {"rays_o": ro[sl], "rays_d": rd[sl], "viewdirs": rv[sl]},
                                    False, True, 2.0, 6.0, return_intermediates=True)
        outs.append(ret[1])
        w_ref.append(inter[0]["weights"])
        print(f"chunk {i}", flush=True)
    ref = [torch.cat([o[j] for o in outs]).numpy() for j in range(3)]
    w_ref = torch.cat(w_ref).numpy()
    rays = frame_rays(c2w, H, W, focal, p0=p0, n=n)
    with torch.no_grad():
        mine = net(rays, False, True, 2.0, 6.0, return_weights=True, return_intermediates=True)
    gpu = [mine[1][j].cpu().numpy() for j in range(3)]
    w_ours = mine[0][3].cpu().numpy()
    t_fine = mine[1][4]["t_vals"].cpu()
    errs = [np.abs(g.astype(np.float64) - r.astype(np.float64)) for g, r in zip(gpu, ref)]
    bad = np.zeros(n, bool)
    for e in errs:
        bad |= (e > A.E2E_ATOL).reshape(n, -1).any(-1)
    rows = np.nonzero(bad)[0]
    sub = {"rays_o": ro[p0:p0 + n][rows], "rays_d": rd[p0:p0 + n][rows],
           "viewdirs": rv[p0:p0 + n][rows]}
    # the reference's fine level on OUR fine samples, through the reference's rays and ours
    on_ours = O.render_level(params, sub, t_fine[rows], 1, True)
    ours_rays = {k: v[rows].cpu() for k, v in rays.items()}
    on_ours_own = O.render_level(params, ours_rays, t_fine[rows], 1, True)
    ro_b, rv_b, rd_b = O.get_rays_fma(dirs, c2w[:3, :4])
    alt = {"rays_o": ro_b[p0:p0 + n][rows], "rays_d": rd_b[p0:p0 + n][rows],
           "viewdirs": rv_b[p0:p0 + n][rows]}
    env, _ = A.fine_envelope(params, sub, alt_rays=alt)
    att = A.Attribution(w_ours[rows], w_ref[rows], 128)
    ray_diff = (g_rd[p0:p0 + n][rows] != rd[p0:p0 + n][rows].double().numpy()).any(-1)
    detail = []
    names = ("rgb", "acc", "depth")
    unexpl = np.zeros(len(rows), bool)
    for j, k in enumerate(names):
        e = errs[j][rows]
        ok = att.rays(on_ours[j if j < 2 else 3].numpy(), ref[j][rows], e, env[j])
        oq = (e > A.E2E_ATOL).reshape(len(rows), -1).any(-1)
        unexpl |= oq & ~ok
    em = np.stack([errs[j][rows].reshape(len(rows), -1).max(-1) for j in range(3)], -1)
    sens = np.stack([np.abs(on_ours[jj].numpy().reshape(len(rows), -1) -
                            ref[j][rows].reshape(len(rows), -1)).max(-1)
                     for j, jj in ((0, 0), (1, 1), (2, 3))], -1)
    sens_own = np.stack([np.abs(on_ours_own[jj].numpy().reshape(len(rows), -1) -
                                gpu[j][rows].reshape(len(rows), -1)).max(-1)
                         for j, jj in ((0, 0), (1, 1), (2, 3))], -1)
    envm = np.stack([np.asarray(env[j]).reshape(len(rows), -1).max(-1) for j in range(3)], -1)
    for r in np.nonzero(unexpl)[0]:
        detail.append({"ray": int(rows[r]), "err": em[r].tolist(), "coarse_dw": float(att.dw[r]),
                       "flip": bool(att.flips[r]), "ref_move_on_our_t": sens[r].tolist(),
                       "ours_vs_ref_level_on_our_t_our_rays": sens_own[r].tolist(),
                       "env": envm[r].tolist(), "ray_dir_differs": bool(ray_diff[r])})
    res.update({"rays": n, "outlier_rays": int(len(rows)), "unattributed": int(unexpl.sum()),
                "outlier_rays_with_ray_dir_diff": int(ray_diff.sum()), "unattributed_detail": detail})
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "unattributed_detail"}))
    for d in detail[:20]:
        print(d)


if __name__ == "__main__":
    main()
