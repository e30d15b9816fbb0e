"""The reference's own end-to-end self-consistency on the headline bench sample (verdict r05 #1):
the fp32 oracle (torch CPU restatement of helper.py:106-252 / model.py:147-199) against itself
re-run as another valid fp32 implementation -- its GEMMs split-K (oracle/attribution.py
GEMM_VARIANTS["k_split"]) and optionally others -- on the 16 x 3,840 centre rays of the bench
frame (bench.py cpu_baseline).  Prints, per variant, the fraction of rays whose rgb / acc /
depth stay within 1e-4 of the fp32 oracle.  CPU only; test/diagnostic infrastructure.

    python tools/diag/self_frac.py [--chunks 16] [--variants k_split,fp64_gemm]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "articulated-object-nerf_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import attribution as A  # noqa: E402
from oracle import nerf_oracle as O  # noqa: E402
from oracle import weights as Wt  # noqa: E402

H, W = 480, 640


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", type=int, default=16)
    ap.add_argument("--variants", default="k_split")
    ap.add_argument("--out", default=None)
    ap.add_argument("--ref-cache", default=None, help=".npz: load the fp32 oracle's outputs "
                    "from it if present, else compute and save them")
    ap.add_argument("--frame", action="append", default=[],
                    help="a bench --dump-frame .npy (H*W x [rgb, depth, acc]) to compare too")
    args = ap.parse_args()
    c2w = np.asarray(O.create_spheric_poses(4.0)[7], np.float32)
    focal = O.focal_from_fovy(H)
    params = O.split_state_dict(Wt.nerf_state_dict(0))
    dirs = O.get_ray_directions(H, W, focal)
    ro, rv, rd = O.get_rays(dirs, torch.as_tensor(c2w)[:3, :4], True)
    n = 3840 * args.chunks
    p0 = (H * W) // 2 - n // 2

    def run():
        outs = []
        for i in range(p0, p0 + n, 3840):
            sl = slice(i, i + 3840)
            ret = O.nerf_forward(params, {"rays_o": ro[sl], "rays_d": rd[sl], "viewdirs": rv[sl]},
                                 False, True, 2.0, 6.0)
            outs.append(ret[1])
        return [torch.cat([o[j] for o in outs]).numpy().astype(np.float64) for j in range(3)]

    t0 = time.perf_counter()
    if args.ref_cache and os.path.exists(args.ref_cache):
        z = np.load(args.ref_cache)
        ref = [z["rgb"], z["acc"], z["depth"]]
    else:
        ref = run()
        if args.ref_cache:
            np.savez(args.ref_cache, rgb=ref[0], acc=ref[1], depth=ref[2])
    res = {"rays": n, "p0": p0, "ref_s": time.perf_counter() - t0, "variants": {}, "frames": {}}

    def fracs(out):
        fr = {}
        for k, a, b in zip(("rgb", "acc", "depth"), out, ref):
            e = np.abs(a - b).reshape(n, -1).max(-1)
            fr[k] = {"frac_within_1e-4": float((e <= A.E2E_ATOL).mean()),
                     "outliers": int((e > A.E2E_ATOL).sum()), "max_abs": float(e.max())}
        return fr

    for fpath in args.frame:
        f = np.load(fpath)[p0:p0 + n].astype(np.float64)
        res["frames"][fpath] = fracs([f[:, :3], f[:, 4], f[:, 3]])
        print(fpath, json.dumps(res["frames"][fpath]), flush=True)
    variants = A.oracle_variants()
    for v in [x for x in args.variants.split(",") if x]:
        t0 = time.perf_counter()
        with variants[v]():
            out = run()
        res["variants"][v] = {"s": time.perf_counter() - t0, **fracs(out)}
        print(v, json.dumps(res["variants"][v]), flush=True)
    if args.out:
        json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
