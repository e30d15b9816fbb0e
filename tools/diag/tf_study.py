"""CPU study for the teacher-forced training gates (verdict r05 #2): the reference's own
self-variance of one Adam step from its recorded state -- the fp32 step against the same step
re-evaluated in fp64 -- per step and per tensor, as relative L2 distance and cosine of the
updates.  Run before the GPU test to fix its constants.

    python tools/diag/tf_study.py [--kind vanilla|art] [--steps 20] [--lr 1e-3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "articulated-object-nerf_amd")]

import numpy as np  # noqa: E402

from oracle import trajectory as T  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="vanilla")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    t0 = time.perf_counter()
    batch = T.make_batch(args.kind, T.batch_rays(args.kind))
    rec = T.reference_run(args.kind, batch, args.steps, args.lr)
    rows = []
    for k, r in enumerate(rec):
        c = T.compare(r["delta64"], r["delta"])
        e = np.array([v[0] for v in c.values()])
        cs = np.array([v[1] for v in c.values()])
        worst = max(c, key=lambda n: c[n][0])
        cg = T.compare(r["grad64"], r["grad"])
        eg = np.array([v[0] for v in cg.values()])
        rows.append({"step": k, "loss": r["loss"], "self_rel_max": float(e.max()),
                     "self_rel_median": float(np.median(e)), "self_cos_min": float(cs.min()),
                     "worst": worst, "grad_self_rel_max": float(eg.max()),
                     "grad_self_rel_median": float(np.median(eg)),
                     "grad_worst": max(cg, key=lambda n: cg[n][0])})
        print(json.dumps(rows[-1]), flush=True)
    print(f"{args.kind}: {time.perf_counter() - t0:.1f} s")
    if args.out:
        json.dump(rows, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
