"""Profiling driver (GPU): K training steps of config C5 (4,096 rays, randomized, Adam) for
rocprofv3 --kernel-trace --stats, in one mode:

    python tools/prof_train_step.py [--art] [--precision f16x3|bf16] [--trunk] [--steps K]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "articulated-object-nerf_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--art", action="store_true")
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--art-forward", default="f16_acts",
                    help="articulated bf16: TrainNumerics.art_forward (f16_acts, f16x3, "
                         "f16_weights, bf16_view, bf16_trunk)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--overlap", type=int, default=0, help="TrainNumerics.overlap_dweight 0 / 1")
    args = ap.parse_args()
    from test_gpu_train import _make_trainable, c5_batch

    from aonerf import train, train_art
    batch, _, _ = c5_batch(seed=12)
    numerics = dict(precision=args.precision, overlap_dweight=bool(args.overlap),
                    art_forward=args.art_forward)
    if args.art:
        from test_gpu_art_train import _make
        batch["instance_id"] = torch.tensor([7], device="cuda")
        batch["articulation_id"] = torch.tensor([3], device="cuda")
        net, lib = _make(0, **numerics)
        opt = train_art.configure_optimizers(net, lib)
    else:
        net = _make_trainable(0, **numerics)
        opt = train.Adam(net.parameters())

    def step():
        opt.zero_grad()
        if args.art:
            loss, _ = train_art.training_step(net, lib, batch, True, True, 2.0, 6.0)
        else:
            loss, _ = train.training_step(net, batch, True, True, 2.0, 6.0)
        loss.backward()
        opt.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    print(f"{'art' if args.art else 'vanilla'} {args.precision} {args.art_forward if args.art else ''}"
          f"{' overlap' if args.overlap else ''}: "
          f"{1e3 * (time.perf_counter() - t0) / args.steps:.3f} ms/step", flush=True)


if __name__ == "__main__":
    main()
