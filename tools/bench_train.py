#!/usr/bin/env python3
"""Training-step throughput (BASELINE configs C5: LitNeRF.training_step on 4096-ray batches,
randomized sampling, Adam with the reference schedule; DDP over N GPUs = N independent
batches + one gradient all-reduce per step, weak scaling).  ``--model art`` times the
articulated auto-decoder's step instead (LitNeRF_AutoDecoder.training_step,
model_autodecoder.py:395-477: NeRF_AE_Art + CodeLibraryArticulated, latent regulariser, Adam
over the MLPs and the code tables).

    python tools/bench_train.py [--model vanilla|art] [--rays 4096] [--steps 10] [--warmup 3]
    python tools/bench_train.py --gpus N [--backend gloo]     (spawns the N ranks itself)
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/bench_train.py --gpus N

A step = draw a batch of pixels of a synthetic 640x480 view (8 poses of create_spheric_poses,
target image PCG64 seed 3), coarse + fine training forward, loss, HIP backward, gradient
all-reduce, fused Adam.  Rank 0 prints one JSON line; timing is the max over ranks with barrier
+ synchronize on both sides.  Algorithmic FLOP per step = 3 x the forward MLP FLOP (dX and dW
each cost one forward) = 3 x 2 x 593,408 x 258 per ray (articulated: 794,880 MAC per sample,
latent columns unfolded, as the reference computes them).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "articulated-object-nerf_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

H, W = 480, 640
MAC = {"vanilla": 593_408, "art": 794_880}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", choices=("vanilla", "art"), default="vanilla")
    ap.add_argument("--rays", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--max-steps", type=int, default=200000, help="schedule length (run_max_steps)")
    ap.add_argument("--precision", choices=("f16x3", "bf16"), default="f16x3",
                    help="the model's train_precision (bf16: C5's bf16 mode)")
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one process per GPU)")
    ap.add_argument("--backend", default="nccl", choices=("nccl", "gloo"))
    args = ap.parse_args()
    from aonerf import launch

    if args.gpus > 1 and not launch.launched_externally():
        sys.exit(launch.spawn_ranks(os.path.abspath(__file__), sys.argv[1:], args.gpus))
    world, rank, local_rank, dev = launch.init_rank(args.backend, expect_world=args.gpus)
    from aonerf import train
    from aonerf.model import NeRF
    from aonerf.parallel import GradAllReduce
    from aonerf.ray_utils import frame_rays
    from aonerf.render import create_spheric_poses, sapien_focal
    from aonerf.synthetic import init_like_reference  # same initial weights as bench.py

    art = args.model == "art"
    if art:
        import types

        from aonerf import train_art
        from aonerf.code_library import CodeLibraryArticulated
        from aonerf.model_autodecoder import NeRF_AE_Art
        from aonerf.synthetic import init_code_library

        net = init_like_reference(NeRF_AE_Art(train_precision=args.precision)).to(dev)
        lib = init_code_library(CodeLibraryArticulated(
            types.SimpleNamespace(N_max_objs=151, N_obj_code_length=128))).to(dev)
        ids = {"instance_id": torch.tensor([7], device=dev),
               "articulation_id": torch.tensor([3], device=dev)}
    else:
        net = init_like_reference(NeRF(train_precision=args.precision)).to(dev)
    poses = create_spheric_poses(4.0)
    focal = sapien_focal(H)
    rays_all = {k: [] for k in ("rays_o", "rays_d", "viewdirs")}
    for k in range(8):
        r = frame_rays(torch.as_tensor(poses[(5 * k) % len(poses)]), H, W, focal)
        for key in rays_all:
            rays_all[key].append(r[key])
    rays_all = {k: torch.cat(v, 0) for k, v in rays_all.items()}
    rng = np.random.Generator(np.random.PCG64(3))
    target_all = torch.from_numpy(rng.uniform(0, 1, size=(8 * H * W, 3)).astype(np.float32)).to(dev)
    gen = torch.Generator(device=dev).manual_seed(1000 + rank)
    params = list(net.parameters()) + (list(lib.parameters()) if art else [])
    opt = train.Adam(params)
    sync = GradAllReduce(params)

    def step(i):
        idx = torch.randint(0, 8 * H * W, (args.rays,), device=dev, generator=gen)
        batch = {k: v[idx] for k, v in rays_all.items()}
        batch["target"] = target_all[idx]
        opt.zero_grad()
        if art:
            batch.update(ids)
            loss, _ = train_art.training_step(net, lib, batch, True, True, 2.0, 6.0)
        else:
            loss, _ = train.training_step(net, batch, True, True, 2.0, 6.0)
        loss.backward()
        sync()
        opt.step(lr=train.learning_rate(i, args.max_steps))
        return loss

    for i in range(args.warmup):
        step(i)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = step(args.warmup + i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = launch.max_over_ranks(time.perf_counter() - t0)
    rays = args.rays * args.steps * world
    flop = 3 * 2 * MAC[args.model] * (65 + 193) * rays
    if rank == 0:
        print(json.dumps({
            "metric": ("training rays/sec (LitNeRF_AutoDecoder.training_step, NeRF_AE_Art, 64c+128f, "
                       "randomized, Adam)" if art else
                       "training rays/sec (LitNeRF.training_step, 64c+128f, randomized, Adam)"),
            "value": rays / dt, "unit": "rays/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": 1000 * dt / args.steps,
            "higher_is_better": True, "scaling": "weak",
            "dtype": "bf16 (bf16 MFMA)" if args.precision == "bf16" and not art else "f16x3 (fp16 hi/lo split MFMA)",
            "data": "synthetic", "config": {"workload": "C5 training step" + (" (articulated)" if art else ""),
                                             "rays_per_rank": args.rays,
                                             "parallelism": f"ddp{world}"},
            "mlp_tflops_algorithmic": flop / dt / 1e12, "final_loss": float(loss.item())}))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
