#!/usr/bin/env python3
"""Articulated render throughput (BASELINE config C3: NeRF_AE_Art on a 320x240 sapien_multi
view, 64c+128f, eval mode, white background, fixed latent codes).

    python tools/bench_articulated.py [--steps 5] [--warmup 2]

One JSON line: rays/s of the whole two-level frame render, and the algorithmic MLP rate with
the reference's unfolded count (2 x 794,880 MAC per sample); the latent
products are folded into per-call biases, so the issued work is 714,880 MAC per sample.
``--layerwise`` times the layer-by-layer aon_gemm path instead of the fused kernel.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "articulated-object-nerf_amd")]

import torch  # noqa: E402

H, W = 240, 320
MAC_UNFOLDED = 794_880


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--layerwise", action="store_true")
    args = ap.parse_args()
    from aonerf.model_autodecoder import NeRF_AE_Art
    from aonerf.ray_utils import frame_rays
    from aonerf.render import create_spheric_poses, sapien_focal
    from aonerf.synthetic import art_latents, init_like_reference

    net = init_like_reference(NeRF_AE_Art()).cuda()
    lat = art_latents(0, device="cuda")
    net.coarse_mlp.fused = net.fine_mlp.fused = not args.layerwise
    rays = frame_rays(torch.as_tensor(create_spheric_poses(4.0)[11]), H, W, sapien_focal(H))

    @torch.no_grad()  # a render (Lightning's eval steps run without autograd)
    def step():
        return net(rays, False, True, 2.0, 6.0, lat)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ret = step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    n = H * W
    flop = 2 * MAC_UNFOLDED * (65 + 193) * n * args.steps
    print(json.dumps({
        "metric": "articulated rays/sec at 320x240x(64c+128f) (NeRF_AE_Art, C3)",
        "value": n * args.steps / dt, "unit": "rays/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": 1000 * dt / args.steps, "higher_is_better": True,
        "dtype": "f16x3 (fp16 hi/lo split MFMA, fp32 accumulate)", "data": "synthetic",
        "config": {"workload": "C3 NeRF_AE_Art frame render", "rays_per_step": n,
                   "mlp_path": "layerwise aon_gemm" if args.layerwise else "fused aon_mlp_art_fwd"},
        "mlp_tflops_algorithmic_unfolded": flop / dt / 1e12,
        "mean_rgb": float(ret[1][0].mean().item())}))


if __name__ == "__main__":
    main()
