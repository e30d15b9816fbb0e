#!/usr/bin/env python3
"""Benchmark: rays/sec of the full two-level render of a synthetic 640x480 frame at 64c+128f
samples (BASELINE.json configs[1]; configs[3] when launched on N GPUs: the frame is split into
N row bands, one per rank, and gathered to rank 0 over RCCL).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--precision fp32]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

A step = generate the frame's rays, coarse sample, coarse MLP, composite, pdf resample, fine
MLP, composite, gather.  value = 307,200 rays x steps / max-over-ranks wall time.  Rank 0 prints
ONE JSON line.  Inputs: create_spheric_poses(4)[7] camera, fovy-35 focal, near 2 / far 6,
random NeRF weights (aonerf.synthetic, PCG64 seed 0: the oracle's test weights bit for bit,
tests/test_synthetic.py).  The CPU baseline is the torch restatement in oracle/ on a bounded
ray sample (test infrastructure, never the measured path).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "articulated-object-nerf_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

H, W = 480, 640
NC, NF = 64, 128
MAC_PER_SAMPLE = 593_408            # NeRFMLP multiply-accumulates per sample
# Dense MFMA peak of the issued instruction, in ALGORITHMIC (fp32-class) FLOP/s: fp32 MFMA
# 157.3 TF; fp16 MFMA 2500 TF, of which f16x3 spends 3 products per fp32-class MAC -> 833.3.
PEAK_TFLOPS = {"fp32": 157.3, "f16x3": 2500.0 / 3}
ISSUED_PEAK = {"fp32": ("v_mfma_f32_16x16x4_f32", 157.3, 1), "f16x3": ("v_mfma_f32_16x16x32_f16", 2500.0, 3)}
PEAK_HBM_GBS = 8000.0


def composite_bytes(S, weights_out=True):
    # per ray: raw (S,4) + t (S) + dirs (3) read; rgb(3) + acc + depth (+ weights (S)) written.
    # The frame render does not ask for the fine level's weights, so that launch skips them.
    return 16 * S + 4 * S + 12 + 20 + (4 * S if weights_out else 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)  # >= 10 timed, 3 warm-up
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--precision", default="f16x3", choices=sorted(PEAK_TFLOPS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-chunks", type=int, default=2, help="3840-ray chunks in the CPU sample")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    from aonerf.model import NeRF
    from aonerf.parallel import render_frame_sharded
    from aonerf.render import create_spheric_poses, sapien_focal
    from aonerf.synthetic import init_like_reference

    net = init_like_reference(NeRF(precision=args.precision)).cuda()
    c2w = create_spheric_poses(4.0)[7]
    focal = sapien_focal(H)

    def step(timers=None):
        return render_frame_sharded(net, c2w, H, W, focal, 2.0, 6.0, True, timers=timers)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    timers = {}
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        frame, _ = step(timers)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    el = torch.tensor([elapsed], device="cuda")
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = el.item()

    # per-launch kernel times from HIP events on the launch stream
    def avg_ms(key):
        ev = timers.get(key, [])
        if not ev:
            return None, 0
        return float(np.mean([a.elapsed_time(b) for a, b, _ in ev])), ev[0][2]

    mlp_ms, rows = avg_ms("mlp1")
    comp_ms, comp_rows = avg_ms("comp1")
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    rays = H * W
    value = rays * args.steps / elapsed
    flops = 2.0 * MAC_PER_SAMPLE * rows
    achieved = flops / (mlp_ms * 1e-3) / 1e12 if mlp_ms else None
    peak = PEAK_TFLOPS[args.precision]
    traffic = None
    tpath = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tpath):
        t = json.load(open(tpath))
        if t.get("precision") == args.precision and t.get("world") == world:
            traffic = t.get("fine_mlp_hbm_bytes")
    out = {
        "metric": "rays/sec at 640×480×(64c+128f) samples; PSNR vs reference",
        "value": value, "unit": "rays/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
        "dtype": "fp32" if args.precision == "fp32" else "f16x3 (fp16 hi/lo split MFMA, fp32 accumulate)",
        "data": "synthetic",
        "config": {"workload": "sapien vanilla 640x480 frame render, 64c+128f (65+193 MLP "
                               "samples/ray), randomized=False, white_bkgd, near 2 far 6",
                   "rays_per_step": rays, "samples_per_ray": (NC + 1) + (NC + 1 + NF),
                   "parallelism": f"row-band x{world} + RCCL gather" if world > 1 else "single GPU",
                   "mlp_precision": args.precision},
        "roofline": {"bound": "mfma", "kernel": ("k_mlp_fwd_f32" if args.precision == "fp32"
                                                  else "k_mlp_fwd_f16x3") + " (fine level)",
                     "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                     "frac": achieved / peak if achieved else None, "traffic": traffic,
                     "launch_ms": mlp_ms, "algorithmic_flop_per_launch": flops,
                     "issued": {"instruction": ISSUED_PEAK[args.precision][0],
                                "issued_tflops": achieved * ISSUED_PEAK[args.precision][2] if achieved else None,
                                "dtype_peak_tflops": ISSUED_PEAK[args.precision][1],
                                "note": "achieved counts algorithmic fp32-class FLOPs (2 x 593,408 "
                                        "MAC/sample); f16x3 issues 3 fp16 products per MAC, so its "
                                        "peak in those units is 2500/3 TF/s"}},
    }
    # the MFMA peak measured on random register operands (tools/mfma_peak.py)
    ppath = os.path.join(ROOT, "profiles", "mfma_peak.json")
    if achieved and os.path.exists(ppath):
        mp = json.load(open(ppath))
        key = "f32_16x16x4_tflops" if args.precision == "fp32" else "f16_16x16x32_tflops"
        if mp.get(key):
            iss = out["roofline"]["issued"]
            iss["measured_dtype_peak_tflops"] = mp[key]
            iss["frac_of_measured_peak"] = iss["issued_tflops"] / mp[key]
            iss["measured_peak_source"] = "profiles/mfma_peak.json (tools/mfma_peak.py)"
    if comp_ms:
        cb = composite_bytes(NC + 1 + NF, weights_out=False) * (comp_rows // (NC + 1 + NF))
        gbs = cb / (comp_ms * 1e-3) / 1e9
        out["roofline_composite"] = {"bound": "hbm", "kernel": "k_composite_fwd (fine level)",
                                     "achieved": gbs, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                                     "frac": gbs / PEAK_HBM_GBS, "launch_ms": comp_ms,
                                     "algorithmic_bytes_per_launch": cb}

    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(frame, c2w, focal, args.cpu_chunks)
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(frame, c2w, focal, nchunks):
    """The oracle (torch CPU restatement of the reference path) on nchunks x 3840 rays of the
    same frame, timed on the host cores; also the PSNR agreement of the GPU render there."""
    from oracle import nerf_oracle as O
    from oracle import weights as Wt

    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    params = O.split_state_dict(Wt.nerf_state_dict(0))
    dirs = O.get_ray_directions(H, W, focal)
    ro, rv, rd = O.get_rays(dirs, c2w[:3, :4], True)
    n = 3840 * nchunks
    p0 = (H * W) // 2 - n // 2  # centre rows (object region)
    t0 = time.perf_counter()
    outs = []
    for i in range(p0, p0 + n, 3840):
        sl = slice(i, i + 3840)
        outs.append(O.nerf_forward(params, {"rays_o": ro[sl], "rays_d": rd[sl], "viewdirs": rv[sl]},
                                   False, True, 2.0, 6.0)[1][0])
    dt = time.perf_counter() - t0
    ref = torch.cat(outs)
    gpu = frame[p0:p0 + n, :3].cpu()
    target = torch.from_numpy(np.random.Generator(np.random.PCG64(3)).uniform(0, 1, (n, 3)).astype(np.float32))
    p_ref = O.psnr_each([ref], [target]).item()
    p_gpu = O.psnr_each([gpu], [target]).item()
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "")
    except OSError:
        pass
    return {"value": n / dt, "unit": "rays/s", "cores": threads, "kind": "port",
            "cpu_model": model, "host_cpu_count": os.cpu_count(),
            "sample": f"{nchunks} x 3840-ray chunks (pixels {p0}..{p0 + n}) of the same frame, "
                      f"oracle/nerf_oracle.py torch-CPU restatement, {threads} threads, {dt:.1f} s",
            "max_abs_rgb_diff_vs_gpu": float((ref - gpu).abs().max()),
            "psnr_gpu_vs_reference_db": O.psnr_each([gpu], [ref]).item(),
            "psnr_delta_db": p_gpu - p_ref}


if __name__ == "__main__":
    main()
