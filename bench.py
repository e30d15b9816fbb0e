#!/usr/bin/env python3
"""Benchmark: rays/sec of the full two-level render of a synthetic 640x480 frame at 64c+128f
samples (BASELINE.json configs[1]; configs[3] when launched on N GPUs: the frame is split into
N row bands, one per rank, and gathered to rank 0 over RCCL).

Sub-records in the same JSON line (after the headline, same timing protocol: warm-up, barrier +
synchronize on both sides, max over ranks):
  "render_fp32"     the same C2 frame on the exact-fp32 MFMA MLP (NeRF(precision="fp32"); N = 1
                    only; min(K, 5) timed steps after 1 warm-up: 0.7 s per frame)
  "articulated"     config C3 -- NeRF_AE_Art 320x240 frame render (N = 1 only)
  "train_step"      config C5 -- LitNeRF.training_step on 4096 rays per rank + Adam (+ the DDP
                    gradient all-reduce over RCCL on N > 1: weak scaling), f16x3 kernels
  "train_step_bf16" the same step in C5's bf16 mode (NeRF(train_precision="bf16"))
  "train_step_art"  C5 on the articulated auto-decoder (LitNeRF_AutoDecoder.training_step)
  "train_step_art_bf16"  the same in the articulated bf16 mode
                    (NeRF_AE_Art(train_precision="bf16"))
each with its own ms_per_step and roofline (MFMA fraction of the fine-level MLP kernels,
HBM byte fractions of the training kernels counting the stored activations).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--precision fp32] [--backend gloo]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

``--gpus N`` (N > 1) without an external launcher spawns the N ranks itself, one process per
GPU, before anything touches the GPU (aonerf.launch; run.py:101-111 takes devices=num_gpus the
same way); under torchrun the launcher's WORLD_SIZE must equal N.  ``--backend gloo`` lets the
ranks share one device (the one-GPU test box rehearses the N-rank path that way; RCCL refuses
two ranks on one device); the default is nccl (RCCL over xGMI).

A step = generate the frame's rays, coarse sample, coarse MLP, the fused coarse composite +
pdf resample (aon_composite_march), fine MLP, composite, gather.  value = 307,200 rays x steps / max-over-ranks wall time.  Rank 0 prints
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
KERNEL = {"fp32": "k_mlp_fwd_f32", "f16x3": "k_mlp_fwd_f16x3"}
PEAK_HBM_GBS = 8000.0


def composite_bytes(S, weights_out=True):
    # per ray: raw (S,4) + t (S) + dirs (3) read; rgb(3) + acc + depth (+ weights (S)) written.
    # The frame render does not ask for the fine level's weights, so that launch skips them.
    return 16 * S + 4 * S + 12 + 20 + (4 * S if weights_out else 0)


def march_bytes(S, Ns):
    # fused coarse composite + resample (aon_composite_march) per ray: raw (S,4) + t (S) + dirs
    # read; rgb + acc + depth and the merged fine t (S + Ns) written.  The coarse weights stay on
    # chip (the eval-mode u is one shared 512-B row, L2-resident: not counted).
    return 16 * S + 4 * S + 12 + 20 + 4 * (S + Ns)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)  # >= 10 timed, 3 warm-up
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--precision", default="f16x3", choices=sorted(PEAK_TFLOPS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-chunks", type=int, default=16,
                    help="3840-ray chunks in the CPU sample (SURVEY.md 8(d): 16)")
    ap.add_argument("--no-extra", action="store_true", help="headline C2 render only")
    ap.add_argument("--backend", default="nccl", choices=("nccl", "gloo"),
                    help="process-group backend for N > 1 (gloo: ranks may share one GPU)")
    ap.add_argument("--dump-frame", default=None,
                    help="rank 0 saves the gathered frame of the last timed step (.npy)")
    args = ap.parse_args()

    from aonerf import launch

    if args.gpus > 1 and not launch.launched_externally():
        # one process per GPU, started before any GPU call in this process
        sys.exit(launch.spawn_ranks(os.path.abspath(__file__), sys.argv[1:], args.gpus))
    world, rank, local_rank, _ = launch.init_rank(args.backend, expect_world=args.gpus)

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
    elapsed = launch.max_over_ranks(time.perf_counter() - t0)
    if rank == 0 and args.dump_frame:
        np.save(args.dump_frame, frame.cpu().numpy())

    # per-launch kernel times from HIP events on the launch stream
    def avg_ms(key):
        ev = timers.get(key, [])
        if not ev:
            return None, 0
        return float(np.mean([a.elapsed_time(b) for a, b, _ in ev])), ev[0][2]

    mlp_ms, rows = avg_ms("mlp1")
    comp_ms, comp_rows = avg_ms("comp1")
    march_ms, march_rows = avg_ms("march0")
    extra = {}

    def run(name, fn, *a, **k):  # progress on stderr (the JSON line stays alone on stdout)
        if rank == 0:
            print(f"[bench] {name}", file=sys.stderr, flush=True)
        extra[name] = fn(*a, **k)

    if not args.no_extra:  # every rank takes part (the C5 step all-reduces over RCCL)
        if world == 1:
            if args.precision != "fp32":
                run("render_fp32", bench_render_fp32, args, c2w, focal)
            run("articulated", bench_articulated, args)
        run("train_step", bench_train, args, world, rank, local_rank)
        run("train_step_bf16", bench_train, args, world, rank, local_rank, precision="bf16")
        run("train_step_art", bench_train, args, world, rank, local_rank, art=True)
        run("train_step_art_bf16", bench_train, args, world, rank, local_rank, art=True,
            precision="bf16")
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
        "backend": args.backend if world > 1 else None,
        "dtype": "fp32" if args.precision == "fp32" else "f16x3 (fp16 hi/lo split MFMA, fp32 accumulate)",
        "data": "synthetic",
        "config": {"workload": "sapien vanilla 640x480 frame render, 64c+128f (65+193 MLP "
                               "samples/ray), randomized=False, white_bkgd, near 2 far 6",
                   "rays_per_step": rays, "samples_per_ray": (NC + 1) + (NC + 1 + NF),
                   "parallelism": f"row-band x{world} + RCCL gather" if world > 1 else "single GPU",
                   "mlp_precision": args.precision},
        "roofline": {"bound": "mfma", "kernel": KERNEL[args.precision] + " (fine level)",
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
        key = {"fp32": "f32_16x16x4_tflops", "f16x3": "f16_16x16x32_tflops"}[args.precision]
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
    if march_ms:
        mb = march_bytes(NC + 1, NF) * (march_rows // (NC + 1))
        gbs = mb / (march_ms * 1e-3) / 1e9
        out["roofline_march"] = {"bound": "hbm", "kernel": "k_composite_march (coarse composite + "
                                 "inverse-CDF resample + merge, fused)", "achieved": gbs,
                                 "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": gbs / PEAK_HBM_GBS,
                                 "launch_ms": march_ms, "algorithmic_bytes_per_launch": mb}

    out.update(extra)
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(net, frame, c2w, focal, args.cpu_chunks)
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def timed(step, steps, warmup, world):
    """W untimed steps, then K steps bracketed by barrier + synchronize; max over ranks (s)."""
    for i in range(warmup):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        step(warmup + i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    from aonerf import launch

    return launch.max_over_ranks(time.perf_counter() - t0)


def ev_ms(timers, key):
    """(mean ms, rows) of the HIP-event pairs recorded under key."""
    ev = timers.get(key, [])
    if not ev:
        return None, 0
    return float(np.mean([a.elapsed_time(b) for a, b, _ in ev])), ev[0][2]


def bench_render_fp32(args, c2w, focal):
    """The C2 frame on the exact-fp32 MFMA path (v_mfma_f32_16x16x4_f32, no hi/lo emulation):
    the non-emulated reference-precision render, measured by the same protocol on fewer steps."""
    from aonerf.model import NeRF
    from aonerf.parallel import render_frame_sharded
    from aonerf.synthetic import init_like_reference

    net = init_like_reference(NeRF(precision="fp32")).cuda()
    timers = {}
    steps, warmup = min(args.steps, 5), 1

    def step(i):
        render_frame_sharded(net, c2w, H, W, focal, 2.0, 6.0, True,
                             timers=timers if i >= warmup else None)

    el = timed(step, steps, warmup, 1)
    mlp_ms, rows = ev_ms(timers, "mlp1")
    flop = 2.0 * MAC_PER_SAMPLE * rows
    ach = flop / (mlp_ms * 1e-3) / 1e12
    return {"metric": "rays/sec at 640x480x(64c+128f), exact-fp32 MLP (NeRF(precision='fp32'))",
            "value": H * W * steps / el, "unit": "rays/s", "steps": steps, "warmup": warmup,
            "ms_per_step": el / steps * 1e3, "dtype": "fp32 (v_mfma_f32_16x16x4_f32)",
            "roofline": {"bound": "mfma", "kernel": "k_mlp_fwd_f32 (fine level)", "achieved": ach,
                         "peak": PEAK_TFLOPS["fp32"], "unit": "TFLOP/s",
                         "frac": ach / PEAK_TFLOPS["fp32"], "launch_ms": mlp_ms,
                         "algorithmic_flop_per_launch": flop}}


ART_MAC_ISSUED = 714_880    # NeRF_AE_Art MAC per sample the fused kernel issues (latents folded)
ART_MAC_UNFOLDED = 794_880  # the reference's count with the latent columns as GEMM inputs


def bench_articulated(args):
    """C3: NeRF_AE_Art, 320x240 frame, 64c+128f, eval mode, white background, fixed latent
    codes; MFMA roofline of the fine-level fused kernel on the 714,880 MAC per sample it issues
    (the latent products are folded into per-call biases; the reference's unfolded count,
    794,880, is reported as a note only)."""
    from aonerf.model_autodecoder import NeRF_AE_Art
    from aonerf.ray_utils import frame_rays
    from aonerf.render import create_spheric_poses, sapien_focal
    from aonerf.synthetic import art_latents, init_like_reference

    h, w = 240, 320
    net = init_like_reference(NeRF_AE_Art()).cuda()
    lat = art_latents(0, device="cuda")
    rays = frame_rays(torch.as_tensor(create_spheric_poses(4.0)[11]), h, w, sapien_focal(h))
    timers = {}

    @torch.no_grad()
    def step(i):
        return net(rays, False, True, 2.0, 6.0, lat, timers=timers if i >= args.warmup else None)

    el = timed(step, args.steps, args.warmup, 1)
    mlp_ms, rows = ev_ms(timers, "mlp1")
    flop = 2.0 * ART_MAC_ISSUED * rows
    ach = flop / (mlp_ms * 1e-3) / 1e12
    return {"metric": "articulated rays/sec at 320x240x(64c+128f) (NeRF_AE_Art, config C3)",
            "value": h * w * args.steps / el, "unit": "rays/s", "steps": args.steps,
            "ms_per_step": el / args.steps * 1e3,
            "config": {"workload": "sapien_multi NeRF_AE_Art 320x240 frame render, 64c+128f, "
                                   "randomized=False, white_bkgd, fixed latent codes",
                       "rays_per_step": h * w},
            "roofline": {"bound": "mfma", "kernel": "k_mlp_art_f16x3 (fine level)",
                         "achieved": ach, "peak": PEAK_TFLOPS["f16x3"], "unit": "TFLOP/s",
                         "frac": ach / PEAK_TFLOPS["f16x3"], "launch_ms": mlp_ms,
                         "algorithmic_flop_per_launch": flop,
                         "note": "achieved counts the 714,880 MAC/sample the kernel issues (x 3 "
                                 "fp16 products); in the reference's unfolded count (794,880 "
                                 "MAC/sample, latent columns as GEMM inputs) the same launch is "
                                 f"{ach * ART_MAC_UNFOLDED / ART_MAC_ISSUED:.1f} TFLOP/s"}}


# bytes per sample of the training kernels (fp32 activations, SURVEY.md 8(d) extended to C5):
# the fused forward writes raw (16) + 2,432 activations (8 x 256 + 256 + 128) + ReLU' bits
# (9 x 32) and reads t (4); the backward chain reads d raw (16) + the bits and writes 2,432
# input gradients; the weight-gradient GEMMs read each layer's dZ and its input X once.
TRAIN_BYTES = {"fwd_train": 4 + 16 + 4 * 2432 + 288, "bwd_chain": 16 + 288 + 4 * 2432,
               "dweight": 4 * (2432 + 2432 + 63 + 27)}
# FLOP per sample: forward 2 x 593,408; input-gradient chain 2 x (593,408 - 256 x 63 - 128 x 27
# (no gradient into the encodings)); weight gradients 2 x 593,408
TRAIN_FLOP = {"fwd_train": 2 * MAC_PER_SAMPLE, "bwd_chain": 2 * (MAC_PER_SAMPLE - 256 * 63 - 128 * 27),
              "dweight": 2 * MAC_PER_SAMPLE}
# bf16 mode: the kept activations and gradients are 2 B (encodings, d raw and masks unchanged)
# (round 3: the forward also keeps pos_enc(x) as bf16, tiled, 128 columns, read by the two
# enc-column weight gradients)
TRAIN_BYTES_BF16 = {"fwd_train": 4 + 16 + 2 * 2432 + 288 + 2 * 128, "bwd_chain": 16 + 288 + 2 * 2432,
                    "dweight": 2 * (2432 + 2432) + 2 * 2 * 128 + 4 * 27}
# articulated level (NeRF_AE_Art, model_autodecoder.py:168-239), bytes per sample: the fused
# forward writes raw (16) + 3,328 activations (hd 4x128, h 8x256, bot 256, hv 4x128) + pos_enc(x')
# (tiled, 64 columns; ABI 11) + the points (3) + ReLU' bits (16 x 32) and reads t; the chain reads
# d raw + bits + x' (enc's columns 0..2) and writes 3,328 gradients + dL/dx' (3); the weight GEMMs
# read every dZ (3,335) and every layer input once (3,486: activations, enc twice, points, view
# encodings)
ART_TRAIN_BYTES = {"art_fwd_train": 4 + 16 + 4 * (3328 + 64 + 3) + 512,
                   "art_bwd_chain": 16 + 512 + 4 * 3 + 4 * (3328 + 3),
                   "art_dweight": 4 * (3335 + 3486)}
# bf16 mode: the kept activations and chain gradients 2 B (points, d raw, dL/dx' fp32; the fp32
# enc keeps columns 0..15 -- x' for the chain -- beside the bf16 128-column copy)
ART_TRAIN_BYTES_BF16 = {"art_fwd_train": 4 + 16 + 2 * 3328 + 4 * (16 + 3) + 512 + 2 * 128,
                        "art_bwd_chain": 16 + 512 + 4 * 3 + 2 * 3328 + 4 * 3,
                        "art_dweight": 2 * (3328 + 3328) + 2 * 2 * 128 + 4 * (3 + 4 + 3 + 27)}
ART_TRAIN_FLOP = {"art_fwd_train": 2 * 714_880, "art_bwd_chain": 2 * (714_880 - 3 * 128 - 128 * 27),
                  "art_dweight": 2 * 714_880}
# dense MFMA peak in algorithmic FLOP/s per training precision: f16x3 issues 3 fp16 products
# per fp32-class MAC, bf16 one bf16 product
TRAIN_PEAK = {"f16x3": 2500.0 / 3, "bf16": 2500.0}


def bench_train(args, world, rank, local_rank, art=False, precision="f16x3"):
    """C5: one LitNeRF.training_step (or LitNeRF_AutoDecoder.training_step) on 4096 rays per rank
    drawn from 8 synthetic 640x480 views, randomized sampling, loss, HIP backward, gradient
    all-reduce (RCCL, N > 1), fused Adam with the reference schedule.  precision: the model's
    training numerics (train_precision: "f16x3" fp32-class, or C5's "bf16")."""
    import types

    from aonerf import train
    from aonerf.model import NeRF
    from aonerf.parallel import GradAllReduce
    from aonerf.ray_utils import frame_rays
    from aonerf.render import create_spheric_poses, sapien_focal
    from aonerf.synthetic import init_like_reference

    dev = torch.device("cuda", torch.cuda.current_device())  # (gloo ranks may share one GPU)
    nrays = 4096
    if art:
        from aonerf import train_art
        from aonerf.code_library import CodeLibraryArticulated
        from aonerf.model_autodecoder import NeRF_AE_Art
        from aonerf.synthetic import init_code_library

        net = init_like_reference(NeRF_AE_Art(train_precision=precision)).to(dev)
        lib = init_code_library(CodeLibraryArticulated(
            types.SimpleNamespace(N_max_objs=151, N_obj_code_length=128))).to(dev)
        ids = {"instance_id": torch.tensor([7], device=dev),
               "articulation_id": torch.tensor([3], device=dev)}
    else:
        net = init_like_reference(NeRF(train_precision=precision)).to(dev)
    poses = create_spheric_poses(4.0)
    focal = sapien_focal(H)
    views = [frame_rays(torch.as_tensor(poses[(5 * k) % len(poses)]), H, W, focal) for k in range(8)]
    rays_all = {key: torch.cat([v[key] for v in views], 0) for key in ("rays_o", "rays_d", "viewdirs")}
    rng = np.random.Generator(np.random.PCG64(3))
    target_all = torch.from_numpy(rng.uniform(0, 1, size=(8 * H * W, 3)).astype(np.float32)).to(dev)
    gen = torch.Generator(device=dev).manual_seed(1000 + rank)
    params = list(net.parameters()) + (list(lib.parameters()) if art else [])
    opt = train.Adam(params)
    # C5's bf16 mode averages its gradients in bf16 (half the bytes on xGMI); two buckets: the
    # fine MLP's all-reduce is issued from its gradient hooks as soon as the fine level's backward
    # (autograd's first) has landed them, and runs beside the coarse level's backward
    fine = list(net.fine_mlp.parameters())
    fine_ids = {id(p) for p in fine}
    sync = GradAllReduce(params, dtype=torch.bfloat16 if precision == "bf16" else torch.float32,
                         buckets=[fine, [p for p in params if id(p) not in fine_ids]])
    timers = {}

    def step(i):
        tm = timers if i >= args.warmup else None
        idx = torch.randint(0, 8 * H * W, (nrays,), device=dev, generator=gen)
        batch = {k: v[idx] for k, v in rays_all.items()}
        batch["target"] = target_all[idx]
        opt.zero_grad()
        if art:
            batch.update(ids)
            loss, _ = train_art.training_step(net, lib, batch, True, True, 2.0, 6.0, timers=tm)
        else:
            loss, _ = train.training_step(net, batch, True, True, 2.0, 6.0, timers=tm)
        loss.backward()
        sync()
        opt.step(lr=train.learning_rate(i, 200000))

    try:
        el = timed(step, args.steps, args.warmup, world)
    finally:
        sync.close()
    ddp = None
    if world > 1:
        # the all-reduce is part of every timed step: the ranks draw different batches, so their
        # parameters stay identical after Adam only if every step averaged the gradients
        import hashlib

        flat = torch.cat([p.detach().reshape(-1).float() for p in params]).cpu().numpy()
        digests = [None] * world
        dist.all_gather_object(digests, hashlib.sha256(flat.tobytes()).hexdigest())
        ddp = {"collective": "GradAllReduce (two buckets per step: the fine MLP's issued from "
                             "its gradient hooks, overlapping the coarse level's backward)",
               "backend": dist.get_backend(), "world": world,
               "bucket_dtype": "bf16" if precision == "bf16" else "fp32",
               "bucket_values": sum(sync.sizes), "buckets": len(sync.spans), "calls": sync.calls,
               "params_identical_across_ranks": len(set(digests)) == 1,
               "param_sha256_rank0": digests[0]}
    mac = ART_MAC_ISSUED if art else MAC_PER_SAMPLE
    samples = nrays * (NC + 1 + NC + 1 + NF)
    ms = el / args.steps * 1e3
    step_flop = 3 * 2.0 * mac * samples
    ach = step_flop / (ms * 1e-3) / 1e12
    rec = {"metric": ("training rays/sec, LitNeRF_AutoDecoder.training_step (NeRF_AE_Art), "
                      "4096 rays/rank, 64c+128f, Adam (config C5)" if art else
                      "training rays/sec, LitNeRF.training_step, 4096 rays/rank, 64c+128f, "
                      "Adam (config C5)"),
           "value": nrays * world * args.steps / el, "unit": "rays/s", "n_gpus": world,
           "steps": args.steps, "ms_per_step": ms, "scaling": "weak",
           "dtype": ("bf16 (bf16 MFMA, fp32 accumulate; the deformation MLP's forward f16x3 for x'; "
                     "bf16 activations and gradients, fp32 compositing / loss / Adam master "
                     "weights)" if precision == "bf16" and art else
                     "bf16 (bf16 MFMA, fp32 accumulate; bf16 activations and gradients, fp32 "
                     "compositing / loss / Adam master weights)" if precision == "bf16" else
                     "f16x3 (fp16 hi/lo split MFMA, fp32 accumulate; fp32 activations)"),
           "config": {"workload": "C5 training step" + (" (articulated)" if art else ""),
                      "rays_per_rank": nrays, "parallelism": f"ddp{world}" if world > 1 else "single GPU",
                      "grad_allreduce_dtype": "bf16" if precision == "bf16" else "fp32"},
           "roofline": {"bound": "hbm+mfma", "kernel": "whole step (3 x forward FLOP)",
                        "achieved": ach, "peak": TRAIN_PEAK[precision], "unit": "TFLOP/s",
                        "frac": ach / TRAIN_PEAK[precision]}}
    if ddp is not None:
        rec["ddp"] = ddp
    if art and precision == "bf16":
        rec["roofline"]["note"] = ("the articulated bf16 mode keeps its forward in fp16x3 "
                                   "(TrainNumerics.art_forward 'f16_acts': 2 fp16 products per "
                                   "MAC past the deformation MLP, which is fp16x3); frac is "
                                   "against the bf16 peak for the whole step")
    kern = {}
    hbm_bytes = 0.0
    names = ("art_fwd_train", "art_bwd_chain", "art_dweight") if art else ("fwd_train", "bwd_chain", "dweight")
    nbytes = ((ART_TRAIN_BYTES_BF16 if precision == "bf16" else ART_TRAIN_BYTES) if art else
              TRAIN_BYTES_BF16 if precision == "bf16" else TRAIN_BYTES)
    nflop = ART_TRAIN_FLOP if art else TRAIN_FLOP
    for name in names:
        t_ms, rows = ev_ms(timers, f"{name}{NC + 1 + NF}")
        if not t_ms:
            continue
        b, f = nbytes[name] * rows, nflop[name] * rows
        hbm_bytes += b
        kern[name] = {"level": "fine", "ms": t_ms, "rows": rows,
                      "algorithmic_bytes": b, "GB/s": b / (t_ms * 1e-3) / 1e9,
                      "hbm_frac": b / (t_ms * 1e-3) / 1e9 / PEAK_HBM_GBS,
                      "TFLOP/s": f / (t_ms * 1e-3) / 1e12,
                      "mfma_frac": f / (t_ms * 1e-3) / 1e12 / TRAIN_PEAK[precision]}
    rec["roofline"]["kernels"] = kern
    if kern:
        tot_ms = sum(k["ms"] for k in kern.values())
        rec["roofline"]["fine_level_hbm_frac"] = hbm_bytes / (tot_ms * 1e-3) / 1e9 / PEAK_HBM_GBS
        rec["roofline"]["fine_level_ms"] = tot_ms
    return rec


def cpu_baseline(net, frame, c2w, focal, nchunks):
    """The oracle (torch CPU restatement of the reference path) on nchunks x 3840 rays of the
    same frame, timed on the host cores; then the parity of the GPU frame on those rays at the
    headline config, on IDENTICAL rays (the oracle takes the GPU's rays; a1/a2 are bit-exact
    against the reference's golden rays in tests): the fraction within 1e-4 per rgb / acc /
    depth against the reference's own self-consistency on the same rays (verdict r05 #1: the
    oracle re-run with its GEMMs split-K, oracle/attribution.py self_consistency; gate = that
    fraction less max(0.1 pp, 3 binomial standard errors)), and every outlier attributed
    (plateau flip, amplification, or the reference's own implementation envelope on that ray) --
    `unattributed` must be 0."""
    from oracle import attribution as A
    from oracle import nerf_oracle as O
    from oracle import weights as Wt

    from aonerf.ray_utils import frame_rays

    # The host's CPU share of this one-GPU job: the pool gives a one-GPU box 16 CPUs
    # (OMP_NUM_THREADS=16 there) of a host whose os.cpu_count() spans every GPU's share; the
    # affinity mask / OMP_NUM_THREADS name that share, so that is what the baseline uses.
    share = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = min(share, omp) if omp > 0 else share
    torch.set_num_threads(threads)
    params = O.split_state_dict(Wt.nerf_state_dict(0))
    n = 3840 * nchunks
    p0 = (H * W) // 2 - n // 2  # centre rows (object region)
    rays = frame_rays(c2w, H, W, focal, p0=p0, n=n)  # the GPU's rays: identical inputs
    rc = {k: v.cpu() for k, v in rays.items()}
    dirs = O.get_ray_directions(H, W, focal)
    _, _, rd_host = O.get_rays(dirs, c2w[:3, :4], True)
    def progress(what):  # (stderr: the JSON line stays alone on stdout)
        return lambda i, m: print(f"[bench] cpu_baseline {what}: {i} / {m} rays", file=sys.stderr,
                                  flush=True)

    t0 = time.perf_counter()
    outs, w_ref = [], []
    with torch.no_grad():
        for i in range(0, n, 3840):
            sub = {k: v[i:i + 3840] for k, v in rc.items()}
            ret, inter = O.nerf_forward(params, sub, False, True, 2.0, 6.0, return_intermediates=True)
            outs.append(ret[1])
            w_ref.append(inter[0]["weights"])
            progress("oracle")(i + 3840, n)
    dt = time.perf_counter() - t0
    ref = [torch.cat([o[j] for o in outs]).numpy() for j in range(3)]  # rgb, acc, depth
    w_ref = torch.cat(w_ref).numpy()
    # the reference's self-consistency on the same rays (another valid fp32 implementation)
    t1 = time.perf_counter()
    selfc = A.self_consistency(params, rc, ref, progress=progress(A.SELF_VARIANT + " re-run"))
    dt_self = time.perf_counter() - t1
    f = frame[p0:p0 + n].cpu().numpy()
    gpu = [f[:, :3], f[:, 4], f[:, 3]]
    # our coarse weights and fine samples on the same rays (the frame's kernels; checked equal)
    with torch.no_grad():
        mine = net(rays, False, True, 2.0, 6.0, return_weights=True, return_intermediates=True)
    subset_equal = all(np.array_equal(mine[1][j].cpu().numpy(), gpu[j]) for j in range(3))
    w_ours = mine[0][3].cpu().numpy()
    t_fine = mine[1][4]["t_vals"].cpu()
    errs = [np.abs(g.astype(np.float64) - r.astype(np.float64)) for g, r in zip(gpu, ref)]
    names = ("rgb", "acc", "depth")
    ours = A.fractions(gpu, ref)
    bad = np.zeros(n, bool)
    for e in errs:
        bad |= (e > A.E2E_ATOL).reshape(n, -1).any(-1)
    rows = np.nonzero(bad)[0]
    floors = {k: A.e2e_floor(selfc[k]["frac"], n) for k in names}
    parity = {"rays": n, "atol": A.E2E_ATOL, "gpu_subset_equals_frame": bool(subset_equal),
              "inputs": "identical rays: the oracle takes the GPU's rays (a1/a2 bit-exact vs the "
                        "reference's golden rays in tests)",
              "ray_generation_host_torch_differs": int(
                  (rays["rays_d"].cpu().numpy() != rd_host[p0:p0 + n].numpy()).any(-1).sum()),
              "max_abs": {k: float(e.max()) for k, e in zip(names, errs)},
              "frac_within_1e-4": {k: ours[k]["frac"] for k in names},
              "outliers": {k: ours[k]["outliers"] for k in names},
              "reference_self_variant": A.SELF_VARIANT + " (the oracle's GEMMs split-K: an fp32-cost "
                                        "re-implementation of the reference)",
              "reference_self_frac_within_1e-4": {k: selfc[k]["frac"] for k in names},
              "reference_self_outliers": {k: selfc[k]["outliers"] for k in names},
              "reference_self_s": dt_self,
              "floors": floors,
              "gate": "ours >= reference self fraction - max(0.1 pp, 3 binomial s.e.)",
              "gate_pass": all(ours[k]["frac"] >= floors[k] for k in names),
              "outlier_rays": int(len(rows)), "attributed": {}, "unattributed": 0}
    if len(rows):
        sub = {k: v[rows] for k, v in rc.items()}
        rgb_o, acc_o, _, depth_o = O.render_level(params, sub, t_fine[rows], 1, True)
        on_ours = [rgb_o.numpy(), acc_o.numpy(), depth_o.numpy()]
        env, worst = A.fine_envelope(params, sub)
        att = A.Attribution(w_ours[rows], w_ref[rows], NF)
        why = {}
        lines = []
        unexplained = np.zeros(len(rows), bool)
        for j, k in enumerate(names):
            e = errs[j][rows]
            ok = att.rays(on_ours[j], ref[j][rows], e, env[j])
            out_q = (e > A.E2E_ATOL).reshape(len(rows), -1).any(-1)
            unexplained |= out_q & ~ok
            for w in att.why[out_q & ok]:
                why[w] = why.get(w, 0) + 1
            top = np.argsort(-e.reshape(len(rows), -1).max(-1))[:3]
            mask = np.zeros(len(rows), bool)
            mask[top] = True
            lines += att.explain(f"bench {k}", e, ok & mask, limit=3,
                                 out=lambda ln: print(ln, file=sys.stderr))
        parity["attributed"] = why  # per criterion, counted per (ray, quantity)
        parity["envelope_attributed_flag"] = why.get("implementation envelope", 0) > max(5, len(rows) // 10)
        parity["unattributed"] = int(unexplained.sum())
        parity["worst"] = lines[:3]
        parity["envelope_max_by_variant"] = {f"{v}/{q}": x for (v, q), x in sorted(worst.items())}
    target = torch.from_numpy(np.random.Generator(np.random.PCG64(3)).uniform(0, 1, (n, 3)).astype(np.float32))
    g_rgb, r_rgb = torch.from_numpy(gpu[0].copy()), torch.from_numpy(ref[0])
    p_ref = O.psnr_each([r_rgb], [target]).item()
    p_gpu = O.psnr_each([g_rgb], [target]).item()
    model = ""
    try:
        with open("/proc/cpuinfo") as fh:
            model = next((ln.split(":", 1)[1].strip() for ln in fh if ln.startswith("model name")), "")
    except OSError:
        pass
    return {"value": n / dt, "unit": "rays/s", "cores": threads, "kind": "port",
            "cpu_model": model, "host_cpu_count": os.cpu_count(),
            "sample": f"{nchunks} x 3840-ray chunks (pixels {p0}..{p0 + n}) of the same frame, "
                      f"oracle/nerf_oracle.py torch-CPU restatement, {threads} threads, {dt:.1f} s",
            "threads_rationale": "the job's CPU share: min(affinity mask, OMP_NUM_THREADS); the "
                                 "GPU box gives a one-GPU job 16 CPUs of the shared host",
            "max_abs_rgb_diff_vs_gpu": float(errs[0].max()),
            "psnr_gpu_vs_reference_db": O.psnr_each([g_rgb], [r_rgb]).item(),
            "psnr_delta_db": p_gpu - p_ref, "parity": parity}


if __name__ == "__main__":
    main()
