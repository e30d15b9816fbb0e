"""Timing driver (GPU): the fused training forwards alone at config C5's fine level (4,096 rays x
193 samples), each mode timed with HIP events over --reps launches.  Run it once with the
release library and once with a timing-only build whose forwards keep nothing
(-DAON_ABL_NO_KEEP, AONERF_LIB=...) to read what the kept-tensor stores cost:

    python tools/prof_fwd_keep.py [--reps 20]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "articulated-object-nerf_amd")):
    sys.path.insert(0, p)
if os.environ.get("AONERF_LIB"):  # an A/B build of the library (tools only)
    from aonerf import _lib as _aon_lib  # noqa: E402

    _aon_lib.use_library(os.environ["AONERF_LIB"])
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    from aonerf import tiles, train, train_art
    from aonerf.model import NeRF
    from aonerf.model_autodecoder import NeRF_AE_Art
    from aonerf.synthetic import art_latents, init_like_reference

    dev = torch.device("cuda")
    B, S = 4096, 193
    R = B * S
    g = torch.Generator(device=dev).manual_seed(5)
    d = torch.nn.functional.normalize(torch.randn(B, 3, device=dev, generator=g), dim=-1)
    o = -4.0 * d + 0.1 * torch.randn(B, 3, device=dev, generator=g)
    t = (2.0 + 4.0 * torch.rand(B, S, device=dev, generator=g)).sort(-1).values.contiguous()
    raw = torch.empty((R, 4), device=dev)
    net = init_like_reference(NeRF()).to(dev)
    P = [(m.weight.detach(), m.bias.detach()) for m in net.fine_mlp._layers()]
    art = init_like_reference(NeRF_AE_Art()).to(dev)
    mlp = art.fine_mlp
    geo = train_art._Geo(mlp)
    PA = [(m.weight.detach(), m.bias.detach()) for m in train_art.art_layers(mlp)]
    lat_d = art_latents(0, device=dev)
    lat = tuple(lat_d[k].reshape(1, -1).contiguous() for k in ("density", "color", "articulation"))
    masks9 = torch.empty((9, tiles.rows(R), 8), dtype=torch.int32, device=dev)
    masks16 = torch.empty((16, tiles.rows(R), 8), dtype=torch.int32, device=dev)
    enc_bf = torch.empty((tiles.rows(R), 128), device=dev, dtype=torch.bfloat16)
    modes = {
        "fwd_train_f16x3": lambda: train._forward_level_fused(P, o, d, d, t, raw, None, masks9),
        "fwd_train_bf16": lambda: train._forward_level_fused(P, o, d, d, t, raw, None, masks9,
                                                             bf16=True, enc=enc_bf),
        "art_fwd_train_f16x3": lambda: train_art._forward_level_fused(geo, PA, lat, o, d, d, t, raw,
                                                                      None, masks16),
        "art_fwd_train_bf16": lambda: train_art._forward_level_fused(geo, PA, lat, o, d, d, t, raw,
                                                                     None, masks16, bf16=True,
                                                                     enc_bf=enc_bf),
    }
    out = {"lib": os.environ.get("AONERF_LIB", "release"), "rows": R}
    for name, fn in modes.items():
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out[name] = round(e0.elapsed_time(e1) / args.reps, 4)  # ms per call (pack + kernel)
        print(name, out[name], "ms", flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
