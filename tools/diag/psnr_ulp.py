"""Which fp32 arithmetic torch's mse2psnr (helper.py:21-22) performs on the device: prints the
stages for a few mse values against candidate restatements (aon_loss_pair's psnr)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "articulated-object-nerf_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from aonerf import train  # noqa: E402

f32 = np.float32
for seed in (4096, 1000, 1, 7, 11):
    g = torch.Generator(device="cuda").manual_seed(seed)
    p0 = torch.rand((seed, 3), device="cuda", generator=g)
    p1 = torch.rand((seed, 3), device="cuda", generator=g)
    tgt = torch.rand((seed, 3), device="cuda", generator=g)
    u0 = train.img2mse(p0, tgt).detach()
    _, _, _, s0, _ = train.loss_pair(p0, p1, tgt)
    lg = torch.log(u0)
    m10 = -10.0 * lg
    want = train.mse2psnr(u0)
    x = f32(u0.item())
    lg_np = f32(np.log(np.float64(x)))
    inv = f32(1.0) / f32(np.log(10.0))
    cands = {
        "mul_inv(torch log)": f32(f32(f32(-10.0) * f32(lg.item())) * inv),
        "div(torch log)": f32(f32(f32(-10.0) * f32(lg.item())) / f32(np.log(10.0))),
        "mul_inv(f64 log)": f32(f32(f32(-10.0) * lg_np) * inv),
        "div(f64 log)": f32(f32(f32(-10.0) * lg_np) / f32(np.log(10.0))),
        "f64 all": f32(-10.0 * np.log(np.float64(x)) / np.log(10.0)),
    }
    print(f"mse {x!r}: torch log {lg.item()!r} (f64-rounded {lg_np!r}), -10 log {m10.item()!r}, "
          f"torch psnr {want.item()!r}, kernel {s0.item()!r}")
    for k, v in cands.items():
        print(f"   {k:20s} {v!r} {'==' if v == f32(want.item()) else '!='}")
