"""A/B helper (GPU): sha256 of every output of one bf16 training step (vanilla NeRF and the
articulated auto-decoder, both forward numerics) on C5's batch with injected uniforms, plus the
mean step time over 10 steps -- run once per library build (AONERF_LIB=...) and diff the JSON
lines: a numerics-preserving kernel change must leave every sha unchanged.

    AONERF_LIB=articulated-object-nerf_amd/lib/variants/libaonerf_X.so python tools/diag/bf16_ab_outputs.py
"""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "articulated-object-nerf_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
if os.environ.get("AONERF_LIB"):  # an A/B build of the library (tools only)
    from aonerf import _lib as _aon_lib  # noqa: E402

    _aon_lib.use_library(os.environ["AONERF_LIB"])
import torch  # noqa: E402


def sha(t):
    return hashlib.sha256(t.detach().contiguous().cpu().numpy().tobytes()).hexdigest()[:16]


def main():
    from test_gpu_art_train import _make
    from test_gpu_train import _make_trainable, c5_batch

    from aonerf import train, train_art
    out = {"lib": os.environ.get("AONERF_LIB", "default")}
    batch, u_c, u_f = c5_batch(seed=12)
    # vanilla
    net = _make_trainable(0, precision="bf16")
    ret = net(batch, True, True, 2.0, 6.0, u_coarse=u_c, u_fine=u_f)
    loss = train.img2mse(ret[1][0], batch["target"]) + train.img2mse(ret[0][0], batch["target"])
    loss.backward()
    torch.cuda.synchronize()
    out["vanilla"] = {"loss": sha(loss), **{n: sha(p.grad) for n, p in net.named_parameters()}}
    opt = train.Adam(net.parameters())
    for i in range(13):
        if i == 3:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        opt.zero_grad()
        ls, _ = train.training_step(net, batch, True, True, 2.0, 6.0)
        ls.backward()
        opt.step()
    torch.cuda.synchronize()
    out["vanilla_ms"] = 1e3 * (time.perf_counter() - t0) / 10
    # articulated
    batch["instance_id"] = torch.tensor([7], device="cuda")
    batch["articulation_id"] = torch.tensor([3], device="cuda")
    for trunk in (False, True):
        net, lib = _make(0, precision="bf16", art_forward="bf16_trunk" if trunk else "f16x3")
        latents = lib(batch)
        ret = net(batch, True, True, 2.0, 6.0, latents, u_coarse=u_c, u_fine=u_f)
        loss = train_art.img2mse(ret[1][0], batch["target"]) + train_art.img2mse(ret[0][0], batch["target"])
        loss.backward()
        torch.cuda.synchronize()
        key = f"art_trunk{int(trunk)}"
        out[key] = {"loss": sha(loss), **{n: sha(p.grad) for n, p in net.named_parameters()},
                    **{n: sha(p.grad) for n, p in lib.named_parameters()}}
        opt = train_art.configure_optimizers(net, lib)
        for i in range(13):
            if i == 3:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
            opt.zero_grad()
            ls, _ = train_art.training_step(net, lib, batch, True, True, 2.0, 6.0)
            ls.backward()
            opt.step()
        torch.cuda.synchronize()
        out[key + "_ms"] = 1e3 * (time.perf_counter() - t0) / 10
    print(json.dumps(out))


if __name__ == "__main__":
    main()
