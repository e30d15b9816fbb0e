"""sha256 of every gradient of one articulated C5 training step (MLPs + code library) -- run under
two library builds (AONERF_LIB=...) to show they compute the same bits.
    python tools/diag/art_grad_sha.py [--precision bf16|f16x3]"""
import argparse
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "articulated-object-nerf_amd"), os.path.join(ROOT, "tests")]
if os.environ.get("AONERF_LIB"):  # an A/B build of the library (tools only)
    from aonerf import _lib as _aon_lib  # noqa: E402

    _aon_lib.use_library(os.environ["AONERF_LIB"])
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="bf16")
    args = ap.parse_args()
    from test_gpu_art_train import _make
    from test_gpu_train import c5_batch

    from aonerf import train_art
    batch, u_c, u_f = c5_batch(seed=12)
    batch["instance_id"] = torch.tensor([7], device="cuda")
    batch["articulation_id"] = torch.tensor([3], device="cuda")
    net, lib = _make(0, precision=args.precision)
    loss, _ = train_art.training_step(net, lib, batch, True, True, 2.0, 6.0, u_coarse=u_c, u_fine=u_f)
    loss.backward()
    h = hashlib.sha256()
    for name, p in list(net.named_parameters()) + list(lib.named_parameters()):
        if p.grad is not None:
            h.update(p.grad.detach().cpu().numpy().tobytes())
    print(f"art {args.precision} loss {loss.item():.9g} grads sha256 {h.hexdigest()}", flush=True)


if __name__ == "__main__":
    main()
