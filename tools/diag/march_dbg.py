"""Debug build check: k_march_rows' weight sum / CDF against the oracle's (torch) on 8 rays."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "articulated-object-nerf_amd"))
sys.path.insert(0, ROOT)
os.environ["AONERF_LIB"] = os.path.join(ROOT, "articulated-object-nerf_amd/lib/variants/libaonerf_dbg.so")
if os.environ.get("AONERF_LIB"):  # an A/B build of the library (tools only)
    from aonerf import _lib as _aon_lib  # noqa: E402

    _aon_lib.use_library(os.environ["AONERF_LIB"])
import torch  # noqa: E402

from aonerf import _lib as L  # noqa: E402
from aonerf import helper  # noqa: E402
from oracle import nerf_oracle as O  # noqa: E402

g = torch.Generator().manual_seed(65128)
B, S, Ns = 8, 65, 128
t = torch.sort(2.0 + 4.0 * torch.rand((B, S), generator=g), -1).values.cuda()
raw = torch.cat([torch.randn((B, S, 3), generator=g), 3.0 * torch.randn((B, S, 1), generator=g)], -1).reshape(-1, 4).cuda()
dirs = torch.randn((B, 3), generator=g).cuda()
u = helper.eval_u(Ns, "cuda")
two = [torch.empty(s, device="cuda") for s in ((B, 3), (B,), (B, S), (B,))]
L.call("aon_composite_fwd", L.ptr(raw), 4, L.ptr(raw[:, 3:]), 4, L.ptr(t), L.ptr(dirs), B, S, 1,
       L.ACT_VANILLA, *[L.ptr(o) for o in two], L.stream())
one = [torch.empty(s, device="cuda") for s in ((B, 3), (B,), (B, S), (B,))]
t1 = torch.empty((B, S + Ns), device="cuda")
L.call("aon_composite_march", L.ptr(raw), L.ptr(t), L.ptr(dirs), B, S, 1, L.ACT_VANILLA, L.ptr(u), 0,
       Ns, L.ptr(one[0]), L.ptr(one[1]), L.ptr(one[2]), L.ptr(one[3]), L.ptr(t1), L.stream())
torch.cuda.synchronize()
w = two[2].cpu()[:, 1:-1]
ws = w.sum(-1)
cdf, _, _ = O._pdf_bins(w, Ns, False)
dbg = one[2].cpu()
for r in range(B):
    print(r, "ws kernel", dbg[r, 0].item(), "torch", ws[r].item(), "eq", dbg[r, 0].item() == ws[r].item(),
          "| cdf mismatches", int((dbg[r, 3:65] != cdf[r, 1:63]).sum()),
          "first", (dbg[r, 3:65] != cdf[r, 1:63]).nonzero().flatten()[:5].tolist())
