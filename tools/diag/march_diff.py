"""Debug: where aon_composite_march's fine t differs from aon_composite_fwd + aon_sample_pdf."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "articulated-object-nerf_amd"))
import torch  # noqa: E402

from aonerf import _lib as L  # noqa: E402
from aonerf import helper  # noqa: E402

g = torch.Generator().manual_seed(65128)
B, S, Ns = 16, 65, 128
t = torch.sort(2.0 + 4.0 * torch.rand((B, S), generator=g), -1).values.cuda()
raw = torch.cat([torch.randn((B, S, 3), generator=g), 3.0 * torch.randn((B, S, 1), generator=g)], -1).reshape(-1, 4).cuda()
dirs = torch.randn((B, 3), generator=g).cuda()
u, us = helper.eval_u(Ns, "cuda"), 0
two = [torch.empty(s, device="cuda") for s in ((B, 3), (B,), (B, S), (B,))]
L.call("aon_composite_fwd", L.ptr(raw), 4, L.ptr(raw[:, 3:]), 4, L.ptr(t), L.ptr(dirs), B, S, 1,
       L.ACT_VANILLA, *[L.ptr(o) for o in two], L.stream())
t2 = torch.empty((B, S + Ns), device="cuda")
L.call("aon_sample_pdf", None, 0, L.ptr(two[2][:, 1:]), S, B, S - 1, Ns, L.ptr(u), us, L.ptr(t), S,
       None, None, L.ptr(t2), None, L.stream())
pdf_only = torch.empty((B, Ns), device="cuda")
L.call("aon_sample_pdf", None, 0, L.ptr(two[2][:, 1:]), S, B, S - 1, Ns, L.ptr(u), us, L.ptr(t), S,
       None, None, L.ptr(pdf_only), None, L.stream()) if False else None
one = [torch.empty(s, device="cuda") for s in ((B, 3), (B,), (B, S), (B,))]
t1 = torch.empty((B, S + Ns), device="cuda")
L.call("aon_composite_march", L.ptr(raw), L.ptr(t), L.ptr(dirs), B, S, 1, L.ACT_VANILLA, L.ptr(u),
       us, Ns, L.ptr(one[0]), L.ptr(one[1]), L.ptr(one[2]), L.ptr(one[3]), L.ptr(t1), L.stream())
torch.cuda.synchronize()
print("weights equal", torch.equal(one[2], two[2]))
d = (t1 != t2)
print("rays with diffs", d.any(1).nonzero().flatten().tolist())
for r in d.any(1).nonzero().flatten().tolist()[:3]:
    idx = d[r].nonzero().flatten().tolist()
    print("ray", r, "n diff", len(idx), "first", idx[:20])
    print("  march", t1[r, idx[:8]].tolist())
    print("  two  ", t2[r, idx[:8]].tolist())
    print("  sorted march row?", bool((t1[r, 1:] >= t1[r, :-1]).all()), "equal as sets?",
          torch.equal(t1[r].sort().values, t2[r].sort().values))
