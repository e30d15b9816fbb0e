"""A/B variant builds beside the release library (aonerf._lib.variant): the weight-streamed
render dataflow (mlp_ws.hip, `make -C csrc variant-ws`) must give the release kernels' outputs
bit for bit -- same products, same accumulation order, same epilogue -- and keep the fp16x3
range guard.  The variant shares the ABI and the packed formats, so one pack (release library)
feeds both; the release library has no run-time kernel selection (ABI 9)."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ws():
    from aonerf import _lib as L

    import os

    path = os.path.join(os.path.dirname(L.LIB_PATH), "variants", "libaonerf_ws.so")
    if not os.path.exists(path):  # an A/B build, not made by build()
        pytest.skip("variant library not built (make -C articulated-object-nerf_amd/csrc variant-ws)")
    return L.variant("ws")


def _fwd(handle, name, *args):
    from aonerf import _lib as L

    st = getattr(handle, name)(*args)
    if st != 0:
        raise RuntimeError(f"{name}: {handle.aon_last_error().decode()}")


def _rays(B, S, seed):
    g = torch.Generator().manual_seed(seed)
    o = (torch.randn(B, 3, generator=g) * 0.1 + torch.tensor([0.0, -3.5, 2.0])).cuda()
    d = torch.nn.functional.normalize(torch.randn(B, 3, generator=g), dim=-1).cuda()
    t = torch.sort(torch.rand(B, S, generator=g) * 4 + 2, dim=-1).values.cuda()
    return o, d, t


@pytest.mark.parametrize("B,S,act", [(1000, 65, 0), (1237, 193, 1), (3, 193, 2), (1, 1, 0)])
def test_mlp_ws_equals_streamed(B, S, act):
    """aon_mlp_fwd: release (LDS-ring weight stream, mlp_f16x3.hip) vs the weight-streamed
    variant on ragged sample counts (partial 128-sample workgroups, one sample), every
    activation mode."""
    from aonerf import _lib as L
    from aonerf.model import NeRF
    from aonerf.synthetic import init_like_reference

    o, d, t = _rays(B, S, B + S)
    mlp = init_like_reference(NeRF()).cuda().fine_mlp
    a = mlp.forward_rays(o, d, d, t, act)
    b = torch.empty_like(a)
    _fwd(_ws(), "aon_mlp_fwd", L.ptr(mlp.packed_weights()), L.PREC["f16x3"], L.ptr(o), L.ptr(d),
         L.ptr(d), L.ptr(t), B, S, act, L.ptr(b), L.stream())
    torch.cuda.synchronize()
    assert torch.equal(a, b), (a - b).abs().max().item()
    assert torch.isfinite(b).all()


@pytest.mark.parametrize("B,S", [(517, 65), (300, 193), (1, 1)])
def test_art_mlp_ws_equals_streamed(B, S):
    """aon_mlp_art_fwd: release (mlp_art.hip) vs the weight-streamed variant."""
    from aonerf import _lib as L
    from aonerf.model_autodecoder import NeRF_AE_Art
    from aonerf.synthetic import art_latents, init_like_reference

    o, d, t = _rays(B, S, B + S)
    mlp = init_like_reference(NeRF_AE_Art()).cuda().fine_mlp
    lat = art_latents(0, device="cuda")
    a = mlp.forward_rays(o, d, d, t, lat)
    b = torch.empty_like(a)
    _fwd(_ws(), "aon_mlp_art_fwd", L.ptr(mlp.packed_weights(lat)), L.ptr(o), L.ptr(d), L.ptr(d),
         L.ptr(t), B, S, 0, L.ptr(b), L.stream())
    torch.cuda.synchronize()
    assert torch.equal(a, b), (a - b).abs().max().item()


@pytest.mark.parametrize("target,status", [(6.0e3, 0), (1.2e4, 1)])
def test_ws_dataflow_range_guard(golden, target, status):
    """The weight-streamed kernel keeps the range guard: status 0 inside fp16x3's range, 1 when a
    hidden activation leaves it -- and its raw outputs equal the release kernel's either way."""
    from aonerf import _lib as L
    from test_gpu_range import _net, _scaled

    g, sd, _, m = _scaled(golden, target)
    net = _net(sd)
    rays = {k: torch.from_numpy(g[k]).cuda() for k in ("rays_o", "rays_d", "viewdirs")}
    t = torch.from_numpy(np.ascontiguousarray(g["coarse_t"])).cuda()
    B, S = t.shape
    mlp = net.coarse_mlp
    outs, stats = [], []
    for handle in (None, _ws()):
        mlp._packed_key = None  # a fresh pack: status word cleared
        packed = mlp.packed_weights()
        if handle is None:
            out = mlp.forward_rays(rays["rays_o"], rays["rays_d"], rays["viewdirs"], t)
        else:
            out = torch.empty((B * S, 4), device="cuda")
            _fwd(handle, "aon_mlp_fwd", L.ptr(packed), L.PREC["f16x3"], L.ptr(rays["rays_o"]),
                 L.ptr(rays["rays_d"]), L.ptr(rays["viewdirs"]), L.ptr(t), B, S, 0, L.ptr(out),
                 L.stream())
        st = ctypes.c_uint32(7)
        L.call("aon_mlp_read_status", L.ptr(packed), packed.numel() * 4, ctypes.byref(st),
               L.stream(packed.device))
        outs.append(out)
        stats.append(st.value)
    print(f"largest hidden activation {m:.1f}: status release {stats[0]}, weight-streamed {stats[1]}")
    assert stats == [status, status]
    assert torch.equal(outs[0], outs[1])
