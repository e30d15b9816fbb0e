"""The compositor's transcendentals against the reference's own CPU arithmetic.

The reference evaluates, on CPU torch:
  - rgb = torch.sigmoid(raw) (model.py:186) -- ATen's vectorised 1/(1 + exp(-x)) with SLEEF's
    expf (u10).  Our act_rgb restates that exp (aon_common.hpp exp_sleef), so the result must be
    bit-identical to torch.sigmoid;
  - alpha = 1 - torch.exp(-sigma * dist) (helper.py:171) -- MKL's vsExp (high accuracy).  Our
    exp_cr is the correctly rounded fp32 exp: bit-identical to numpy's fp64 exp rounded to fp32,
    and equal to torch.exp except where MKL itself is not correctly rounded (~1% of elements,
    never more than 1 ulp of exp apart).
Probed through aon_composite_fwd with rays built so the outputs ARE the activations:
S = 1 (dist = 1e10 -> alpha = 1, weight 1, comp = rgb exactly, no white background) for the
sigmoid, and S = 2 with t = [0, 1], |d| = 1 (weights[:, 0] = alpha_0 exactly) for the exp.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N = 1 << 20


def _composite(rgb, sigma, t, dirs, act):
    from aonerf import _lib as L
    B, S = t.shape
    comp = torch.empty((B, 3), device="cuda")
    acc = torch.empty((B,), device="cuda")
    w = torch.empty((B, S), device="cuda")
    depth = torch.empty((B,), device="cuda")
    L.call("aon_composite_fwd", L.ptr(rgb), 3, L.ptr(sigma), 1, L.ptr(t), L.ptr(dirs), B, S, 0,
           act, L.ptr(comp), L.ptr(acc), L.ptr(w), L.ptr(depth), L.stream(rgb.device))
    torch.cuda.synchronize()
    return comp.cpu(), w.cpu()


def test_sigmoid_bit_identical_to_torch_cpu():
    from aonerf import _lib as L
    g = torch.Generator().manual_seed(0)
    raw = torch.rand((N, 3), generator=g) * 48.0 - 24.0
    raw[:8] = torch.tensor([[0.0, -0.0, 1e-8], [88.0, -88.0, 103.0], [-104.5, 30.0, -30.0],
                            [1e-30, -1e-30, 17.0], [-17.0, 0.5, -0.5], [3.0, -3.0, 7.25],
                            [-7.25, 11.0, -11.0], [20.0, -20.0, 15.5]])
    want = torch.sigmoid(raw)
    sig = torch.ones((N, 1, 1))
    t = torch.zeros((N, 1))
    dirs = torch.tensor([[1.0, 0.0, 0.0]]).expand(N, 3).contiguous()
    comp, _ = _composite(raw.reshape(N, 1, 3).cuda(), sig.cuda(), t.cuda(), dirs.cuda(),
                         L.ACT_VANILLA)
    diff = (comp.view(torch.int32) != want.view(torch.int32)).sum().item()
    print(f"sigmoid: {diff} of {3 * N} values differ from torch.sigmoid (CPU)")
    assert diff == 0


def test_alpha_exp_correctly_rounded():
    from aonerf import _lib as L
    g = torch.Generator().manual_seed(1)
    sigma = torch.rand((N,), generator=g) * 40.0
    sigma[:6] = torch.tensor([0.0, 1e-7, 1e-3, 87.0, 103.0, 120.0])
    # t = [0, 1], dirs = (1, 0, 0): D = 1, weights[:, 0] = alpha_0 * 1 (helper.py:171-176)
    t = torch.tensor([[0.0, 1.0]]).expand(N, 2).contiguous()
    dirs = torch.tensor([[1.0, 0.0, 0.0]]).expand(N, 3).contiguous()
    sig = torch.stack([sigma, torch.ones(N)], -1).reshape(N, 2, 1)
    rgb = torch.zeros((N, 2, 3))
    _, w = _composite(rgb.cuda(), sig.cuda(), t.cuda(), dirs.cuda(), L.ACT_VANILLA)
    got = w[:, 0].numpy()
    x = (-sigma).numpy()
    cr = (np.float32(1.0) - np.exp(x.astype(np.float64)).astype(np.float32)).astype(np.float32)
    ref = (1.0 - torch.exp(-sigma)).numpy()
    n_cr = int((got.view(np.int32) != cr.view(np.int32)).sum())
    n_ref = int((got.view(np.int32) != ref.view(np.int32)).sum())
    # one ulp of exp in [0.5, 1) is 2^-24; 1 - e adds at most one more rounding of that size
    dmax = float(np.abs(got.astype(np.float64) - ref).max())
    print(f"alpha: {n_cr} differ from the correctly rounded exp, {n_ref} of {N} from torch.exp "
          f"(CPU), max |diff| {dmax:.3e}")
    assert n_cr == 0
    assert n_ref <= 0.02 * N and dmax <= 2.0 ** -23


def test_pos_enc_sin_correctly_rounded():
    """aon_pos_enc (the in-register encoders share pos_enc_feature): every sin feature equals
    fp32(sin(fp64(argument))) with the argument formed as the reference forms it (helper.py:
    136-140: x * 2^d, then + fp32(pi/2) for the second half)."""
    from aonerf import helper as H
    g = torch.Generator().manual_seed(3)
    x = (torch.rand((1 << 18, 3), generator=g) * 12.0 - 6.0)
    # the last 4,096 points far out: arguments x 2^9 past kSinCrMax (2^20) take the fp64 OCML sine
    x[-4096:] *= 1000.0
    got = H.pos_enc(x.cuda(), 0, 10).cpu().numpy()
    xb = (x[:, None, :] * torch.tensor([2.0 ** i for i in range(10)])[:, None]).reshape(-1, 30)
    args = torch.cat([xb, xb + 0.5 * np.pi], -1).numpy()
    want = np.sin(args.astype(np.float64)).astype(np.float32)
    ne = int((got[:, 3:].view(np.int32) != want.view(np.int32)).sum())
    ref = torch.sin(torch.from_numpy(args)).numpy()
    n_ref = int((got[:, 3:].view(np.int32) != ref.view(np.int32)).sum())
    print(f"pos_enc: {ne} features off the correctly rounded sin, {n_ref} of {want.size} differ "
          f"from torch.sin (CPU)")
    assert ne == 0
    assert np.array_equal(got[:, :3], x.numpy())
