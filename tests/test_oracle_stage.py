"""The oracle's teacher-forcing hooks used by the articulated gradient gates (CPU):

* ``pos_enc_at`` evaluated at a tensor's own fp32 points equals ``pos_enc`` (value and
  gradient), so forcing x' to a GPU's fp32 x' changes nothing but the point;
* ``art_mlp_forward(xp_fixed=own x')`` equals the plain forward and its gradients;
* ``art_mlp_forward_kept`` fed a forward's OWN intermediates reproduces that forward's raw
  outputs and every parameter / latent gradient (fp64): its backward is the reference
  model_autodecoder.py:168-239's backward, only evaluated at given forward values.
"""
import numpy as np
import torch

from oracle import nerf_oracle as O
from oracle import weights as W


def _setup(dtype, B=5, S=7, seed=3):
    params = [{k: v.to(dtype).requires_grad_(True) for k, v in p.items()}
              for p in O.split_state_dict(W.art_state_dict(0))]
    lat = {k: torch.from_numpy(v).to(dtype).requires_grad_(True) for k, v in W.art_latents(1).items()}
    g = torch.Generator().manual_seed(seed)
    pos = ((torch.rand(B, S, 3, generator=g) - 0.5) * 2).to(dtype)
    cond = O.pos_enc(torch.nn.functional.normalize(torch.randn(B, 3, generator=g), dim=-1), 0, 4).to(dtype)
    draw = torch.randn(B * S, 4, generator=g).to(dtype)
    return params[1], lat, pos, cond, draw


def _grads(p, lat):
    out = {k: v.grad.clone() for k, v in p.items()}
    out.update({f"latent {k}": v.grad.clone() for k, v in lat.items()})
    for v in list(p.values()) + list(lat.values()):
        v.grad = None
    return out


def test_pos_enc_at_own_points_equals_pos_enc():
    g = torch.Generator().manual_seed(0)
    x = ((torch.rand(50, 3, generator=g) - 0.5) * 8).requires_grad_(True)
    gy = torch.randn(50, 63, generator=g)
    y = O.pos_enc(x, 0, 10)
    y.backward(gy)
    gx = x.grad.clone()
    x.grad = None
    y2 = O.pos_enc_at(x.detach(), x, 0, 10)
    y2.backward(gy)
    np.testing.assert_array_equal(y2.detach().numpy(), y.detach().numpy())
    np.testing.assert_allclose(x.grad.numpy(), gx.numpy(), rtol=1e-6, atol=1e-6 * gx.abs().max().item())


def test_xp_forced_at_own_points_is_the_plain_forward():
    p, lat, pos, cond, draw = _setup(torch.float32)
    rgb, sig, xp = O.art_mlp_forward(p, pos, cond, lat, return_xp=True)
    torch.autograd.backward([rgb.reshape(-1, 3), sig.reshape(-1, 1)], [draw[:, :3], draw[:, 3:]])
    ref = _grads(p, lat)
    rgb2, sig2 = O.art_mlp_forward(p, pos, cond, lat, xp_fixed=xp.detach())
    np.testing.assert_array_equal(rgb2.detach().numpy(), rgb.detach().numpy())
    np.testing.assert_array_equal(sig2.detach().numpy(), sig.detach().numpy())
    torch.autograd.backward([rgb2.reshape(-1, 3), sig2.reshape(-1, 1)], [draw[:, :3], draw[:, 3:]])
    got = _grads(p, lat)
    for k, v in ref.items():
        s = v.abs().max().item()
        assert (got[k] - v).abs().max().item() <= 1e-5 * max(s, 1e-30), k


def test_kept_forward_reproduces_backward_fp64():
    p, lat, pos, cond, draw = _setup(torch.float64)
    S = pos.shape[1]
    with torch.no_grad():  # the fp32 points the GPU would hand over
        xp32 = O.art_mlp_forward(p, pos, cond, lat, return_xp=True)[2].float()
    rec = {}
    rgb, sig = O.art_mlp_forward(p, pos, cond, lat, xp_fixed=xp32, record=rec)
    torch.autograd.backward([rgb.reshape(-1, 3), sig.reshape(-1, 1)], [draw[:, :3], draw[:, 3:]])
    ref = _grads(p, lat)
    kept = {k: ([x.detach() for x in v] if isinstance(v, list) else v.detach()) for k, v in rec.items()}
    kept["xp"] = kept["xp"].float()
    r2, s2 = O.art_mlp_forward_kept(p, kept, cond, lat, S)
    np.testing.assert_allclose(r2.detach().numpy(), rgb.reshape(-1, 3).detach().numpy(), rtol=0, atol=1e-12)
    np.testing.assert_allclose(s2.detach().numpy(), sig.reshape(-1, 1).detach().numpy(), rtol=0, atol=1e-12)
    torch.autograd.backward([r2, s2], [draw[:, :3], draw[:, 3:]])
    got = _grads(p, lat)
    for k, v in ref.items():
        s = v.abs().max().item()
        assert (got[k] - v).abs().max().item() <= 1e-12 * max(s, 1e-30), k
