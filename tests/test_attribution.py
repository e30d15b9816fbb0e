"""CPU checks of the end-to-end attribution machinery (oracle/attribution.py) that the GPU parity
gates and bench.py's cpu_baseline use: the implementation-envelope variants are what they claim
(+-1 ulp, exact cases kept, deterministic; correctly rounded), and an equally valid fp32
implementation of the reference -- the oracle with re-associated GEMMs, standing in for "ours" --
has every end-to-end outlier explained."""
import math

import numpy as np
import torch

from oracle import attribution as A
from oracle import nerf_oracle as O
from oracle import weights as W


def test_ulp_jitter_is_one_ulp_deterministic_and_keeps_exact_cases():
    x = torch.linspace(-40.0, 40.0, 10001)
    x[::97] = 0.0
    f = A.ulp_jitter(torch.exp, 2)
    a, b = f(x), f(x)
    assert torch.equal(a, b)  # seeded: a re-run draws the same pattern
    r = torch.exp(x)
    up, dn = torch.nextafter(r, torch.full_like(r, math.inf)), torch.nextafter(r, torch.full_like(r, -math.inf))
    assert bool(((a == r) | (a == up) | (a == dn)).all())
    assert bool((a[::97] == 1.0).all())  # exp(0) stays exactly 1
    moved = (a != r).float().mean().item()
    assert 0.55 < moved < 0.78  # about two thirds of the elements move
    s = A.ulp_jitter(torch.sin, 1)(x)
    assert bool((s[::97] == 0.0).all())


def test_correctly_rounded_variant():
    x = torch.from_numpy(np.random.default_rng(0).uniform(-5120, 5120, 4096).astype(np.float32))
    cr = A.correctly_rounded(torch.sin)(x)
    want = np.sin(x.numpy().astype(np.float64)).astype(np.float32)
    assert np.array_equal(cr.numpy(), want)


def test_variants_restore_torch():
    sin, exp = torch.sin, torch.exp
    for ctx in A.TRANSCENDENTAL_VARIANTS.values():
        with ctx():
            pass
    assert torch.sin is sin and torch.exp is exp
    before = O.mlp_forward
    for ctx in A.oracle_variants().values():
        with ctx():
            pass
    assert O.mlp_forward is before


def test_every_outlier_of_a_valid_implementation_is_attributed(golden):
    """'Ours' = the oracle with k-split GEMMs (a pure re-association); against the reference's
    golden end-to-end output every ray beyond 1e-4 must be explained by (a)-(c)."""
    g = golden("forward_eval.npz")
    params = O.split_state_dict(W.nerf_state_dict(0))
    rays = {k: torch.from_numpy(g[k]) for k in ("rays_o", "rays_d", "viewdirs")}
    with A.oracle_variants()["k_split"]():
        ours, inter = O.nerf_forward(params, rays, False, True, 2.0, 6.0, return_intermediates=True)
    t_f = inter[1]["t_vals"]
    rgb_o, acc_o, _, depth_o = O.render_level(params, rays, t_f, 1, True)
    on_ours = {"rgb": rgb_o.numpy(), "acc": acc_o.numpy(), "depth": depth_o.numpy()}
    att = A.Attribution(inter[0]["weights"].numpy(), g["coarse_weights"], 128)
    for j, k in enumerate(("rgb", "acc", "depth")):
        err = np.abs(ours[1][j].numpy().astype(np.float64) - g[f"fine_{k}"])
        ok = att.rays(on_ours[k], g[f"fine_{k}"], err, g[f"env_fine_{k}"])
        bad = (err > A.E2E_ATOL).reshape(len(err), -1).any(-1)
        assert not (bad & ~ok).any(), (k, np.nonzero(bad & ~ok)[0])
        assert set(att.why[bad]) <= {"plateau flip", "amplification", "implementation envelope"}


def test_fine_envelope_shapes_and_worst(golden):
    g = golden("forward_eval.npz")
    params = O.split_state_dict(W.nerf_state_dict(0))
    rays = {k: torch.from_numpy(g[k][:16]) for k in ("rays_o", "rays_d", "viewdirs")}
    env, worst = A.fine_envelope(params, rays)
    assert env[0].shape == (16, 3) and env[1].shape == (16,) and env[2].shape == (16,)
    assert {v for v, _ in worst} == set(A.oracle_variants())
    assert all(np.isfinite(e).all() for e in env)
