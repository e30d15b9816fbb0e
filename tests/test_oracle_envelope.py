"""The reference's own sensitivity envelope (CPU only).

The fine level re-samples along the coarse CDF, so a change of one fp32 ulp in the coarse MLP
outputs moves fine samples by delta-cdf / pdf.  These tests run the oracle with equally valid
re-associations of the reference's fp32 GEMMs (and with an fp64 GEMM, i.e. a MORE accurate
reference) and record how far the reference itself moves -- the envelope that the GPU
end-to-end gate in test_gpu_parity.py is set against.
"""
import numpy as np
import pytest
import torch

from oracle import nerf_oracle as O
from oracle import weights as W


def mlp_with(linear):
    def mlp(p, x, cond, **_):
        S, C = x.shape[1:]
        x = x.reshape(-1, C)
        inp = x
        for i in range(8):
            x = torch.relu(linear(x, p[f"pts_linears.{i}.weight"], p[f"pts_linears.{i}.bias"]))
            if i == 4:
                x = torch.cat([x, inp], -1)
        dens = linear(x, p["density_layer.weight"], p["density_layer.bias"]).reshape(-1, S, 1)
        bott = linear(x, p["bottleneck_layer.weight"], p["bottleneck_layer.bias"])
        c = torch.tile(cond[:, None, :], (1, S, 1)).reshape(-1, cond.shape[-1])
        x = torch.relu(linear(torch.cat([bott, c], -1), p["views_linear.0.weight"], p["views_linear.0.bias"]))
        return linear(x, p["rgb_layer.weight"], p["rgb_layer.bias"]).reshape(-1, S, 3), dens
    return mlp


VARIANTS = {
    "fp64_gemm": lambda x, w, b: (x.double() @ w.double().T + b.double()).float(),
    "k_split": lambda x, w, b: (x[:, : w.shape[1] // 2] @ w[:, : w.shape[1] // 2].T
                                + x[:, w.shape[1] // 2:] @ w[:, w.shape[1] // 2:].T) + b,
}


@pytest.mark.parametrize("variant", sorted(VARIANTS))
def test_reference_reassociation_envelope(golden, monkeypatch, variant):
    g = golden("forward_eval.npz")
    params = O.split_state_dict(W.nerf_state_dict(0))
    monkeypatch.setattr(O, "mlp_forward", mlp_with(VARIANTS[variant]))
    rays = {k: torch.from_numpy(g[k]) for k in ("rays_o", "rays_d", "viewdirs")}
    ret = O.nerf_forward(params, rays, False, True, 2.0, 6.0)
    coarse = np.abs(ret[0][2].numpy() - g["coarse_depth"]).max()
    fine = np.abs(ret[1][2].numpy() - g["fine_depth"]).max()
    print(f"{variant}: coarse depth {coarse:.2e}, fine depth {fine:.2e}")
    assert coarse < 1e-5          # the coarse level is insensitive
    assert 1e-5 < fine < 1e-3     # the fine level moves by ~1e-4 under a pure re-association
