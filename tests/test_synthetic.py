"""The product-side synthetic weights (aonerf.synthetic, used by bench.py and tools/) equal the
oracle's test weights bit for bit, so the GPU legs and the CPU baselines see the same model."""
import numpy as np
import torch

from oracle import weights as W


def test_vanilla_weights_match_oracle():
    from aonerf.model import NeRF
    from aonerf.synthetic import init_like_reference

    sd = init_like_reference(NeRF()).state_dict()
    want = W.nerf_state_dict(0)
    assert set(sd) == set(want)
    assert W.digest({k: v.numpy() for k, v in sd.items()}) == W.digest(want)


def test_articulated_weights_and_latents_match_oracle():
    from aonerf.model_autodecoder import NeRF_AE_Art
    from aonerf.synthetic import art_latents, init_like_reference

    sd = init_like_reference(NeRF_AE_Art()).state_dict()
    want = W.art_state_dict(0)
    assert set(sd) == set(want)
    assert W.digest({k: v.numpy() for k, v in sd.items()}) == W.digest(want)
    lat, lat_o = art_latents(0), W.art_latents(0)
    for k in lat_o:
        np.testing.assert_array_equal(lat[k].numpy(), lat_o[k])
        assert lat[k].dtype == torch.float32


def test_code_library_matches_oracle():
    import types

    from aonerf.code_library import CodeLibraryArticulated
    from aonerf.synthetic import init_code_library

    lib = CodeLibraryArticulated(types.SimpleNamespace(N_max_objs=151, N_obj_code_length=128))
    sd = init_code_library(lib).state_dict()
    want = W.code_library_state_dict(0)
    assert set(sd) == set(want)
    for k in want:
        np.testing.assert_array_equal(sd[k].numpy(), want[k])
