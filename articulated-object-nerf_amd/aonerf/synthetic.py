"""Seeded synthetic parameters for benches and tools (no checkpoints are available offline).

The reference initialises with the unseeded torch RNG (models/vanilla_nerf/model.py:65-93,
model_autodecoder.py:82-166), so benches need a reproducible stand-in: every nn.Linear of each
level's MLP, in registration order, draws weight then bias from numpy PCG64(seed) with the
reference's bounds -- xavier_uniform (sqrt(6 / (fan_in + fan_out))) except ``views_linear.0``
(torch's default, 1 / sqrt(fan_in)), biases 1 / sqrt(fan_in).  The test-side generator in
oracle/weights.py draws the same stream; tests/test_synthetic.py checks the two agree bit for
bit, so a bench's GPU leg and its CPU baseline run on identical weights.
"""
import numpy as np
import torch
import torch.nn as nn


@torch.no_grad()
def init_like_reference(model, seed=0):
    """Fill ``model`` (NeRF or NeRF_AE_Art: coarse_mlp then fine_mlp) in place; returns it."""
    rng = np.random.Generator(np.random.PCG64(seed))
    for mlp in (model.coarse_mlp, model.fine_mlp):
        for name, m in mlp.named_modules():
            if not isinstance(m, nn.Linear):
                continue
            fo, fi = m.weight.shape
            wb = np.sqrt(6.0 / (fi + fo)) if name != "views_linear.0" else 1.0 / np.sqrt(fi)
            w = rng.uniform(-wb, wb, size=(fo, fi)).astype(np.float32)
            bb = 1.0 / np.sqrt(fi)
            b = rng.uniform(-bb, bb, size=(fo,)).astype(np.float32)
            m.weight.copy_(torch.from_numpy(w))
            m.bias.copy_(torch.from_numpy(b))
    return model


def art_latents(seed=0, n_obj_code=128, n_art_code=32, device=None):
    """Latent codes shaped as CodeLibraryArticulated.forward returns them (reference
    models/code_library.py:36-53): density / color (1, 128), articulation (1, 32), drawn with
    the xavier bounds of its Embedding rows (8 objects, 10 articulations)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    b_obj = np.sqrt(6.0 / (8 + n_obj_code))
    b_art = np.sqrt(6.0 / (10 + n_art_code))
    out = {"density": rng.uniform(-b_obj, b_obj, size=(1, n_obj_code)),
           "color": rng.uniform(-b_obj, b_obj, size=(1, n_obj_code)),
           "articulation": rng.uniform(-b_art, b_art, size=(1, n_art_code))}
    return {k: torch.from_numpy(v.astype(np.float32)).to(device) for k, v in out.items()}


@torch.no_grad()
def init_code_library(lib, seed=0):
    """Fill a CodeLibraryArticulated's three tables in place from PCG64(seed) with their
    xavier_uniform bounds (reference models/code_library.py:31-33); the same stream as the
    test-side oracle/weights.py code_library_state_dict."""
    rng = np.random.Generator(np.random.PCG64(seed))
    for emb in (lib.embedding_instance_shape, lib.embedding_instance_appearance,
                lib.embedding_instance_articulation):
        n, c = emb.weight.shape
        b = np.sqrt(6.0 / (n + c))
        emb.weight.copy_(torch.from_numpy(rng.uniform(-b, b, size=(n, c)).astype(np.float32)))
    return lib
