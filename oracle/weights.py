"""Deterministic NeRF weights for parity tests and benches (test infrastructure only).

The reference initialises with the unseeded torch RNG (reference models/vanilla_nerf/model.py:
65-93; only numpy/random are seeded, model.py:35-36), so parity is checked on weights that
both sides regenerate from numpy PCG64.  Bounds follow the reference's init:
  * xavier_uniform on every weight except ``views_linear.0`` (model.py:66,74,91-93),
  * torch's default nn.Linear init elsewhere: weight bound 1/sqrt(fan_in) for
    ``views_linear.0`` (model.py:79) and bias bound 1/sqrt(fan_in) for all layers.
Shapes follow NeRFMLP.__init__ (model.py:62-85).
"""
import hashlib

import numpy as np


def mlp_shapes(min_deg_point=0, max_deg_point=10, deg_view=4, netdepth=8, netwidth=256,
               netdepth_condition=1, netwidth_condition=128, skip_layer=4, input_ch=3,
               input_ch_view=3, num_rgb_channels=3, num_density_channels=1):
    """Ordered [(name, (out, in), xavier)] exactly as NeRFMLP registers its Linear layers."""
    pos_size = ((max_deg_point - min_deg_point) * 2 + 1) * input_ch
    view_pos_size = (deg_view * 2 + 1) * input_ch_view
    out = [("pts_linears.0", (netwidth, pos_size), True)]
    for idx in range(netdepth - 1):
        k = netwidth + pos_size if (idx % skip_layer == 0 and idx > 0) else netwidth
        out.append((f"pts_linears.{idx + 1}", (netwidth, k), True))
    out.append(("views_linear.0", (netwidth_condition, netwidth + view_pos_size), False))
    for idx in range(netdepth_condition - 1):
        out.append((f"views_linear.{idx + 1}", (netwidth_condition, netwidth_condition), True))
    out.append(("bottleneck_layer", (netwidth, netwidth), True))
    out.append(("density_layer", (num_density_channels, netwidth), True))
    out.append(("rgb_layer", (num_rgb_channels, netwidth_condition), True))
    return out


def mlp_weights(rng, **kw):
    """One NeRFMLP's parameters as {name.weight/name.bias: float32 ndarray}."""
    params = {}
    for name, (fo, fi), xavier in mlp_shapes(**kw):
        wb = np.sqrt(6.0 / (fi + fo)) if xavier else 1.0 / np.sqrt(fi)
        params[f"{name}.weight"] = rng.uniform(-wb, wb, size=(fo, fi)).astype(np.float32)
        bb = 1.0 / np.sqrt(fi)
        params[f"{name}.bias"] = rng.uniform(-bb, bb, size=(fo,)).astype(np.float32)
    return params


def nerf_state_dict(seed=0, **kw):
    """A full ``NeRF`` state_dict ({coarse_mlp.*, fine_mlp.*}) from PCG64(seed)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    sd = {}
    for level in ("coarse_mlp", "fine_mlp"):
        for k, v in mlp_weights(rng, **kw).items():
            sd[f"{level}.{k}"] = v
    return sd


def digest(sd):
    """sha256 over the state dict in key order (pins the regenerated weights to the fixtures)."""
    h = hashlib.sha256()
    for k in sorted(sd):
        h.update(k.encode())
        h.update(np.ascontiguousarray(sd[k]).tobytes())
    return h.hexdigest()


# ---------------------------------------------------------------------------- articulated
def art_mlp_shapes(min_deg_point=0, max_deg_point=10, deg_view=4, netdepth=8, netwidth=256,
                   netdepth_deformation=4, netwidth_deformation=128, netdepth_condition=4,
                   netwidth_condition=128, shape_latent_dim=128, appearance_latent_dim=128,
                   articulation_latent_dim=32, skip_layer=4, input_ch=3, input_ch_view=3,
                   num_rgb_channels=3, num_density_channels=1):
    """Ordered [(name, (out, in), xavier)] of the articulated NeRFMLP
    (reference models/vanilla_nerf/model_autodecoder.py:60-166, deformation_mlp=True,
    enc_after=True): a deformation MLP on cat[xyz, shape, articulation] whose 3-vector output is
    added to xyz before pos_enc, a trunk on cat[pos_enc(xyz'), shape], a view branch on
    cat[bottleneck, enc_dir, appearance].  ``views_linear.0`` keeps torch's default init."""
    pos_size_def = input_ch + shape_latent_dim + articulation_latent_dim
    pos_size = ((max_deg_point - min_deg_point) * 2 + 1) * input_ch + shape_latent_dim
    view_pos_size = (deg_view * 2 + 1) * input_ch_view
    out = [("deformations_linear.0", (netwidth_deformation, pos_size_def), True)]
    for idx in range(netdepth_deformation - 1):
        out.append((f"deformations_linear.{idx + 1}", (netwidth_deformation, netwidth_deformation), True))
    out.append(("deformation_layer", (3, netwidth_deformation), True))
    out.append(("pts_linears.0", (netwidth, pos_size), True))
    for idx in range(netdepth - 1):
        k = netwidth + pos_size if (idx % skip_layer == 0 and idx > 0) else netwidth
        out.append((f"pts_linears.{idx + 1}", (netwidth, k), True))
    out.append(("views_linear.0", (netwidth_condition, netwidth + view_pos_size + appearance_latent_dim),
                False))
    for idx in range(netdepth_condition - 1):
        out.append((f"views_linear.{idx + 1}", (netwidth_condition, netwidth_condition), True))
    out.append(("bottleneck_layer", (netwidth, netwidth), True))
    out.append(("density_layer", (num_density_channels, netwidth), True))
    out.append(("rgb_layer", (num_rgb_channels, netwidth_condition), True))
    return out


def art_state_dict(seed=0):
    """A full ``NeRF_AE_Art`` state_dict ({coarse_mlp.*, fine_mlp.*}) from PCG64(seed)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    sd = {}
    for level in ("coarse_mlp", "fine_mlp"):
        for name, (fo, fi), xavier in art_mlp_shapes():
            wb = np.sqrt(6.0 / (fi + fo)) if xavier else 1.0 / np.sqrt(fi)
            sd[f"{level}.{name}.weight"] = rng.uniform(-wb, wb, size=(fo, fi)).astype(np.float32)
            bb = 1.0 / np.sqrt(fi)
            sd[f"{level}.{name}.bias"] = rng.uniform(-bb, bb, size=(fo,)).astype(np.float32)
    return sd


def art_latents(seed=0, n_obj_code=128, n_art_code=32):
    """Latent codes as CodeLibraryArticulated.forward returns them (reference
    models/code_library.py:36-53): density / color (1, 128), articulation (1, 32); xavier
    bounds of Embedding(N_max_objs=8 / N_max_articulations=10, dim) rows."""
    rng = np.random.Generator(np.random.PCG64(seed))
    b_obj = np.sqrt(6.0 / (8 + n_obj_code))
    b_art = np.sqrt(6.0 / (10 + n_art_code))
    return {"density": rng.uniform(-b_obj, b_obj, size=(1, n_obj_code)).astype(np.float32),
            "color": rng.uniform(-b_obj, b_obj, size=(1, n_obj_code)).astype(np.float32),
            "articulation": rng.uniform(-b_art, b_art, size=(1, n_art_code)).astype(np.float32)}


def code_library_state_dict(seed=0, n_max_objs=151, n_obj_code=128, n_max_articulations=10,
                            n_art_code=32):
    """A ``CodeLibraryArticulated`` state_dict (reference models/code_library.py:12-34): three
    nn.Embedding tables with xavier_uniform bounds sqrt(6 / (rows + dim)); N_max_objs = 151 and
    N_obj_code_length = 128 are the reference's opt.py:75,84 defaults."""
    rng = np.random.Generator(np.random.PCG64(seed))
    out = {}
    for name, (n, c) in (("embedding_instance_shape", (n_max_objs, n_obj_code)),
                         ("embedding_instance_appearance", (n_max_objs, n_obj_code)),
                         ("embedding_instance_articulation", (n_max_articulations, n_art_code))):
        b = np.sqrt(6.0 / (n + c))
        out[f"{name}.weight"] = rng.uniform(-b, b, size=(n, c)).astype(np.float32)
    return out
