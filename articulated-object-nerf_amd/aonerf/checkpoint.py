"""Drop-in for the reference's checkpoint helpers (utils/__init__.py:117-147): the model weights
of a pytorch-lightning checkpoint (``./results/{exp}/last.ckpt``, run.py:156-163) as a plain
state_dict whose keys lose the LightningModule attribute prefix (``model.`` for LitNeRF's
``self.model = NeRF()``, model.py:218, and LitNeRF_AutoDecoder's ``self.model = NeRF_AE_Art()``;
``code_library.`` for its CodeLibraryArticulated, model_autodecoder.py:356-357).

Loading is weights-only (``torch.load(..., weights_only=True)``): tensors, containers and
numbers deserialise, nothing in the file executes.  A checkpoint that needs arbitrary unpickling
is refused (pickle.UnpicklingError from torch) rather than run.
"""
import torch


def _load(ckpt_path):
    return torch.load(ckpt_path, map_location=torch.device("cpu"), weights_only=True)


def extract_model_state_dict(ckpt_path, model_name="model", prefixes_to_ignore=()):
    """utils/__init__.py:117-132: entries of the (Lightning) state_dict whose key starts with
    ``model_name``, with ``model_name + '.'`` stripped; keys starting with any of
    ``prefixes_to_ignore`` (after stripping) are dropped, as the reference prints them."""
    checkpoint = _load(ckpt_path)
    if "state_dict" in checkpoint:  # a pytorch-lightning checkpoint
        checkpoint = checkpoint["state_dict"]
    out = {}
    for k, v in checkpoint.items():
        if not k.startswith(model_name):
            continue
        k = k[len(model_name) + 1:]
        if any(k.startswith(p) for p in prefixes_to_ignore):
            print("ignore", k)
            continue
        out[k] = v
    return out


def load_ckpt(model, ckpt_path, model_name="model", prefixes_to_ignore=(), load_latent=True):
    """utils/__init__.py:134-140: update the model's state_dict with the checkpoint's entries
    and load it (strict, so a key the model does not have is an error, as in the reference).
    ``load_latent`` is accepted for signature parity (unused there too)."""
    if not ckpt_path:
        return
    model_dict = model.state_dict()
    model_dict.update(extract_model_state_dict(ckpt_path, model_name, prefixes_to_ignore))
    model.load_state_dict(model_dict)


def load_latent_codes(ckpt_path):
    """utils/__init__.py:142-147: the ``shape_codes`` / ``texture_codes`` embedding tables of a
    checkpoint's state_dict.  (No model in the reference registers those names: a checkpoint of
    LitNeRF_AutoDecoder holds ``code_library.embedding_instance_*`` instead, and this raises
    KeyError on it exactly as the reference does.)"""
    sd = _load(ckpt_path)["state_dict"]
    return sd["shape_codes.weight"], sd["texture_codes.weight"]
