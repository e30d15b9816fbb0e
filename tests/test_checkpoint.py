"""Checkpoint loading (aonerf.checkpoint: reference utils/__init__.py:117-147, run.py:156-163).

tests/golden/checkpoint_manifest.json was written by make_golden.py case_checkpoint from the
REFERENCE's own extract_model_state_dict / load_ckpt applied to Lightning checkpoints of LitNeRF
and LitNeRF_AutoDecoder (PCG64 weights, the reference modules' state_dict keys).  Here the same
checkpoints are rebuilt from OUR modules' state_dicts (so the key layout must equal the
reference's), saved, and read back with our weights-only loader: every case's keys, order,
shapes and tensor bytes (sha256) must equal the reference's.
"""
import hashlib
import json
import os
import pickle
import types

import numpy as np
import pytest
import torch

from oracle import weights as W

HERE = os.path.dirname(os.path.abspath(__file__))
MANIFEST = json.load(open(os.path.join(HERE, "golden", "checkpoint_manifest.json")))


def sha(t):
    return hashlib.sha256(t.detach().contiguous().cpu().numpy().tobytes()).hexdigest()


def our_checkpoints():
    from aonerf.code_library import CodeLibraryArticulated
    from aonerf.model import NeRF
    from aonerf.model_autodecoder import NeRF_AE_Art

    net = NeRF()
    net.load_state_dict({k: torch.from_numpy(v) for k, v in W.nerf_state_dict(0).items()})
    art = NeRF_AE_Art()
    art.load_state_dict({k: torch.from_numpy(v) for k, v in W.art_state_dict(0).items()})
    lib = CodeLibraryArticulated(types.SimpleNamespace(N_max_objs=151, N_obj_code_length=128))
    lib.load_state_dict({k: torch.from_numpy(v) for k, v in W.code_library_state_dict(0).items()})
    van = {"model." + k: v for k, v in net.state_dict().items()}
    artsd = {"model." + k: v for k, v in art.state_dict().items()}
    artsd.update({"code_library." + k: v for k, v in lib.state_dict().items()})
    meta = MANIFEST["meta"]
    return {"vanilla": dict(meta, state_dict=van, optimizer_states=[], lr_schedulers=[]),
            "articulated": dict(meta, state_dict=artsd, optimizer_states=[], lr_schedulers=[])}


@pytest.fixture(scope="module")
def ckpt_dir(tmp_path_factory):
    d = tmp_path_factory.mktemp("ckpt")
    for name, ck in our_checkpoints().items():
        torch.save(ck, d / f"{name}.ckpt")
    return d


def test_layout_equals_reference(ckpt_dir):
    """Our modules' parameter names and shapes ARE the reference's (drop-in checkpoints)."""
    for name, ck in our_checkpoints().items():
        got = [[k, list(v.shape)] for k, v in ck["state_dict"].items()]
        assert got == MANIFEST["layouts"][name], name


def test_extract_model_state_dict_equals_reference(ckpt_dir):
    from aonerf.checkpoint import extract_model_state_dict

    for case in MANIFEST["cases"]:
        ext = extract_model_state_dict(str(ckpt_dir / f"{case['checkpoint']}.ckpt"),
                                       case["model_name"], case["prefixes_to_ignore"])
        assert list(ext) == case["keys"], case
        assert [list(v.shape) for v in ext.values()] == case["shapes"]
        assert [sha(v) for v in ext.values()] == case["sha256"]


def test_load_ckpt_equals_reference(ckpt_dir):
    from aonerf.checkpoint import load_ckpt
    from aonerf.model import NeRF

    net = NeRF()
    load_ckpt(net, str(ckpt_dir / "vanilla.ckpt"))
    assert {k: sha(v) for k, v in net.state_dict().items()} == MANIFEST["load_ckpt_vanilla_sha256"]
    load_ckpt(net, "")  # no path: a no-op (utils/__init__.py:135-136)
    with pytest.raises(RuntimeError):  # strict load: a model without these keys
        load_ckpt(torch.nn.Linear(2, 2), str(ckpt_dir / "vanilla.ckpt"))


class _Payload:
    def __reduce__(self):
        return (print, ("executed",))


def test_weights_only_refuses_code(tmp_path):
    """A checkpoint whose unpickling would run code is refused, not executed."""
    from aonerf.checkpoint import extract_model_state_dict

    p = tmp_path / "evil.ckpt"
    torch.save({"state_dict": {"model.x": torch.zeros(1)}, "hook": _Payload()}, p)
    with pytest.raises(pickle.UnpicklingError):
        extract_model_state_dict(str(p))


@pytest.mark.gpu
def test_render_from_checkpoint(ckpt_dir):
    """A NeRF restored through load_ckpt renders exactly what one given the weights directly
    renders (the packed MFMA streams are rebuilt from the loaded parameters)."""
    from aonerf.checkpoint import load_ckpt
    from aonerf.model import NeRF
    from aonerf.render import create_spheric_poses, render_frame, sapien_focal

    a = NeRF().cuda()
    a.load_state_dict({k: torch.from_numpy(v) for k, v in W.nerf_state_dict(0).items()})
    b = NeRF()
    load_ckpt(b, str(ckpt_dir / "vanilla.ckpt"))
    b = b.cuda()
    c2w = create_spheric_poses(4.0)[3]
    with torch.no_grad():
        fa = render_frame(a, c2w, 24, 32, sapien_focal(24))
        fb = render_frame(b, c2w, 24, 32, sapien_focal(24))
    assert torch.equal(fa, fb)
    assert np.isfinite(fa.cpu().numpy()).all()
