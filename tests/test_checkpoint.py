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


def _pl152_checkpoint(state_dict):
    """A checkpoint with every top-level entry pytorch-lightning 1.5.2 (the reference's pin,
    requirements.txt) writes from run.py's Trainer: CheckpointConnector.dump_checkpoint adds
    epoch / global_step / version / state_dict / loops / callbacks (keyed by the callback's
    state_key string) / optimizer_states / lr_schedulers / hyper_parameters (dict(model.hparams):
    LitNeRF.__init__ updates it with vars(argparse hparams), model.py:216).  The structure is
    restated from PL 1.5.2's published format (the library is absent here): parity unpinned
    beyond the types it uses."""
    params = list(state_dict.values())
    adam = {"state": {i: {"step": 1200, "exp_avg": torch.zeros_like(p), "exp_avg_sq": torch.ones_like(p)}
                      for i, p in enumerate(params[:3])},
            "param_groups": [{"lr": 4.9e-4, "betas": (0.9, 0.999), "eps": 1e-8, "weight_decay": 0,
                              "amsgrad": False, "params": list(range(len(params)))}]}
    ckpt_key = ("ModelCheckpoint{'monitor': 'val/psnr', 'mode': 'max', 'every_n_train_steps': 0, "
                "'every_n_epochs': 10, 'train_time_interval': None, 'save_on_train_epoch_end': True}")
    return {
        "epoch": 9, "global_step": 1200, "pytorch-lightning_version": "1.5.2",
        "state_dict": state_dict,
        "loops": {"fit_loop": {"state_dict": {}, "epoch_loop.state_dict": {"_batches_that_stepped": 1200},
                               "epoch_progress": {"total": {"ready": 10, "started": 10,
                                                            "processed": 10, "completed": 9},
                                                  "current": {"ready": 10, "started": 10,
                                                              "processed": 10, "completed": 9}}},
                  "validate_loop": {"state_dict": {}}, "test_loop": {"state_dict": {}},
                  "predict_loop": {"state_dict": {}}},
        "callbacks": {ckpt_key: {"monitor": "val/psnr", "best_model_score": torch.tensor(27.5),
                                 "best_model_path": "/results/exp/epoch=9.ckpt",
                                 "current_score": torch.tensor(27.5), "dirpath": "/results/exp",
                                 "best_k_models": {"/results/exp/epoch=9.ckpt": torch.tensor(27.5)},
                                 "kth_best_model_path": "/results/exp/epoch=9.ckpt",
                                 "kth_value": torch.tensor(27.5),
                                 "last_model_path": "/results/exp/last.ckpt"}},
        "optimizer_states": [adam], "lr_schedulers": [],
        "hyper_parameters": {"root_dir": "data/laptop", "dataset_name": "sapien", "exp_name": "exp",
                             "img_wh": [640, 480], "white_back": True, "chunk": 3840,
                             "batch_size": 4096, "num_epochs": 100, "num_gpus": 8, "run_eval": True,
                             "render_name": None, "is_optimize": None, "finetune_lpips": False,
                             "lr_init": 5e-4, "lr_final": 5e-6, "lr_delay_steps": 2500,
                             "lr_delay_mult": 0.01, "randomized": True},
    }


def test_full_pl152_checkpoint_loads_weights_only(tmp_path):
    """a checkpoint with PL 1.5.2's whole key set (hyper_parameters, callbacks,
    loops, Adam optimizer_states) is accepted by the weights-only loader, and yields the same
    model weights as the minimal one."""
    from aonerf.checkpoint import extract_model_state_dict, load_ckpt
    from aonerf.model import NeRF

    ck = our_checkpoints()["vanilla"]
    p = tmp_path / "last.ckpt"
    torch.save(_pl152_checkpoint(ck["state_dict"]), p)
    full = torch.load(p, map_location="cpu", weights_only=True)  # nothing refused
    assert full["hyper_parameters"]["img_wh"] == [640, 480]
    ext = extract_model_state_dict(str(p))
    assert [sha(v) for v in ext.values()] == [sha(v) for v in ck["state_dict"].values()]
    net = NeRF()
    load_ckpt(net, str(p))
    assert {k: sha(v) for k, v in net.state_dict().items()} == MANIFEST["load_ckpt_vanilla_sha256"]
