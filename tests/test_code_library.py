"""CodeLibraryArticulated (reference models/code_library.py:12-71) on CPU: parameter names and
shapes (so the reference's checkpoints load), the training lookup, and the test-time
interpolated articulation table against the reference's own output (art_train_step.npz)."""
import types

import numpy as np
import torch

from oracle import weights as W


def _lib():
    from aonerf.code_library import CodeLibraryArticulated

    lib = CodeLibraryArticulated(types.SimpleNamespace(N_max_objs=151, N_obj_code_length=128))
    lib.load_state_dict({k: torch.from_numpy(v) for k, v in W.code_library_state_dict(0).items()})
    return lib


def test_state_dict_layout():
    lib = _lib()
    shapes = {k: tuple(v.shape) for k, v in lib.state_dict().items()}
    assert shapes == {"embedding_instance_shape.weight": (151, 128),
                      "embedding_instance_appearance.weight": (151, 128),
                      "embedding_instance_articulation.weight": (10, 32)}


def test_lookup_and_interpolation(golden):
    g = golden("art_train_step.npz")
    lib = _lib()
    batch = {"instance_id": torch.tensor([7]), "articulation_id": torch.tensor([3])}
    lat = lib(batch)
    tables = W.code_library_state_dict(0)
    np.testing.assert_array_equal(lat["density"].detach().numpy(),
                                  tables["embedding_instance_shape.weight"][[7]])
    np.testing.assert_array_equal(lat["articulation"].detach().numpy(),
                                  tables["embedding_instance_articulation.weight"][[3]])
    interp = lib.get_interpolated_articulations(2, "cpu").detach().numpy()
    np.testing.assert_array_equal(interp, g["art_interp"])
    test = lib(batch, is_test=True)
    np.testing.assert_array_equal(test["articulation"].detach().numpy(), g["art_interp"][[3]])
