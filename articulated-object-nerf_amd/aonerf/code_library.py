"""Drop-in for ``CodeLibraryArticulated`` (reference models/code_library.py:12-71): the per-instance
shape / appearance codes and per-articulation codes of the auto-decoder, as nn.Embedding tables
with the reference's parameter names, init and forward.

The lookup is one row per table (batch["instance_id"] / batch["articulation_id"] hold a single
id in the reference's batch-size-1 loader, model_autodecoder.py:706-713); its autograd is torch's
embedding backward, which scatters the (1, C) latent gradients computed by the HIP training
kernels (train_art.py) into the tables.
"""
import torch
import torch.nn as nn
import torch.nn.init as init

N_MAX_ARTICULATIONS = 10
N_ART_CODE_LENGTH = 32


class CodeLibraryArticulated(nn.Module):
    """reference models/code_library.py:12-34 (hparams: N_max_objs, N_obj_code_length)."""

    def __init__(self, hparams):
        super().__init__()
        self.embedding_instance_shape = nn.Embedding(hparams.N_max_objs, hparams.N_obj_code_length)
        self.embedding_instance_appearance = nn.Embedding(hparams.N_max_objs,
                                                          hparams.N_obj_code_length)
        self.embedding_instance_articulation = nn.Embedding(N_MAX_ARTICULATIONS, N_ART_CODE_LENGTH)
        init.xavier_uniform_(self.embedding_instance_shape.weight)
        init.xavier_uniform_(self.embedding_instance_appearance.weight)
        init.xavier_uniform_(self.embedding_instance_articulation.weight)

    def forward(self, batch, is_test=False):
        """code_library.py:36-53 -> {density, color: (..., 128), articulation: (..., 32)}."""
        ret = {"density": self.embedding_instance_shape(batch["instance_id"]),
               "color": self.embedding_instance_appearance(batch["instance_id"])}
        if is_test:
            table = self.get_interpolated_articulations(2, batch["articulation_id"].device)
            ret["articulation"] = table[batch["articulation_id"]]
        else:
            ret["articulation"] = self.embedding_instance_articulation(batch["articulation_id"])
        return ret

    def get_interpolated_articulations(self, max_interpolations=2, device="cuda"):
        """code_library.py:55-71: the 10 articulation codes at even rows, midpoints between
        neighbours at odd rows ((prev + next) / 2) -> (2 * 10 - 1, 32)."""
        if max_interpolations != 2:
            raise ValueError("the reference interleaves exactly one midpoint (max_interpolations=2)")
        w = self.embedding_instance_articulation.weight.to(device)
        n = N_MAX_ARTICULATIONS
        out = torch.zeros((n * max_interpolations - 1, w.shape[1]), device=device)
        out[0::2] = w[:n]
        out[1::2] = (out[0:-1:2] + out[2::2]) / 2
        return out
