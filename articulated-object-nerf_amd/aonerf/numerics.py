"""Per-model training numerics (reentrant, no mutable globals).

A model carries its own ``TrainNumerics`` (``NeRF(train_precision=...)``,
``NeRF_AE_Art(train_precision=...)``, or a whole ``train_numerics=TrainNumerics(...)``): two
models in one process train at different precisions, each exactly as it would alone.  Nothing in
aonerf reads a module-level switch to pick kernels or precisions; the render precision is the
ctor's ``precision`` as before.

Fields:
  precision       "f16x3" -- the parity mode: three fp16 MFMA products per MAC on hi/lo operands,
                  fp32 activations (LitNeRF.training_step, model.py:256-282, at fp32-class
                  accuracy); "bf16" -- BASELINE config C5's bf16 step: one bf16 MFMA per product
                  in the forward (vanilla), the backward chain and the weight-gradient GEMMs,
                  activations and gradients kept as bf16; compositing, loss, their backward and
                  Adam fp32 on fp32 master weights.
  fused_forward   the level's forward as ONE fused kernel that also stores the activations
                  (aon_mlp_fwd_train / aon_mlp_art_fwd_train); False: layer by layer on aon_gemm.
  fused_backward  every input gradient in one fused kernel (aon_mlp_bwd / aon_mlp_art_bwd);
                  False: every product an aon_gemm (plus aon_pos_enc_bwd, articulated).
  overlap_dweight the fine level's weight-gradient GEMMs on a side stream, concurrent with the
                  coarse level's backward (measured slower on MI355X; off).
  art_forward     the articulated bf16 mode's forward past the deformation MLP (which is always
                  fp16x3: x' feeds pos_enc's sin(2^9 x')): "f16_acts" (default: two fp16 MFMAs
                  per product, activations rounded once to fp16), "f16x3" (fp16x3 throughout,
                  only the stores bf16), and three A/B modes held off by their measured gates --
                  "f16_weights" (weights rounded to fp16), "bf16_view" (view branch bf16),
                  "bf16_trunk" (trunk, heads and view branch bf16).  Ignored in f16x3 mode.
  batch_dweights  the level's whole-tile weight-gradient products as aon_gemm_batch launches
                  (False: one aon_gemm per product; same bits).
  batch_128       with batch_dweights, the 128-column-tile products batched too.
"""
import dataclasses

PRECISIONS = ("f16x3", "bf16")
# art_forward -> aon_mlp_art_fwd_train_bf16's `mixed` code (include/aonerf.h) and whether the
# pack is the mixed stream (aon_mlp_art_pack_mixed) or the plain fp16x3 one
ART_FORWARD = {"f16x3": (0, False), "bf16_trunk": (1, True), "bf16_view": (2, True),
               "f16_weights": (3, True), "f16_acts": (4, False)}


@dataclasses.dataclass(frozen=True)
class TrainNumerics:
    precision: str = "f16x3"
    fused_forward: bool = True
    fused_backward: bool = True
    overlap_dweight: bool = False
    art_forward: str = "f16_acts"
    batch_dweights: bool = True
    batch_128: bool = True

    def __post_init__(self):
        if self.precision not in PRECISIONS:
            raise ValueError(f"train precision must be one of {PRECISIONS}, got {self.precision!r}")
        if self.art_forward not in ART_FORWARD:
            raise ValueError(f"art_forward must be one of {sorted(ART_FORWARD)}, "
                             f"got {self.art_forward!r}")

    @property
    def bf16(self):
        return self.precision == "bf16"

    def replace(self, **kw):
        return dataclasses.replace(self, **kw)


DEFAULT = TrainNumerics()


def resolve(train_precision="f16x3", train_numerics=None):
    """The ctor kwargs -> one TrainNumerics (train_numerics wins; its precision must agree with
    an explicitly different train_precision)."""
    if train_numerics is None:
        return TrainNumerics(precision=train_precision)
    if not isinstance(train_numerics, TrainNumerics):
        raise TypeError("train_numerics must be an aonerf.numerics.TrainNumerics")
    if train_precision not in (train_numerics.precision, "f16x3"):
        raise ValueError("train_precision and train_numerics.precision disagree")
    return train_numerics
