"""Per-model training numerics (verdict r05 #5; SURVEY 8(b): no mutable globals).  CPU only:
the models are built on the host, no kernel runs."""
import pytest

from aonerf import linalg, model, model_autodecoder, train, train_art
from aonerf.numerics import ART_FORWARD, TrainNumerics


def test_no_module_level_switches():
    """The round-5 module switches are gone: the kernels and precisions a model trains with are
    its own TrainNumerics, the march fusion and range check its own attributes."""
    gone = {train: ("PRECISION", "FUSED_FORWARD", "FUSED_BACKWARD", "OVERLAP_DWEIGHT", "TIMERS",
                    "RANGE_CHECK"),
            train_art: ("PRECISION", "FUSED_FORWARD", "FUSED_BACKWARD", "BF16_TRUNK", "BF16_VIEW",
                        "F16_WEIGHTS", "F16_ACTS"),
            model: ("FUSED_MARCH", "RANGE_CHECK"), linalg: ("BATCH", "BATCH128")}
    for mod, names in gone.items():
        for n in names:
            assert not hasattr(mod, n), (mod.__name__, n)


def test_numerics_per_model():
    a = model.NeRF()
    b = model.NeRF(train_precision="bf16", fused_march=False)
    assert a.train_numerics == TrainNumerics() and a.fused_march and a.range_check
    assert b.train_numerics.precision == "bf16" and b.train_numerics.bf16 and not b.fused_march
    assert a.train_numerics.precision == "f16x3"  # b's setting did not leak
    c = model_autodecoder.NeRF_AE_Art(train_numerics=TrainNumerics(precision="bf16",
                                                                    art_forward="f16x3"))
    assert c.train_numerics.art_forward == "f16x3"
    assert model_autodecoder.NeRF_AE_Art().train_numerics.art_forward == "f16_acts"


def test_numerics_validation():
    with pytest.raises(ValueError):
        TrainNumerics(precision="fp16")
    with pytest.raises(ValueError):
        TrainNumerics(art_forward="bf16_everything")
    with pytest.raises(ValueError):
        model.NeRF(train_precision="bf16", train_numerics=TrainNumerics(precision="f16x3"))
    with pytest.raises(TypeError):
        model.NeRF(train_numerics={"precision": "bf16"})
    t = TrainNumerics()
    with pytest.raises(Exception):
        t.precision = "bf16"  # frozen: a model's numerics are replaced, never mutated
    assert t.replace(precision="bf16").bf16 and not t.bf16
    # the kernel's mixed codes (include/aonerf.h aon_mlp_art_fwd_train_bf16)
    assert {k: v[0] for k, v in ART_FORWARD.items()} == {
        "f16x3": 0, "bf16_trunk": 1, "bf16_view": 2, "f16_weights": 3, "f16_acts": 4}
