"""CPU-side checks of the C ABI: the library loads, exports every symbol include/aonerf.h
declares, and rejects invalid arguments with the documented status/message -- all without
touching a GPU (argument validation happens before any HIP call)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "aonerf.h")


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(aon_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def L():
    from aonerf import _lib

    return _lib


def test_header_symbols_exported(L):
    lib = L.lib()
    syms = declared_symbols()
    assert len(syms) >= 12
    for s in syms:
        assert hasattr(lib, s), f"{s} declared in aonerf.h but not exported"
    assert set(syms) <= set(L._SIGNATURES), "ctypes binding misses a declared entry point"


def test_abi_version_and_sizes(L):
    lib = L.lib()
    assert lib.aon_abi_version() == L.ABI_VERSION == 13
    # precision 3 (ABI 12's 32x32x16 render stream) is withdrawn: no packed size
    assert lib.aon_mlp_packed_bytes(3) == 0
    assert lib.aon_mlp_packed_bytes(99) == 0


@pytest.mark.parametrize("name,args", [
    ("aon_composite_fwd", (None, 3, None, 1, None, None, 4, 8, 1, 1, None, None, None, None, None)),
    ("aon_sample_pdf", (None, 0, None, 0, 4, 1, 128, None, 0, None, 0, None, None, None, None, None)),
    ("aon_mlp_fwd", (None, 0, None, None, None, None, 4, 8, 0, None, None)),
    ("aon_pos_enc", (None, 4, 0, 10, None, None)),
    ("aon_frame_rays", (0, 4, 1.0, None, 0, 0, None, None, None, None)),
])
def test_invalid_arguments_raise(L, name, args):
    with pytest.raises(ValueError, match=name):
        L.call(name, *args)


def test_abi10_argument_checks(L):
    """ABI 10's new entry points refuse bad arguments before any launch (no GPU needed):
    aon_cast_rays_tiled's width (a multiple of 16 holding every encoding), the articulated bf16
    forward's `mixed` range and aon_gemm's n_store on an exact-fp32 tiny product."""
    p = ctypes.c_void_p(16)
    with pytest.raises(ValueError, match="width"):
        L.call("aon_cast_rays_tiled", p, p, p, 4, 8, 0, 10, 48, p, None)  # 63 encodings > 48
    with pytest.raises(ValueError, match="width"):
        L.call("aon_cast_rays_tiled", p, p, p, 4, 8, 0, 10, 72, p, None)  # not a multiple of 16
    with pytest.raises(ValueError, match="bad arguments"):
        L.call("aon_cast_rays_tiled", None, p, p, 4, 8, 0, 10, 64, p, None)
    with pytest.raises(ValueError, match="mixed"):
        L.call("aon_mlp_art_fwd_train_bf16", p, p, p, p, p, 1, 1, None, p, p, p, p, p, p, p, p, p,
               5, None)
    with pytest.raises(ValueError, match="mixed"):
        L.call("aon_mlp_art_pack_mixed", None, 4, p, None)
    a = L.AonGemmArgs(M=2, N=4, K=3, A=16, lda=3, a_kc=1, B=16, ldb=4, b_kc=0, b_rdiv=1, C=16,
                      ldc=4, a_scale=1.0, b_scale=1.0, exact_fp32=1, n_store=2)
    with pytest.raises(ValueError, match="n_store"):
        L.call("aon_gemm", ctypes.byref(a), None, 0, None)


def test_abi11_argument_checks(L):
    """ABI 11: the articulated training forward keeps pos_enc(x') tiled with 16-byte stores, so
    enc must be 16-byte aligned, and the bf16 entry requires enc_bf (its fp32 enc keeps x' only)."""
    p, odd = ctypes.c_void_p(16), ctypes.c_void_p(20)
    with pytest.raises(ValueError, match="enc_bf"):
        L.call("aon_mlp_art_fwd_train_bf16", p, p, p, p, p, 1, 1, None, p, p, p, p, p, p, p, p,
               None, 4, None)
    with pytest.raises(ValueError, match="enc must be 16-byte aligned"):
        L.call("aon_mlp_art_fwd_train", p, p, p, p, p, 1, 1, None, p, p, p, p, odd, p, p, p, None)
    with pytest.raises(ValueError, match="16-byte aligned"):
        L.call("aon_mlp_art_bwd", p, p, p, odd, 1, p, p, p, p, p, p, None)


def test_pdf_shape_limits(L):
    with pytest.raises(ValueError, match="bad shape"):
        L.call("aon_sample_pdf", ctypes.c_void_p(16), 0, ctypes.c_void_p(16), 0, 4, 1000, 128,
               ctypes.c_void_p(16), 0, None, 0, None, None, ctypes.c_void_p(16), None, None)


def test_cpu_tensors_rejected():
    import torch
    from aonerf import helper

    with pytest.raises(ValueError, match="MI355X only"):
        helper.pos_enc(torch.zeros(4, 3), 0, 10)


def _fake_pairs(shapes):
    """(weight, bias) stand-ins with the given shapes: the C side only reads the shape fields
    before it refuses, so the pointers are never dereferenced."""
    import torch

    return [(torch.empty(o, i), torch.empty(o)) for o, i in shapes]


def _struct_with(L, cls, n, shapes):
    prm = cls()
    for i, (o, k) in enumerate(shapes):
        prm.w_rows[i], prm.w_cols[i], prm.b_len[i] = o, k, o
    # every pointer non-null: only the shape check stands between the struct and a launch
    for name, typ in cls._fields_:
        if name.endswith(("_w", "_b")):
            v = getattr(prm, name)
            if isinstance(v, int) or v is None:
                setattr(prm, name, 16)
            else:
                for j in range(len(v)):
                    v[j] = 16
    return prm


def _registration_order(mlp):
    ps = list(mlp.parameters())
    return [(ps[2 * i], ps[2 * i + 1]) for i in range(len(ps) // 2)]


def test_registration_order_rejected_python(L):
    """nn.Module.parameters() in registration order (pts_linears, views_linear,
    bottleneck, density, rgb) is not the kernels' layer order.  The Python builders refuse it
    with ValueError naming the layer -- before any pointer exists -- for both MLPs, and the
    training path's _params_struct (train.py / train_art.py) goes through them."""
    from aonerf import train, train_art
    from aonerf.model import NeRFMLP
    from aonerf.model_autodecoder import NeRFMLP as ArtMLP

    mlp = NeRFMLP(0, 10, 4)
    reg = _registration_order(mlp)
    with pytest.raises(ValueError, match="density_layer.*layer order"):
        L.mlp_params(reg)
    with pytest.raises(ValueError, match="density_layer.*layer order"):
        train._params_struct(reg)
    # the kernels' order passes the shape check (and then needs GPU tensors)
    good = [(m.weight, m.bias) for m in mlp._layers()]
    with pytest.raises(ValueError, match="GPU tensor"):
        L.mlp_params(good)
    with pytest.raises(ValueError, match="12 \\(weight, bias\\) pairs"):
        L.mlp_params(good[:11])
    art = ArtMLP(0, 10, 4)
    reg = _registration_order(art)
    with pytest.raises(ValueError, match="density_layer.*layer order"):
        L.mlp_art_params(reg)
    with pytest.raises(ValueError, match="density_layer.*layer order"):
        train_art._params_struct(reg)
    good = [(m.weight, m.bias) for m in train_art.art_layers(art)]
    with pytest.raises(ValueError, match="GPU tensor"):
        L.mlp_art_params(good)


def test_registration_order_rejected_c(L):
    """The same refusal on the C side (aon_mlp_params / aon_mlp_art_params carry the shapes,
    ABI 9): every pack returns < 0 naming the layer before any launch -- no GPU needed."""
    reg = [(256, 63)] + [(256, 256)] * 4 + [(256, 319), (256, 256), (256, 256), (128, 283),
                                             (256, 256), (1, 256), (3, 128)]
    prm = _struct_with(L, L.AonMlpParams, 12, reg)
    for fn, args in (("aon_mlp_pack", (1, ctypes.c_void_p(16), None)),
                     ("aon_mlp_bwd_pack", (ctypes.c_void_p(16), None)),
                     ("aon_mlp_bwd_pack_bf16", (ctypes.c_void_p(16), None))):
        with pytest.raises(ValueError, match=f"{fn}: density_layer: weight 128 x 283"):
            L.call(fn, ctypes.byref(prm), *args)
    art_reg = ([(128, 163)] + [(128, 128)] * 3 + [(3, 128), (256, 191)] + [(256, 256)] * 4 +
               [(256, 447), (256, 256), (256, 256), (128, 411)] + [(128, 128)] * 3 +
               [(256, 256), (1, 256), (3, 128)])
    prm = _struct_with(L, L.AonMlpArtParams, 20, art_reg)
    for fn in ("aon_mlp_art_pack", "aon_mlp_art_pack_bf16", "aon_mlp_art_bwd_pack",
               "aon_mlp_art_bwd_pack_bf16"):
        with pytest.raises(ValueError, match=f"{fn}: density_layer: weight 128 x 411"):
            L.call(fn, ctypes.byref(prm), ctypes.c_void_p(16), None)
    # a latent-carrying layer narrower than its per-sample columns
    ok = list(L.ART_SHAPES)
    ok[10] = (256, 300)
    prm = _struct_with(L, L.AonMlpArtParams, 20, ok)
    with pytest.raises(ValueError, match="pts_linears.5: weight 256 x 300.*>= 319"):
        L.call("aon_mlp_art_pack", ctypes.byref(prm), ctypes.c_void_p(16), None)


def test_gemm_small_batch_validation(L):
    """aon_gemm_small_batch refuses, before any launch: a product off the exact-fp32 tiny path,
    two products on one C that differ in shape or do not accumulate, and overlapping outputs
    (column slices of one matrix at the same row stride do not overlap)."""
    def args(C, M, N, K, ldc, acc=0, exact=1):
        return L.AonGemmArgs(M=M, N=N, K=K, A=16, lda=K, a_kc=1, B=16, ldb=K, b_kc=1, C=C,
                             ldc=ldc, accumulate=acc, a_scale=1.0, b_scale=1.0, exact_fp32=exact)

    def run(*items):
        arr = (L.AonGemmArgs * len(items))(*items)
        L.call("aon_gemm_small_batch", arr, len(items), None)

    with pytest.raises(ValueError, match="exact_fp32 tiny products only"):
        run(args(4096, 4, 4, 4, 4, exact=0))
    with pytest.raises(ValueError, match="match in shape and accumulate"):
        run(args(4096, 4, 4, 4, 4), args(4096, 4, 4, 4, 4, acc=0))
    with pytest.raises(ValueError, match="outputs overlap"):
        run(args(1 << 20, 8, 8, 4, 16), args((1 << 20) + 4 * 4, 8, 8, 4, 16))
