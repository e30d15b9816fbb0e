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
    assert lib.aon_abi_version() == 8
    assert lib.aon_mlp_packed_bytes(0) == 2368 * 1024 + 2464 * 4 + 16  # + the status block
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


def test_pdf_shape_limits(L):
    with pytest.raises(ValueError, match="bad shape"):
        L.call("aon_sample_pdf", ctypes.c_void_p(16), 0, ctypes.c_void_p(16), 0, 4, 1000, 128,
               ctypes.c_void_p(16), 0, None, 0, None, None, ctypes.c_void_p(16), None, None)


def test_cpu_tensors_rejected():
    import torch
    from aonerf import helper

    with pytest.raises(ValueError, match="MI355X only"):
        helper.pos_enc(torch.zeros(4, 3), 0, 10)
