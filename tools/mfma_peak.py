#!/usr/bin/env python3
"""Measured MFMA peaks on this MI355X: one JSON line with TFLOP/s of
back-to-back v_mfma_f32_16x16x32_f16, v_mfma_f32_16x16x4_f32 and the f16x3 triple on random
register operands, every CU busy (tools/mfma_peak.hip, built by __graft_entry__.build() into
articulated-object-nerf_amd/lib/libaon_mfma_peak.so).

    python tools/mfma_peak.py [--iters 20000]
"""
import argparse
import ctypes
import json
import os

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "articulated-object-nerf_amd", "lib", "libaon_mfma_peak.so")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20000)
    args = ap.parse_args()
    lib = ctypes.CDLL(LIB)
    lib.aon_mfma_peak.restype = ctypes.c_double
    lib.aon_mfma_peak.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                  ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)]
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    blocks = cus * 8  # 8 x 4 waves per CU: 8 waves per SIMD in flight
    out = torch.empty(blocks * 256, device="cuda")
    stamps = torch.zeros(2, dtype=torch.int64, device="cuda")
    res = {"cus": cus, "blocks": blocks, "iters": args.iters}
    for name, kind, iters in (("f16_16x16x32", 0, args.iters), ("f32_16x16x4", 1, args.iters // 4),
                              ("f16x3_triple_16x16x32", 2, args.iters // 3)):
        clk = ctypes.c_double(0.0)
        res[name + "_tflops"] = lib.aon_mfma_peak(kind, iters, blocks, ctypes.c_void_p(out.data_ptr()),
                                                  ctypes.c_void_p(stamps.data_ptr()), ctypes.byref(clk))
        res[name + "_clock_ghz"] = clk.value
    res["spec_tflops"] = {"f16_dense": 2500.0, "f32_matrix": 157.3}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
