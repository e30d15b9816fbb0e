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
    ap.add_argument("--mix", action="store_true", help="also the fine MLP's instruction mix (k_mfma_mix)")
    ap.add_argument("--out", default=None, help="also write the JSON here")
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
                              ("f16x3_triple_16x16x32", 2, args.iters // 3),
                              ("f16_32x32x16", 3, args.iters), ("f16x3_triple_32x32x16", 4, args.iters // 3)):
        clk = ctypes.c_double(0.0)
        res[name + "_tflops"] = lib.aon_mfma_peak(kind, iters, blocks, ctypes.c_void_p(out.data_ptr()),
                                                  ctypes.c_void_p(stamps.data_ptr()), ctypes.byref(clk))
        res[name + "_clock_ghz"] = clk.value
    res["spec_tflops"] = {"f16_dense": 2500.0, "f32_matrix": 157.3}
    if args.mix:
        res["mix"] = mix(lib, cus, args.iters)
    print(json.dumps(res))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


# one v_mfma_f32_16x16x32_f16 = 2 x 16 x 16 x 32 FLOP in 16 cycles of one SIMD (4 SIMDs per CU):
# issued TFLOP/s / (SIMDs x 1024 FLOP) = the MFMA-pipe rate in GHz-equivalent ("MFMA busy x
# held clock"), which the fine MLP sustains at ~1.3
FLOP_PER_SIMD_CYCLE = 2 * 16 * 16 * 32 / 16


def mix(lib, cus, iters):
    """k_mfma_mix (tools/mfma_peak.hip): the streamed MLP kernel's per-wave mix -- per MFMA 1.25
    v_fma_f32 and 0.75 ds_read_b128 (+0.125 ds_write_b128) -- with no true dependencies, one
    512-thread workgroup per CU; each component alone and together."""
    lib.aon_mfma_mix.restype = ctypes.c_double
    lib.aon_mfma_mix.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                 ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)]
    blocks = 2 * cus
    out = torch.empty(blocks * 512, device="cuda")
    stamps = torch.zeros(2, dtype=torch.int64, device="cuda")
    iters = iters // 3 * 3
    simds = 4 * cus
    names = {0: "mfma_only", 1: "mfma+valu", 2: "mfma+lds_read", 3: "mfma+valu+lds_read",
             7: "mfma+valu+lds_read+lds_write"}
    res = {"blocks": blocks, "iters": iters, "waves_per_simd": 2,
           "per_mfma": {"v_fma_f32": 1.25, "ds_read_b128": 0.75, "ds_write_b128": 0.125},
           "fine_mlp_per_mfma": {"valu": 4216 / 3516, "ds_read_b128": 2515 / 3516,
                                 "source": "profiles/r02/counters_ncol1.json (DESIGN.md §4)"},
           "fine_mlp_ghz_equivalent": 1381e12 / (simds * FLOP_PER_SIMD_CYCLE) / 1e9}
    for k, name in names.items():
        clk = ctypes.c_double(0.0)
        tf = lib.aon_mfma_mix(k, iters, blocks, ctypes.c_void_p(out.data_ptr()),
                              ctypes.c_void_p(stamps.data_ptr()), ctypes.byref(clk))
        ghz_eq = tf * 1e12 / (simds * FLOP_PER_SIMD_CYCLE) / 1e9
        res[name] = {"issued_tflops": tf, "clock_ghz": clk.value, "ghz_equivalent": ghz_eq,
                     "mfma_busy": ghz_eq / clk.value if clk.value else None}
    return res


if __name__ == "__main__":
    main()
