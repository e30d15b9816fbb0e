#!/usr/bin/env python3
"""Counter-based utilisation of the fused MLP kernel from a scripts/prof_counters.sh session:

    python scripts/ctr_summary.py gpurun_out/ctr4 profiles/r01_f16x3/counters.json [KERNEL]

KERNEL: a substring of the kernel name (default "f16x3", the fused MLP); the last launch of it
in each pass is summarised.

MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x cycles), LDS busy = SQ_LDS_IDX_ACTIVE / (CUs x
cycles), cycles = GRBM_GUI_ACTIVE / 8 XCDs (MI355X_MICROARCH.md), L2 hit rate, dynamic
instruction mix per wave.  Counter passes are separate runs of tools/prof_mlp.py (same launch).
"""
import csv
import glob
import json
import sys


def agg(path, kernel="f16x3"):
    f = glob.glob(f"{path}/**/*counter_collection.csv", recursive=True)
    out, grid, dur = {}, 0, 0.0
    for r in csv.DictReader(open(f[0])):
        if kernel not in r["Kernel_Name"]:
            continue
        out[r["Counter_Name"]] = out.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        grid = int(r["Grid_Size"])
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    return out, grid, dur


def main():
    src, dst = sys.argv[1], sys.argv[2]
    kern = sys.argv[3] if len(sys.argv) > 3 else "f16x3"
    a, grid, dur_a = agg(f"{src}/A", kern)
    b, _, dur_b = agg(f"{src}/B", kern)
    c, _, _ = agg(f"{src}/C", kern)
    cus, simds = 256, 1024
    cycles = b["GRBM_GUI_ACTIVE"] / 8
    waves = grid / 64
    res = {
        "kernel": kern, "grid_threads": grid,
        "duration_ms_profiled": dur_b * 1e3, "clock_ghz_profiled": cycles / dur_b / 1e9,
        "mfma_busy_frac": a["SQ_VALU_MFMA_BUSY_CYCLES"] / (simds * cycles),
        "lds_busy_frac": b["SQ_LDS_IDX_ACTIVE"] / (cus * cycles),
        "lds_bank_conflict_cycles": a["SQ_LDS_BANK_CONFLICT"],
        "wait_inst_any_frac_of_wave_cycles": a["SQ_WAIT_INST_ANY"] / a["SQ_WAVE_CYCLES"],
        "l2_hit_rate": c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]),
        "per_wave": {"mfma": b["SQ_INSTS_MFMA"] / waves,
                     "valu_non_mfma": (b["SQ_INSTS_VALU"] - b["SQ_INSTS_MFMA"]) / waves,
                     "lds": b["SQ_INSTS_LDS"] / waves},
        "note": "MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE/8); profiled "
                "passes run a lower clock than unprofiled ones (DVFS), so compare fractions",
        "raw": {"A": a, "B": b, "C": c},
    }
    json.dump(res, open(dst, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "raw"}, indent=1))


if __name__ == "__main__":
    main()
