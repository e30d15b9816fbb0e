#!/usr/bin/env python3
"""Per-wave and per-ray instruction / wait summary of the fused march from a
scripts/prof_march_counters.sh session:  python scripts/march_ctr_summary.py gpurun_out/ctr_march out.json
SQ_*_CYCLES and SQ_WAIT_* count quad-cycles (MI355X_MICROARCH.md PMC units); cycles per SIMD =
GRBM_GUI_ACTIVE / 8 XCDs."""
import csv
import glob
import json
import os
import sys


def agg(path):
    f = glob.glob(f"{path}/**/*counter_collection.csv", recursive=True)
    out = {}
    for r in csv.DictReader(open(f[0])):
        if "march" not in r["Kernel_Name"]:
            continue
        out[r["Counter_Name"]] = out.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def main():
    src, dst = sys.argv[1], sys.argv[2]
    res = {}
    for lib in sorted(d for d in os.listdir(src) if os.path.isdir(os.path.join(src, d))):
        c = {}
        for p in ("A", "B"):
            c.update(agg(os.path.join(src, lib, p)))
        waves = c.get("SQ_WAVES", 0.0) or 1.0
        t = json.loads([ln for ln in open(os.path.join(src, f"{lib}.timing.json")) if ln.startswith("{")][-1])
        rays = 307200
        r = {"timing": t, "waves": waves, "rays_per_wave": rays / waves}
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
                  "SQ_INSTS_SMEM"):
            r[k + "_per_wave"] = c.get(k, 0.0) / waves
            r[k + "_per_ray"] = c.get(k, 0.0) / rays
        for k in ("SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                  "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
            r[k] = c.get(k, 0.0)
        wc = c.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        r["wait_frac_of_wave_cycles"] = c.get("SQ_WAIT_ANY", 0.0) / wc
        r["wait_inst_frac"] = c.get("SQ_WAIT_INST_ANY", 0.0) / wc
        r["active_valu_frac"] = c.get("SQ_ACTIVE_INST_VALU", 0.0) / wc
        r["grbm_gui_active"] = c.get("GRBM_GUI_ACTIVE", 0.0)
        res[lib] = r
    json.dump(res, open(dst, "w"), indent=1)
    for lib, r in res.items():
        print(lib, {k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items() if "per_ray" in k or "frac" in k},
              r["timing"]["ms"])


if __name__ == "__main__":
    main()
