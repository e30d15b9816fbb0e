#!/usr/bin/env python3
"""Per-kernel counter utilisation from scripts/prof_train_counters.sh: python
scripts/train_ctr_summary.py gpurun_out/OUT [dst.json].  Sums every dispatch of a kernel (both
levels, all steps): MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8),
LDS busy = SQ_LDS_IDX_ACTIVE / (256 CUs x cycles), instruction mix per wave."""
import csv
import glob
import json
import sys


def agg(path):
    f = glob.glob(f"{path}/**/*counter_collection.csv", recursive=True)
    per = {}
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"].split("(")[0][:90]
        d = per.setdefault(k, {"waves": 0.0, "disp": set()})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        if r["Dispatch_Id"] not in d["disp"]:
            d["disp"].add(r["Dispatch_Id"])
            d["waves"] += int(r["Grid_Size"]) / 64
    return per


def agg_opt(path, k):
    if not glob.glob(f"{path}/**/*counter_collection.csv", recursive=True):
        return None
    return agg(path).get(k)


def main():
    src = sys.argv[1]
    a, b = agg(f"{src}/A"), agg(f"{src}/B")
    res = {}
    for k in b:
        if k not in a or "GRBM_GUI_ACTIVE" not in b[k]:
            continue
        cyc = b[k]["GRBM_GUI_ACTIVE"] / 8
        if cyc < 1e5:
            continue
        w = b[k]["waves"]
        c_, d_ = agg_opt(f"{src}/C", k), agg_opt(f"{src}/D", k)
        e_ = agg_opt(f"{src}/E", k)
        disp = len(b[k]["disp"])
        extra = {}
        if c_ and d_:  # HBM bytes per dispatch: FETCH_SIZE doubled (gfx950), KiB units
            extra["fetch_bytes_per_dispatch"] = 2 * 1024 * c_["FETCH_SIZE"] / disp
            extra["write_bytes_per_dispatch"] = 1024 * d_["WRITE_SIZE"] / disp
        if e_:
            extra["vmem_wr_per_wave"] = e_["SQ_INSTS_VMEM_WR"] / w
            extra["vmem_rd_per_wave"] = e_["SQ_INSTS_VMEM_RD"] / w
            extra["salu_per_wave"] = e_["SQ_INSTS_SALU"] / w
            extra["vmem_wr_issue_frac"] = e_["SQ_INST_CYCLES_VMEM_WR"] / e_["SQ_WAVE_CYCLES"]
        res[k] = {"dispatches": disp, "mfma_busy": a[k]["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * cyc),
                  "lds_busy": b[k]["SQ_LDS_IDX_ACTIVE"] / (256 * cyc),
                  "wait_inst_any_frac": a[k]["SQ_WAIT_INST_ANY"] / a[k]["SQ_WAVE_CYCLES"],
                  "wait_inst_lds_frac": a[k]["SQ_WAIT_INST_LDS"] / a[k]["SQ_WAVE_CYCLES"],
                  "mfma_per_wave": b[k]["SQ_INSTS_MFMA"] / w,
                  "valu_non_mfma_per_wave": (b[k]["SQ_INSTS_VALU"] - b[k]["SQ_INSTS_MFMA"]) / w,
                  "lds_per_wave": b[k]["SQ_INSTS_LDS"] / w,
                  "valu_mfma_coexec_frac": b[k]["SQ_VALU_MFMA_COEXEC_CYCLES"] / (1024 * cyc),
                  "active_valu_frac": b[k]["SQ_ACTIVE_INST_VALU"] / (1024 * cyc), **extra}
    print(json.dumps(res, indent=1))
    if len(sys.argv) > 2:
        json.dump(res, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
