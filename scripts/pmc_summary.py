#!/usr/bin/env python3
"""Summarise a scripts/gpu_round.sh session into profiles/<name>/.

    python scripts/pmc_summary.py gpurun_out/r01a profiles/r01_fp32 [--precision fp32] (default f16x3, the headline)

Copies the rocprofv3 kernel stats, and turns the FETCH_SIZE / WRITE_SIZE passes into per-launch
HBM bytes per kernel (MI355X_MICROARCH.md "HBM": both counters in KiB; gfx950 FETCH_SIZE counts
half the bytes of a wide coalesced stream, so it is doubled).  Writes profiles/pmc_traffic.json
for bench.py's roofline.traffic (fine-level MLP launch).
"""
import csv
import json
import os
import shutil
import sys


def load(path, counter):
    out = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        key = (r["Kernel_Name"].split("(")[0], int(r["Grid_Size"]))
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        out.setdefault(key, []).append((float(r["Counter_Value"]), dur))
    return out


def main():
    src, dst = sys.argv[1], sys.argv[2]
    precision = sys.argv[sys.argv.index("--precision") + 1] if "--precision" in sys.argv else "f16x3"
    os.makedirs(dst, exist_ok=True)
    for name in ("kt/run_kernel_stats.csv", "bench.json", "pytest_gpu.log"):
        p = os.path.join(src, name)
        if os.path.exists(p):
            shutil.copy(p, os.path.join(dst, os.path.basename(name)))
    trace = os.path.join(src, "kt/run_kernel_trace.csv")
    if os.path.exists(trace):  # per (kernel, grid) averages: coarse / fine launches share names
        acc = {}
        for r in csv.DictReader(open(trace)):
            key = (r["Kernel_Name"].split("(")[0], int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]))
            dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            acc.setdefault(key, []).append(dur)
        with open(os.path.join(dst, "kernel_trace_by_grid.csv"), "w") as f:
            f.write("kernel,grid,calls,avg_ns,total_ns\n")
            for (k, g), v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
                f.write(f"\"{k}\",{g},{len(v)},{sum(v) / len(v):.0f},{sum(v)}\n")
    fetch = load(os.path.join(src, "pmc_fetch/run_counter_collection.csv"), "FETCH_SIZE")
    write = load(os.path.join(src, "pmc_write/run_counter_collection.csv"), "WRITE_SIZE")
    rows = []
    for key in sorted(fetch, key=lambda k: -k[1]):
        if key not in write or "rocclr" in key[0]:
            continue
        f = sum(v for v, _ in fetch[key]) / len(fetch[key])
        w = sum(v for v, _ in write[key]) / len(write[key])
        d = sum(t for _, t in fetch[key]) / len(fetch[key])
        hbm = (2 * f + w) * 1024
        rows.append({"kernel": key[0], "grid": key[1], "fetch_kib_raw": f, "write_kib": w,
                     "hbm_bytes_per_launch": hbm, "duration_s_profiled": d,
                     "hbm_gbs": hbm / d / 1e9})
    json.dump(rows, open(os.path.join(dst, "pmc_hbm.json"), "w"), indent=1)
    tag = "mlp_fwd_f16x3<0, 1, false" if precision == "f16x3" else "mlp_fwd_f32"
    mlp = [r for r in rows if tag in r["kernel"]]
    if mlp:
        fine = max(mlp, key=lambda r: r["grid"])
        json.dump({"precision": precision, "world": 1, "fine_mlp_hbm_bytes": fine["hbm_bytes_per_launch"],
                   "source": dst, "kernel": fine["kernel"], "grid": fine["grid"],
                   "note": "(2*FETCH_SIZE + WRITE_SIZE) KiB per launch, separate --pmc passes"},
                  open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "profiles", "pmc_traffic.json"), "w"), indent=1)
    for r in rows:
        print(f"{r['kernel'][:40]:40s} grid {r['grid']:>10d}  {r['hbm_bytes_per_launch'] / 1e6:10.1f} MB"
              f"  {r['hbm_gbs']:8.1f} GB/s")


if __name__ == "__main__":
    main()
