"""Per-kernel totals from a rocprofv3 rocpd database (run_results.db) -> stdout, per step:
python scripts/rocpd_kernel_stats.py DB STEPS [CSV_OUT]"""
import csv
import sqlite3
import sys

con = sqlite3.connect(sys.argv[1])
steps = int(sys.argv[2])
q = """select k.kernel_name, count(*), sum(d.end - d.start), avg(d.end - d.start)
       from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol k on d.kernel_id = k.id
       group by k.kernel_name"""
rows = list(con.execute(q))
rows.sort(key=lambda r: -r[2])
tot = sum(r[2] for r in rows)
print(f"total kernel time {tot / 1e6 / steps:.3f} ms/step over {steps} steps")
for name, n, t, a in rows[:24]:
    print(f"{t / 1e6 / steps:8.3f} ms/step {n / steps:6.1f}/step {a / 1e3:8.1f} us  {name[:100]}")
if len(sys.argv) > 3:
    with open(sys.argv[3], "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs"])
        for r in rows:
            w.writerow(r)
