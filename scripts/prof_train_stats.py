"""Summarise a rocprofv3 kernel_stats.csv per training step: python scripts/prof_train_stats.py CSV STEPS"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2])
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot / 1e6 / steps:.3f} ms/step (kernel time, {steps} steps incl. warm-up)")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:22]:
    print(f"{float(r['TotalDurationNs']) / 1e6 / steps:8.3f} ms/step {int(r['Calls']) / steps:5.1f} calls "
          f"{float(r['AverageNs']) / 1e3:8.1f} us  {r['Name'][:100]}")
