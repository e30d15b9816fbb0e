"""Effective clock per kernel from a GRBM_GUI_ACTIVE pass (MI355X_MICROARCH.md 'DVFS give-back':
GRBM_GUI_ACTIVE summed over the 8 XCDs / 8 / the dispatch's duration), mean over dispatches of
each (kernel, grid):  python scripts/clock_summary.py <run_counter_collection.csv> [OUT.json]"""
import csv
import json
import sys
from collections import defaultdict

acc = defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if r["Counter_Name"] != "GRBM_GUI_ACTIVE":
        continue
    dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    if dur <= 0:
        continue
    acc[f"{r['Kernel_Name'][:70]} grid {r['Grid_Size']}"].append(float(r["Counter_Value"]) / 8 / dur / 1e9)
out = {k: round(sum(v) / len(v), 3) for k, v in acc.items() if len(v) and "rocclr" not in k}
if len(sys.argv) > 2:
    json.dump(out, open(sys.argv[2], "w"), indent=1)
for k, v in out.items():
    print(f"{v:6.3f} GHz  {k}")
