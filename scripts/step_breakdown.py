"""One training step's kernels from a rocprofv3 kernel trace of tools/prof_train_step.py: the
last complete step (between the last two Adam launches), per kernel duration and the gap before
it, plus the step's span and busy time.   python scripts/step_breakdown.py <run_kernel_trace.csv>"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
adam = [i for i, r in enumerate(rows) if "k_adam" in r["Kernel_Name"]]
# a step's Adam may be several launches in a row (AON_ADAM_MAX_TENSORS per launch): the step
# starts after the last launch of the previous group
ends = [i for j, i in enumerate(adam) if j + 1 == len(adam) or adam[j + 1] != i + 1]
st = rows[ends[-2] + 1:ends[-1] + 1]
t0, t1 = int(st[0]["Start_Timestamp"]), int(st[-1]["End_Timestamp"])
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in st)
print(f"step span {(t1 - t0) / 1e6:.3f} ms, kernels busy {busy / 1e6:.3f} ms, {len(st)} kernels")
prev = None
for r in st:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(e - s) / 1e3:9.1f} us  gap {(s - prev) / 1e3 if prev else 0:6.1f}  "
          f"{r['Kernel_Name'][:100]}")
    prev = e
