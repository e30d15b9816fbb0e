"""Per-step kernel time of a training bench run from its rocprofv3 kernel trace (csv): the last
STEPS steps, delimited by the Adam launch that ends each step (aon::k_adam):

    python scripts/train_step_breakdown.py KERNEL_TRACE_CSV [STEPS=10]

Prints the step span, kernels and busy time per step, then every kernel's ms and launches per
step, largest first."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
ends = [i for i, x in enumerate(iv) if "k_adam" in x[2]]
if len(ends) < steps + 1:
    sys.exit(f"only {len(ends)} Adam launches in the trace")
seg = iv[ends[-steps - 1] + 1:ends[-1] + 1]
span = (seg[-1][1] - seg[0][0]) / 1e6
tot = collections.defaultdict(lambda: [0, 0])
for s, e, n in seg:
    k = n.split("(")[0][:100]
    tot[k][0] += e - s
    tot[k][1] += 1
busy = sum(v[0] for v in tot.values()) / 1e6
print(f"{steps} steps: span {span / steps:.3f} ms/step, {len(seg) / steps:.1f} kernels/step, "
      f"kernel time {busy / steps:.3f} ms/step")
for k, v in sorted(tot.items(), key=lambda kv: -kv[1][0]):
    print(f"{v[0] / 1e6 / steps:8.3f} ms {v[1] / steps:5.1f}  {k}")
