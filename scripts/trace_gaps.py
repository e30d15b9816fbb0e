"""GPU idle time between kernels in a rocprofv3 kernel trace (csv), over the trace's last
FRACTION of wall time (the timed steps of a bench run; warm-up and set-up fall in the front):

    python scripts/trace_gaps.py KERNEL_TRACE_CSV [FRACTION=0.5] [STEPS]

Prints the busy fraction (union of kernel intervals / span), the idle time, the number of
gaps above 2 / 10 / 50 us and, with STEPS (the timed steps inside that window), per step."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 0
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
t_end = max(e for _, e, _ in iv)
t_beg = iv[0][0]
cut = t_end - frac * (t_end - t_beg)
iv = [x for x in iv if x[0] >= cut]
span = iv[-1][1] - iv[0][0]
busy, cur_s, cur_e, gaps = 0, iv[0][0], iv[0][1], []
for s, e, _ in iv[1:]:
    if s > cur_e:
        busy += cur_e - cur_s
        gaps.append(s - cur_e)
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
idle = span - busy
print(f"kernels {len(iv)}  span {span / 1e6:.3f} ms  busy {busy / 1e6:.3f} ms ({busy / span:.3f})  "
      f"idle {idle / 1e6:.3f} ms")
for th in (2, 10, 50):
    g = [x for x in gaps if x > th * 1000]
    print(f"gaps > {th} us: {len(g)}  totalling {sum(g) / 1e6:.3f} ms")
if steps:
    print(f"per step: {len(iv) / steps:.1f} kernels, span {span / 1e6 / steps:.3f} ms, "
          f"busy {busy / 1e6 / steps:.3f} ms, idle {idle / 1e6 / steps:.3f} ms")
