"""Per-kernel breakdown of ONE steady-state training step from a rocprofv3 kernel_trace CSV.

Steps are delimited by the optimizer kernel (default adam_flat); prints the last complete step.
Usage: python tools/step_breakdown.py <kernel_trace.csv> [delimiter-substring]"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
delim = sys.argv[2] if len(sys.argv) > 2 else "adam_flat"
ends = [i for i, r in enumerate(rows) if delim in r["Kernel_Name"]]
a, b = ends[-2], ends[-1]
agg = collections.defaultdict(lambda: [0, 0])
for r in rows[a + 1: b + 1]:
    k = r["Kernel_Name"][:100]
    agg[k][0] += 1
    agg[k][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
busy = 0
for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{t / 1e3:8.1f} us {n:4d}x  {k}")
    busy += t
window = int(rows[b]["End_Timestamp"]) - int(rows[a]["End_Timestamp"])
print(f"kernels {b - a}  busy {busy / 1e3:.1f} us  window {window / 1e3:.1f} us")
