"""Summarise a rocprofv3 kernel_stats CSV per step: python tools/kstats.py <csv> <steps> [top]."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
    print(f'{float(r["TotalDurationNs"]) / 1e3 / steps:9.1f} us/step {int(r["Calls"]) / steps:6.1f} calls '
          f'{float(r["AverageNs"]) / 1e3:8.1f} us  {r["Name"][:110]}')
print(f"total {tot / 1e3 / steps:.1f} us/step")
