#!/usr/bin/env python3
"""Kernel statistics from a rocprofv3 SQLite (rocpd) output: tools/rocpd_stats.py RUN_results.db [TOP]
Prints per kernel: calls, total / mean / min / max duration (us), share of the total kernel time."""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
top = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rows = db.execute(
    "select s.kernel_name, count(*), sum(d.end - d.start), min(d.end - d.start), max(d.end - d.start) "
    "from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id "
    "group by s.kernel_name order by 3 desc").fetchall()
tot = sum(r[2] for r in rows) or 1
print(f"{'calls':>7} {'total_us':>11} {'mean_us':>9} {'min_us':>9} {'max_us':>9} {'share':>6}  kernel")
for name, n, t, mn, mx in rows[:top]:
    print(f"{n:7d} {t / 1e3:11.1f} {t / n / 1e3:9.2f} {mn / 1e3:9.2f} {mx / 1e3:9.2f} {100 * t / tot:5.1f}%  {name[:110]}")
