#!/usr/bin/env python3
"""One steady-state step of a rocprofv3 kernel trace, kernel by kernel.

    python tools/trace_step.py <run_kernel_trace.csv> <first-kernel-of-step substring> [step index from the end]
                               [substring every counted step must contain]

Prints, for the chosen step (default: the 3rd-last occurrence of the marker kernel, i.e. inside the
timed window), every kernel dispatch from that marker to the next one: start offset, duration, the gap
to the previous kernel's end on ANY queue, the queue id, grid and name; then the sum of kernel
durations against the wall span, and the busiest kernels."""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    marker = sys.argv[2]
    back = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    rows.sort(key=lambda r: r["s"])
    must = sys.argv[4] if len(sys.argv) > 4 else None
    idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    if must:  # keep markers whose step (up to the next marker) contains `must` (training, not eval)
        keep = []
        for j, i in enumerate(idx):
            end = idx[j + 1] if j + 1 < len(idx) else len(rows)
            if any(must in r["Kernel_Name"] for r in rows[i:end]):
                keep.append(i)
        idx = keep + [idx[-1]]
    if len(idx) < back + 1:
        raise SystemExit(f"marker {marker!r} seen {len(idx)} times")
    a, b = idx[-back - 1], idx[-back]
    step = rows[a:b]
    t0 = step[0]["s"]
    prev_end = rows[a - 1]["e"] if a else t0
    busy = 0
    print(f"{'start':>8} {'dur':>7} {'gap':>7} {'queue':>5} {'grid':>8}  kernel (us)")
    for r in step:
        gap = (r["s"] - prev_end) / 1e3
        dur = (r["e"] - r["s"]) / 1e3
        busy += dur
        q = r.get("Queue_Id", r.get("Stream_Id", "?"))
        grid = r.get("Grid_Size_X", r.get("Grid_Size", "?"))
        print(f"{(r['s'] - t0) / 1e3:8.1f} {dur:7.2f} {gap:7.2f} {q:>5} {grid:>8}  {r['Kernel_Name'][:100]}")
        prev_end = max(prev_end, r["e"])
    span = (rows[b]["s"] - t0) / 1e3
    print(f"step span {span:.1f} us (marker to marker), sum of kernel durations {busy:.1f} us, "
          f"{len(step)} dispatches")


if __name__ == "__main__":
    main()
