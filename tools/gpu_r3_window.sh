#!/bin/bash
# Round 3: the driver's 20-step window of bench.py - where the extra ~0.3 ms of some processes goes
# (enqueue vs completion wait), with the cyclic GC paused in the window (default) or left on.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out
: > $O/window.log
for i in 1 2 3; do
  for g in on pause collect; do
    DCT_BENCH_GC=$g DCT_BENCH_DEBUG=1 DCT_BENCH_DEBUG_REPEAT=2 timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 \
      > $O/win_$g.log 2>&1 || exit 1
    { echo "== run $i gc_on_in_window=$g"; grep "bench debug" $O/win_$g.log; } >> $O/window.log
  done
done
cat $O/window.log
