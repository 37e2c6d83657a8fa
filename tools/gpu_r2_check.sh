#!/bin/bash
# Round-2 first GPU pass: GPU test tier, smoke, the driver-shaped headline bench (20 steps / 5
# warmup) next to long runs, and a kernel trace of the short run (where its wall time goes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
for s in "20 5" "200 20" "20000 2000"; do
  set -- $s
  timeout -k 10 300 python bench.py --steps $1 --warmup $2 > gpurun_out/bench_weather_s$1.log 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_w20 -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof_w20.log 2>&1 || exit $?
