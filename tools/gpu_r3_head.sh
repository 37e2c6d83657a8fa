#!/bin/bash
# Round 3 re-entry check at HEAD: full GPU tier, smoke, the driver's bench command, a long run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > $O/pytest_gpu_head.log 2>&1
rc=$?; tail -6 $O/pytest_gpu_head.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_head.log 2>&1 || exit $?
tail -2 $O/smoke_head.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_head_s20.log 2>&1 || exit $?
grep '^{' $O/bench_head_s20.log | cut -c1-600
timeout -k 10 300 python bench.py --steps 20000 --warmup 2000 --no-reference-model > $O/bench_head_long.log 2>&1 || exit $?
grep '^{' $O/bench_head_long.log | cut -c1-400
echo done
