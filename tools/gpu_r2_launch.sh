#!/bin/bash
# Bound-launch check: its GPU test, the launch-overhead probe and the driver-shaped bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "bound or fused_train" > gpurun_out/pytest_bound.log 2>&1 || exit $?
timeout -k 10 120 python tools/launch_overhead.py > gpurun_out/launch_overhead.log 2>&1 || exit $?
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_s20_$i.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
