#!/bin/bash
# Row-parallel weather kernel: fused-MLP numerics tests, trainer/xgmi tests, launch probe, benches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_trainer_gpu.py tests/test_xgmi_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_rows.log 2>&1 || exit $?
timeout -k 10 120 python tools/launch_overhead.py > gpurun_out/launch_overhead_rows.log 2>&1 || exit $?
timeout -k 10 120 python tools/bench_window_probe.py > gpurun_out/window_probe_rows.log 2>&1 || exit $?
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_rows_s20_$i.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py > gpurun_out/bench_rows_default.log 2>&1 || exit $?
DCT_MLP_ROWS=0 timeout -k 10 300 python bench.py > gpurun_out/bench_wave_default.log 2>&1 || exit $?
