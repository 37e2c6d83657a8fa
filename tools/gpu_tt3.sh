#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_tabtransformer.py -m gpu -x -v \
  -k "tt_ or hip_path or hip_fit or gemm" --timeout 120 --timeout-method thread > gpurun_out/pytest_tt3.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --model tabtransformer > gpurun_out/bench_tt.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tt -o run --output-format csv -- \
  python3 bench.py --model tabtransformer --rows 1000000 --steps 50 --warmup 5 > gpurun_out/prof_tt.log 2>&1 || exit $?
