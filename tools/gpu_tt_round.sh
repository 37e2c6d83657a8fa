#!/bin/bash
# TabTransformer round: kernel/model GPU tests, bench, rocprofv3 kernel stats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_tabtransformer.py tests/test_trainer_gpu.py tests/test_kernels_gpu.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/pytest_tt_round.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --model tabtransformer > gpurun_out/bench_tt.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tt -o run --output-format csv -- \
  python3 bench.py --model tabtransformer --rows 1000000 --steps 50 --warmup 5 > gpurun_out/prof_tt.log 2>&1 || exit $?
