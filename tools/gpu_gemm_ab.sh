#!/bin/bash
# One gpurun session: GEMM numerics tests, pipeline-depth A/B on the tabular shapes, tabular bench
# (default vs 2-stage), rocprofv3 kernel stats of the tabular and TabTransformer steps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm" \
  > gpurun_out/pytest_gemm.log 2>&1 || exit $?
timeout -k 10 300 python tools/bench_gemm_mlp.py > gpurun_out/gemm_ab.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --model tabular-mlp-4x1024 > gpurun_out/bench_tab.log 2>&1 || exit $?
DCT_GEMM_STAGES=2 timeout -k 10 300 python bench.py --model tabular-mlp-4x1024 > gpurun_out/bench_tab_s2.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tab -o run --output-format csv -- \
  python3 bench.py --model tabular-mlp-4x1024 --rows 2000000 --steps 50 --warmup 5 > gpurun_out/prof_tab.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tt -o run --output-format csv -- \
  python3 bench.py --model tabtransformer --rows 1000000 --steps 50 --warmup 5 > gpurun_out/prof_tt.log 2>&1 || exit $?
