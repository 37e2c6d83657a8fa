#!/bin/bash
# split-K epilogue A/B (natural vs LDS-restaged atomics) + GEMM numerics + tabular/TT benches
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "gemm" --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gemm.log 2>&1 || exit $?
AB_SET=lds timeout -k 10 300 python tools/bench_gemm_mlp.py --rounds 3 > gpurun_out/gemm_ab_lds.log 2>&1 || exit $?
DCT_GEMM_SPLIT_LDS=0 timeout -k 10 300 python bench.py --model tabular-mlp-4x1024 > gpurun_out/bench_tab_nat.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --model tabular-mlp-4x1024 > gpurun_out/bench_tab.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --model tabtransformer > gpurun_out/bench_tt.log 2>&1 || exit $?
