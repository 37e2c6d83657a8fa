#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python tools/bench_gemm_mlp.py > gpurun_out/gemm_ab2.log 2>&1 || exit $?
timeout -k 10 300 python tools/bench_gemm.py > gpurun_out/bench_gemm.log 2>&1 || exit $?
