#!/bin/bash
# kernel/TT iteration: numerics tests, TT bench + profile, tabular bench, GEMM microbench.
set -u
mkdir -p gpurun_out
bash tools/gpu_tt_iter.sh || exit $?
timeout -k 10 600 python bench.py --model tabular-mlp-4x1024 > gpurun_out/bench_tab.log 2>&1 || { tail -5 gpurun_out/bench_tab.log; exit 5; }
grep -o '"ms_per_step": [0-9.]*\|"model_tflops_per_gpu": [0-9.]*' gpurun_out/bench_tab.log
timeout -k 10 300 python tools/bench_gemm.py > gpurun_out/gemm.log 2>&1 || exit 6
cat gpurun_out/gemm.log | tail -12
