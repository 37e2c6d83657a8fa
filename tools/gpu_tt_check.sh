#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_kernels_gpu.py tests/test_tabtransformer.py tests/test_graph_engine_gpu.py -q -rf -x > gpurun_out/pytest_k.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_k.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --model tabtransformer > gpurun_out/bench_tt.log 2>&1 || { tail -20 gpurun_out/bench_tt.log; exit 4; }
grep -o '"ms_per_step": [0-9.]*\|"val_acc": [0-9.]*' gpurun_out/bench_tt.log
timeout -k 10 600 python bench.py --model tabular-mlp-4x1024 > gpurun_out/bench_tab.log 2>&1 || exit 5
grep -o '"ms_per_step": [0-9.]*\|"model_tflops_per_gpu": [0-9.]*' gpurun_out/bench_tab.log
timeout -k 10 300 python tools/bench_gemm.py > gpurun_out/gemm.log 2>&1 || exit 6
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tt -o run --output-format csv -- \
  python3 bench.py --model tabtransformer --rows 1000000 --steps 10 --warmup 5 > gpurun_out/prof_tt.log 2>&1
