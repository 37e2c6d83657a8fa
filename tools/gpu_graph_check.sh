#!/bin/bash
# GEMM + graph-engine checks and benches (one gpurun call).
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_graph_engine_gpu.py -q -rf -x > gpurun_out/pytest_graph.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_graph.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --model tabular-mlp-4x1024 > gpurun_out/tab100m.log 2>&1 || exit 4
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tab -o run --output-format csv -- \
  python3 bench.py --model tabular-mlp-4x1024 --rows 2000000 --steps 30 --warmup 5 > gpurun_out/prof_tab.log 2>&1
