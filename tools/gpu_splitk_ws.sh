#!/bin/bash
# Split-K workspace fixup: GEMM numerics, graph-engine tests, then tabular bench (workspace vs atomics) + TT bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_property_gpu.py tests/test_graph_engine_gpu.py \
  -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm or graph or fused_mlp" > gpurun_out/pytest_splitk_ws.log 2>&1 || exit $?
DCT_GEMM_SPLIT_WS=1 timeout -k 10 150 python bench.py --model tabular-mlp-4x1024 > gpurun_out/bench_tab_ws.log 2>&1 || exit $?
timeout -k 10 150 python bench.py --model tabular-mlp-4x1024 > gpurun_out/bench_tab_atomic.log 2>&1 || exit $?
DCT_GEMM_SPLIT_WS=1 DCT_GEMM_SPLIT_WG=512 timeout -k 10 150 python bench.py --model tabular-mlp-4x1024 > gpurun_out/bench_tab_ws512.log 2>&1 || exit $?
DCT_GEMM_SPLIT_WS=1 timeout -k 10 150 python bench.py --model tabtransformer > gpurun_out/bench_tt_ws.log 2>&1 || exit $?
for f in ws atomic ws512; do echo "tab $f $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_tab_$f.log)"; done
echo "tt ws $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_tt_ws.log)"
