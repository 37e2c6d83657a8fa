#!/bin/bash
# dX GEMM backward-mask epilogue: aux tile prefetched before the k-loop.  GEMM numerics, the
# tabular microbench shapes and the tabular step (A/B against the previous build is by commit).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "gemm or fused_head" > gpurun_out/pytest_aux.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_graph_engine_gpu.py \
  >> gpurun_out/pytest_aux.log 2>&1 || exit $?
out=gpurun_out/aux_ab.log
: > $out
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --model tabular-mlp-4x1024 > gpurun_out/aux_b.json 2>&1 || exit $?
  python -c "import json; d=json.loads([l for l in open('gpurun_out/aux_b.json') if l.startswith('{')][-1]); print('aux prefetch: tabular %.4f ms/step  %.3fM samples/s' % (d['ms_per_step'], d['value']/1e6))" >> $out
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tab -o run --output-format csv -- \
  python3 bench.py --model tabular-mlp-4x1024 --rows 2000000 --steps 50 --warmup 5 > gpurun_out/prof_tab.log 2>&1 || exit $?
