#!/bin/bash
# Split-K dW slices summed inside Adam (wide-MLP executor without a reducer) vs the reduce pass
# into g: numerics, tabular step A/B/A/B (DCT_DW_INTO_ADAM=1/0), kernel stats of both modes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_graph_engine_gpu.py \
  > gpurun_out/pytest_dw_adam.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "gemm or fused_head or adam" >> gpurun_out/pytest_dw_adam.log 2>&1 || exit $?
out=gpurun_out/dw_adam_ab.log
: > $out
for f in 1 0 1 0; do
  DCT_DW_INTO_ADAM=$f timeout -k 10 300 python bench.py --model tabular-mlp-4x1024 > gpurun_out/da_b.json 2>&1 || exit $?
  python -c "import json; d=json.loads([l for l in open('gpurun_out/da_b.json') if l.startswith('{')][-1]); print('DCT_DW_INTO_ADAM=$f tabular %.4f ms/step  %.3fM samples/s  loss %s -> %s' % (d['ms_per_step'], d['value']/1e6, d['extra']['loss_first'], d['extra']['loss_last']))" >> $out
done
for f in 0 1; do
  DCT_DW_INTO_ADAM=$f timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_da$f -o run --output-format csv -- \
    python3 bench.py --model tabular-mlp-4x1024 --rows 2000000 --steps 50 --warmup 5 > gpurun_out/prof_da$f.log 2>&1 || exit $?
done
