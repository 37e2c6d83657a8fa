#!/bin/bash
# 3-layer 128-h weather MLP (mlp_block.hip): numerics (block vs LDS kernel, vs torch Adam) and the
# weather-mlp-3x128 bench, 3 runs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "block or fused_train or grad_mode or dropout or eval" > gpurun_out/pytest_block.log 2>&1 || exit $?
out=gpurun_out/block_ab.log
: > $out
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --model weather-mlp-3x128 > gpurun_out/blk_b.json 2>&1 || exit $?
  python -c "import json; d=json.loads([l for l in open('gpurun_out/blk_b.json') if l.startswith('{')][-1]); print('${TAG:-run} 3x128 %.3f us/step  %.0f samples/s  loss %s -> %s' % (d['extra']['us_per_step'], d['value'], d['extra']['loss_first'], d['extra']['loss_last']))" >> $out
done
