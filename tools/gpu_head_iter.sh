#!/bin/bash
# Tabular classifier head: fused skinny_head kernel numerics + executor parity, head microbench
# (tools/bench_head.py), then the tabular bench with the fused head (default) and the four-kernel
# chain (DCT_FUSED_HEAD=0), A/B/A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  "tests/test_kernels_gpu.py::test_fused_skinny_head_matches_fp32_reference_and_chain" \
  "tests/test_kernels_gpu.py::test_fused_head_executor_step_matches_unfused" \
  tests/test_graph_engine_gpu.py > gpurun_out/pytest_head.log 2>&1 || exit $?
timeout -k 10 120 python tools/bench_head.py > gpurun_out/bench_head.log 2>&1 || exit $?
out=gpurun_out/head_ab.log
: > $out
for f in 1 0 1 0; do
  DCT_FUSED_HEAD=$f timeout -k 10 300 python bench.py --model tabular-mlp-4x1024 > gpurun_out/head_b.json 2>&1 || exit $?
  python -c "import json; d=json.loads([l for l in open('gpurun_out/head_b.json') if l.startswith('{')][-1]); print('DCT_FUSED_HEAD=$f tabular %.3f ms/step  %.2fM samples/s  loss %s -> %s' % (d['ms_per_step'], d['value']/1e6, d['extra']['loss_first'], d['extra']['loss_last']))" >> $out
done
