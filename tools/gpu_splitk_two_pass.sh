#!/bin/bash
# Two-pass split-K (partials + ordered reduce) vs fp32 atomics: numerics, microbench on the dW
# shapes (with larger split targets), tabular and TabTransformer steps A/B/A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "gemm or fused_head or tt_" > gpurun_out/pytest_two_pass.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_graph_engine_gpu.py \
  tests/test_tabtransformer.py >> gpurun_out/pytest_two_pass.log 2>&1 || exit $?
AB_SET=twopass timeout -k 10 300 python tools/bench_gemm_mlp.py --rounds 3 > gpurun_out/gemm_two_pass.log 2>&1 || exit $?
out=gpurun_out/two_pass_ab.log
: > $out
for m in tabular-mlp-4x1024 tabtransformer; do
for f in 1 0 1 0; do
  DCT_GEMM_SPLIT_TWO_PASS=$f timeout -k 10 300 python bench.py --model $m > gpurun_out/tp_b.json 2>&1 || exit $?
  python -c "import json; d=json.loads([l for l in open('gpurun_out/tp_b.json') if l.startswith('{')][-1]); print('DCT_GEMM_SPLIT_TWO_PASS=$f $m %.4f ms/step  %.3fM samples/s  loss %s -> %s' % (d['ms_per_step'], d['value']/1e6, d['extra']['loss_first'], d['extra']['loss_last']))" >> $out
done
done
