#!/bin/bash
# Round 3: block3 with scaled-moment Adam + wave-priority A/B (DCT_B3_PRIO 0/1/2), stamps, and the
# DDP reducer inline (same-stream) mode A/B on the forced-DDP wide models.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest -q -rf -x --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_graph_engine_gpu.py tests/test_trainer_gpu.py tests/test_ddp_reducer_gpu.py \
  -k "block or fused or grad_mode or dropout or eval or dw_slices or force or reducer" > $O/pytest_block7.log 2>&1
rc=$?; tail -15 $O/pytest_block7.log; [ $rc -eq 0 ] || exit 1
: > $O/block_ab7.log
for v in 0 1 2 0 1 2; do
  DCT_B3_PRIO=$v timeout -k 10 300 python bench.py --steps 20000 --warmup 2000 --no-reference-model > $O/bench_long_p$v.json 2>&1 || exit $?
  python -c "import json; d=json.loads([l for l in open('$O/bench_long_p$v.json') if l.startswith('{')][-1]); print('prio$v %.3f us/step %.0f samples/s loss %s -> %s' % (d['extra']['us_per_step'], d['value'], d['extra']['loss_first'], d['extra']['loss_last']))" >> $O/block_ab7.log
done
cat $O/block_ab7.log
for v in 0 1; do
  DCT_B3_PRIO=$v timeout -k 10 120 python tools/prof_block.py 4000 > $O/prof_block7_p$v.log 2>&1 || exit $?
  cat $O/prof_block7_p$v.log
done
: > $O/reducer_inline_ab.log
for m in tabular-mlp-4x1024 tabtransformer; do
  for inl in 0 1 0 1; do
    DCT_FORCE_DDP=1 DCT_REDUCER_INLINE=$inl timeout -k 10 400 python bench.py --model $m > $O/bench_${m}_inl$inl.json 2>&1 || exit $?
    python -c "import json; d=json.loads([l for l in open('$O/bench_${m}_inl$inl.json') if l.startswith('{')][-1]); print('$m force_ddp=1 inline=$inl %.4f ms/step %.0f samples/s' % (d['ms_per_step'], d['value']))" >> $O/reducer_inline_ab.log
  done
done
cat $O/reducer_inline_ab.log
echo done
