#!/bin/bash
# Round 3: 16-wave 3x128 kernel (mlp_block4.hip) - numerics subset, long-run A/B against the 8-wave
# mlp_block3 (DCT_MLP_BLOCK=3), the driver's 20-step window, stamps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
DCT_MLP_BLOCK=4 timeout -k 10 300 python -u -m pytest -q -rf -x --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_graph_engine_gpu.py tests/test_trainer_gpu.py -k "block or fused or grad_mode or dropout or eval or dw_slices or force" \
  > $O/pytest_block8.log 2>&1
rc=$?; tail -25 $O/pytest_block8.log; [ $rc -eq 0 ] || exit 1
: > $O/block_ab8.log
for v in 4 3 4 3; do
  blk=$v
  DCT_MLP_BLOCK=$blk timeout -k 10 300 python bench.py --steps 20000 --warmup 2000 --no-reference-model > $O/bench_long_b$v.json 2>&1 || exit $?
  python -c "import json; d=json.loads([l for l in open('$O/bench_long_b$v.json') if l.startswith('{')][-1]); print('block$v %.3f us/step %.0f samples/s loss %s -> %s' % (d['extra']['us_per_step'], d['value'], d['extra']['loss_first'], d['extra']['loss_last']))" >> $O/block_ab8.log
done
cat $O/block_ab8.log
for i in 1 2 3; do
  DCT_MLP_BLOCK=4 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_s20_b4_$i.log 2>&1 || exit $?
  python -c "import json; d=json.loads([l for l in open('$O/bench_s20_b4_$i.log') if l.startswith('{')][-1]); print('s20 block4', d['value'], d['extra']['us_per_step'], d['extra'].get('reference_model_us_per_step'))"
done
DCT_MLP_BLOCK=4 timeout -k 10 120 python tools/prof_block.py 4000 > $O/prof_block8.log 2>&1 || exit $?
cat $O/prof_block8.log
echo done
