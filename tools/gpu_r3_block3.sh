#!/bin/bash
# Round 3, iteration 4 of the 3x128 kernel: coalesced W1 prologue / epilogue through a swizzled LDS
# staging tile, MFMA variant as the default.  Numerics subset, long-run A/B (MF default vs
# DCT_MLP_BLOCK_MF=0), the driver's 20-step window, stamps, kernel trace of the 20-step bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 700 python -u -m pytest -q -rf --timeout 150 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_ddp_reducer_gpu.py tests/test_graph_engine_gpu.py tests/test_trainer_gpu.py \
  -k "block or fused or grad_mode or dropout or eval or bound or reducer or dw_slices or phase or force" \
  > $O/pytest_block3.log 2>&1
rc=$?; tail -8 $O/pytest_block3.log; [ $rc -le 1 ] || exit $rc
: > $O/block_ab3.log
for mf in 1 0 1 0; do
  DCT_MLP_BLOCK_MF=$mf timeout -k 10 300 python bench.py --steps 20000 --warmup 2000 --no-reference-model > $O/bench_long_mf$mf.json 2>&1 || exit $?
  python -c "import json; d=json.loads([l for l in open('$O/bench_long_mf$mf.json') if l.startswith('{')][-1]); print('mf=$mf %.3f us/step %.0f samples/s loss %s -> %s' % (d['extra']['us_per_step'], d['value'], d['extra']['loss_first'], d['extra']['loss_last']))" >> $O/block_ab3.log
done
cat $O/block_ab3.log
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_s20_$i.log 2>&1 || exit $?
  python -c "import json; d=json.loads([l for l in open('$O/bench_s20_$i.log') if l.startswith('{')][-1]); print('s20 run $i', d['value'], d['extra']['us_per_step'], d['extra'].get('reference_model_us_per_step'))"
done
timeout -k 10 120 python tools/prof_block.py 4000 > $O/prof_block3.log 2>&1 || exit $?
DCT_MLP_BLOCK_MF=0 timeout -k 10 120 python tools/prof_block.py 4000 > $O/prof_block3_nomf.log 2>&1 || exit $?
cat $O/prof_block3.log $O/prof_block3_nomf.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_s20 -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 > $O/prof_s20.log 2>&1 || exit $?
echo done
