#!/bin/bash
# Round 3, iteration 2-3 of the 3x128 kernel: 4x4x1 MFMA probe, numerics subset, A/B of the variants
# (block2, block2 + MFMA F2/dW1, mlp_block.hip v1), stamps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 60 ./tools/probes/mfma4x4_probe > $O/mfma4x4_probe.log 2>&1 || exit $?
tail -9 $O/mfma4x4_probe.log
timeout -k 10 700 python -u -m pytest -q -rf --timeout 150 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_ddp_reducer_gpu.py tests/test_graph_engine_gpu.py -k "block or fused or grad_mode or dropout or eval or bound or reducer or dw_slices or phase" \
  > $O/pytest_block2.log 2>&1
rc=$?; tail -8 $O/pytest_block2.log; [ $rc -le 1 ] || exit $rc
: > $O/block_ab2.log
for v in 1 1mf v1 1 1mf v1; do
  mf=0; blk=$v; [ "$v" = "1mf" ] && { mf=1; blk=1; }
  DCT_MLP_BLOCK=$blk DCT_MLP_BLOCK_MF=$mf timeout -k 10 300 python bench.py --steps 20000 --warmup 2000 --no-reference-model > $O/bench_long_$v.json 2>&1 || exit $?
  python -c "import json; d=json.loads([l for l in open('$O/bench_long_$v.json') if l.startswith('{')][-1]); print('block=$v %.3f us/step %.0f samples/s loss %s -> %s' % (d['extra']['us_per_step'], d['value'], d['extra']['loss_first'], d['extra']['loss_last']))" >> $O/block_ab2.log
done
cat $O/block_ab2.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_s20_c.log 2>&1 || exit $?
DCT_MLP_BLOCK_MF=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_s20_mf.log 2>&1 || exit $?
for f in $O/bench_s20_c.log $O/bench_s20_mf.log; do python -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); print('$f', d['value'], d['extra']['us_per_step'], d['extra'].get('reference_model_us_per_step'))"; done
timeout -k 10 120 python tools/prof_block.py 4000 > $O/prof_block2.log 2>&1 || exit $?
DCT_MLP_BLOCK_MF=1 timeout -k 10 120 python tools/prof_block.py 4000 > $O/prof_block2_mf.log 2>&1 || exit $?
cat $O/prof_block2.log $O/prof_block2_mf.log
rocprofv3 -L > $O/rocprof_counters.txt 2>&1 || true
echo done
