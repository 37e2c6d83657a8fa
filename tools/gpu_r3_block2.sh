#!/bin/bash
# Round 3, iteration 2 of the 3x128 kernel: numerics subset, A/B vs mlp_block.hip, stamps, counters.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest -q -rf --timeout 150 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_ddp_reducer_gpu.py tests/test_graph_engine_gpu.py -k "block or fused or grad_mode or dropout or eval or bound or reducer or dw_slices or phase" \
  > $O/pytest_block2.log 2>&1
rc=$?; tail -6 $O/pytest_block2.log; [ $rc -le 1 ] || exit $rc
: > $O/block_ab2.log
for v in 1 v1 1 v1; do
  DCT_MLP_BLOCK=$v timeout -k 10 300 python bench.py --steps 20000 --warmup 2000 --no-reference-model > $O/bench_long_$v.json 2>&1 || exit $?
  python -c "import json; d=json.loads([l for l in open('$O/bench_long_$v.json') if l.startswith('{')][-1]); print('block=$v %.3f us/step %.0f samples/s loss %s -> %s' % (d['extra']['us_per_step'], d['value'], d['extra']['loss_first'], d['extra']['loss_last']))" >> $O/block_ab2.log
done
cat $O/block_ab2.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_s20_c.log 2>&1 || exit $?
tail -1 $O/bench_s20_c.log | cut -c1-300
timeout -k 10 120 python tools/prof_block.py 4000 > $O/prof_block2.log 2>&1 || exit $?
cat $O/prof_block2.log
rocprofv3 -L > $O/rocprof_counters.txt 2>&1 || true
grep -o "SQ_[A-Z_]*" $O/rocprof_counters.txt | sort -u > $O/sq_counters.txt || true
wc -l $O/sq_counters.txt
echo done
