#!/bin/bash
# Round 3: full GPU tier, then the one-barrier 3x128 kernel (csrc/mlp_block2.hip): driver-shaped
# bench, long-run A/B against mlp_block.hip (DCT_MLP_BLOCK=v1), per-phase stamps, kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 150 --timeout-method thread > $O/pytest_gpu_r3.log 2>&1
rc=$?
tail -15 $O/pytest_gpu_r3.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc   # 1 = test failures (read the log); anything else: stop
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_s20_a.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_s20_b.log 2>&1 || exit $?
tail -1 $O/bench_s20_a.log
for v in 1 v1 1 v1; do
  DCT_MLP_BLOCK=$v timeout -k 10 300 python bench.py --steps 20000 --warmup 2000 --no-reference-model > $O/bench_long_$v.json 2>&1 || exit $?
  python -c "import json; d=json.loads([l for l in open('$O/bench_long_$v.json') if l.startswith('{')][-1]); print('block=$v %.3f us/step %.0f samples/s loss %s -> %s' % (d['extra']['us_per_step'], d['value'], d['extra']['loss_first'], d['extra']['loss_last']))" >> $O/block_ab.log
done
cat $O/block_ab.log
timeout -k 10 120 python tools/prof_block.py 4000 > $O/prof_block.log 2>&1 || exit $?
cat $O/prof_block.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_3x128 -o run -- python3 bench.py --steps 20000 --warmup 2000 --no-reference-model > $O/rocprof_3x128.log 2>&1 || exit $?
echo done
