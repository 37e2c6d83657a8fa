#!/bin/bash
# Round 3: mlp_block5 grad mode (the 3x128 DDP step kernel) - numerics tests, forced-DDP (W = 1) step
# A/B against mlp_block3's grad mode, kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 500 python -u -m pytest -q -rf -x --timeout 150 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_trainer_gpu.py tests/test_ddp_reducer_gpu.py tests/test_graph_engine_gpu.py \
  -k "grad_mode or force or fused_train or block_kernel or ddp or cursor" > $O/pytest_b5g.log 2>&1
rc=$?; tail -3 $O/pytest_b5g.log; [ $rc -eq 0 ] || exit 1
: > $O/b5g_ab.log
for blk in 5 3 5 3; do
  DCT_MLP_BLOCK=$blk DCT_FORCE_DDP=1 timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --no-reference-model > $O/bench_b5g.json 2>&1 || exit $?
  python -c "import json; d=json.loads([l for l in open('$O/bench_b5g.json') if l.startswith('{')][-1]); print('block$blk force_ddp %.2f us/step %.0f samples/s loss %s -> %s' % (d['extra']['us_per_step'], d['value'], d['extra']['loss_first'], d['extra']['loss_last']))" >> $O/b5g_ab.log
done
cat $O/b5g_ab.log
DCT_FORCE_DDP=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b5g -o run --output-format csv -- \
  python3 bench.py --steps 200 --warmup 20 --no-reference-model > $O/prof_b5g.log 2>&1 || exit $?
python3 tools/kstats.py $O/prof_b5g/run_kernel_stats.csv 220 8
echo done
