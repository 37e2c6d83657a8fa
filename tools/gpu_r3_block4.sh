#!/bin/bash
# Round 3, iteration 5: L2 prefetch helper workgroups, scalar-cache cursor reads, no scratch; VALU probe
# Numerics subset, long-run A/B (prefetch on / off), the driver's 20-step window, stamps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 60 ./tools/probes/valu_probe > $O/valu_probe.log 2>&1 || exit $?
cat $O/valu_probe.log
timeout -k 10 700 python -u -m pytest -q -rf --timeout 150 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_ddp_reducer_gpu.py tests/test_graph_engine_gpu.py tests/test_trainer_gpu.py \
  -k "block or fused or grad_mode or dropout or eval or bound or reducer or dw_slices or phase or force" \
  > $O/pytest_block4.log 2>&1
rc=$?; tail -8 $O/pytest_block4.log; [ $rc -le 1 ] || exit $rc
: > $O/block_ab4.log
for mf in 1 0 1 0; do
  DCT_B2_PREFETCH=$mf timeout -k 10 300 python bench.py --steps 20000 --warmup 2000 --no-reference-model > $O/bench_long_pf$mf.json 2>&1 || exit $?
  python -c "import json; d=json.loads([l for l in open('$O/bench_long_pf$mf.json') if l.startswith('{')][-1]); print('prefetch=$mf %.3f us/step %.0f samples/s loss %s -> %s' % (d['extra']['us_per_step'], d['value'], d['extra']['loss_first'], d['extra']['loss_last']))" >> $O/block_ab4.log
done
cat $O/block_ab4.log
for i in 1 0 1 0 1; do
  DCT_B2_PREFETCH=$i timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_s20_pf$i.log 2>&1 || exit $?
  python -c "import json; d=json.loads([l for l in open('$O/bench_s20_pf$i.log') if l.startswith('{')][-1]); print('s20 prefetch=$i', d['value'], d['extra']['us_per_step'], d['extra'].get('reference_model_us_per_step'))"
done
timeout -k 10 120 python tools/prof_block.py 4000 > $O/prof_block4.log 2>&1 || exit $?
DCT_B2_PREFETCH=0 timeout -k 10 120 python tools/prof_block.py 4000 > $O/prof_block4_nopf.log 2>&1 || exit $?
cat $O/prof_block4.log $O/prof_block4_nopf.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_s20b -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 > $O/prof_s20b.log 2>&1 || exit $?
echo done
