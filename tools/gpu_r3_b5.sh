#!/bin/bash
# Round 3: lean weather kernel (mlp_block5.hip) - numerics tests, long-run A/B (block, dZ1 on the MFMA,
# wave priority), per-phase stamps, the driver's bench window.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest -q -rf -x --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "fused_train or block_kernel or grad_mode or dropout or eval" > $O/pytest_b5.log 2>&1
rc=$?; tail -3 $O/pytest_b5.log; [ $rc -eq 0 ] || exit 1
: > $O/b5_ab.log
for cfg in ${B5_CFGS:-5,1,0 5,0,0 5,1,1 5,1,0 5,0,0 5,1,1}; do
  IFS=, read blk dxm prio <<< "$cfg"
  DCT_MLP_BLOCK=$blk DCT_B5_DXM=$dxm DCT_B3_PRIO=$prio timeout -k 10 200 python bench.py --steps 20000 --warmup 2000 --no-reference-model > $O/bench_b5.json 2>&1 || exit $?
  python -c "import json; d=json.loads([l for l in open('$O/bench_b5.json') if l.startswith('{')][-1]); print('block$blk dxm$dxm prio$prio %.3f us/step %.0f samples/s loss %s -> %s' % (d['extra']['us_per_step'], d['value'], d['extra']['loss_first'], d['extra']['loss_last']))" >> $O/b5_ab.log
done
cat $O/b5_ab.log
for dxm in 1 0; do
  DCT_B5_DXM=$dxm timeout -k 10 120 python tools/prof_block.py 4000 > $O/prof_b5_$dxm.log 2>&1 || exit $?
  cat $O/prof_b5_$dxm.log
done
for i in 1 2; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_b5_s20_$i.log 2>&1 || exit $?
  grep '^{' $O/bench_b5_s20_$i.log | cut -c1-200
done
echo done
