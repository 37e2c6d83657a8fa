#!/bin/bash
# Round 3: 16-wave kernel wave-priority A/B (DCT_B4_PRIO 0/1/2) and MFMA on/off, stamps of the winner.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
: > $O/block_ab9.log
for v in 0 1 2 1; do
  DCT_MLP_BLOCK=4 DCT_B4_PRIO=$v timeout -k 10 300 python bench.py --steps 20000 --warmup 2000 --no-reference-model > $O/bench_long_b4p$v.json 2>&1 || exit $?
  python -c "import json; d=json.loads([l for l in open('$O/bench_long_b4p$v.json') if l.startswith('{')][-1]); print('block4 prio$v %.3f us/step %.0f samples/s loss %s -> %s' % (d['extra']['us_per_step'], d['value'], d['extra']['loss_first'], d['extra']['loss_last']))" >> $O/block_ab9.log
done
DCT_MLP_BLOCK=4 DCT_B4_PRIO=1 DCT_MLP_BLOCK_MF=0 timeout -k 10 300 python bench.py --steps 20000 --warmup 2000 --no-reference-model > $O/bench_long_b4p1v.json 2>&1 || exit $?
python -c "import json; d=json.loads([l for l in open('$O/bench_long_b4p1v.json') if l.startswith('{')][-1]); print('block4 prio1 VALU %.3f us/step %.0f samples/s' % (d['extra']['us_per_step'], d['value']))" >> $O/block_ab9.log
DCT_MLP_BLOCK=3 timeout -k 10 300 python bench.py --steps 20000 --warmup 2000 --no-reference-model > $O/bench_long_b3x.json 2>&1 || exit $?
python -c "import json; d=json.loads([l for l in open('$O/bench_long_b3x.json') if l.startswith('{')][-1]); print('block3 %.3f us/step %.0f samples/s' % (d['extra']['us_per_step'], d['value']))" >> $O/block_ab9.log
cat $O/block_ab9.log
for v in 1 2; do
  DCT_MLP_BLOCK=4 DCT_B4_PRIO=$v timeout -k 10 120 python tools/prof_block.py 4000 > $O/prof_block9_p$v.log 2>&1 || exit $?
  cat $O/prof_block9_p$v.log
done
echo done
