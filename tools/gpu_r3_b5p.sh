#!/bin/bash
# Round 3: mlp_block5 wave-priority A/B (DCT_B3_PRIO bits: 1 young static, 4 young boosted over the
# loss / dZ2 / dZ1 chain), stamps of the best setting.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest -q -rf -x --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "fused_train and dims1" > $O/pytest_b5p.log 2>&1
rc=$?; tail -2 $O/pytest_b5p.log; [ $rc -eq 0 ] || exit 1
: > $O/b5p_ab.log
for prio in 0 1 4 5 0 1 4 5; do
  DCT_B3_PRIO=$prio timeout -k 10 200 python bench.py --steps 20000 --warmup 2000 --no-reference-model > $O/bench_b5p.json 2>&1 || exit $?
  python -c "import json; d=json.loads([l for l in open('$O/bench_b5p.json') if l.startswith('{')][-1]); print('prio$prio %.3f us/step %.0f samples/s' % (d['extra']['us_per_step'], d['value']))" >> $O/b5p_ab.log
done
cat $O/b5p_ab.log
for prio in 4 5; do
  DCT_B3_PRIO=$prio timeout -k 10 120 python tools/prof_block.py 4000 > $O/prof_b5p_$prio.log 2>&1 || exit $?
  cat $O/prof_b5p_$prio.log
done
echo done
