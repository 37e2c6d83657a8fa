#!/bin/bash
# Round 3: mlp_block5 grad-mode batch staging (DCT_B5_STAGE) A/B on the W = 1 DDP step rehearsal
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out
: > $O/stage_ab.log
for i in 1 2 3; do
  for st in 0 1; do
    DCT_B5_STAGE=$st DCT_FORCE_DDP=1 DCT_XG_GRAD=1 timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --no-reference-model > $O/bst.json 2>&1 || exit 1
    python -c "import json; d=json.loads([l for l in open('$O/bst.json') if l.startswith('{')][-1]); print('stage=$st %.2f us/step' % d['extra']['us_per_step'])" >> $O/stage_ab.log
  done
done
cat $O/stage_ab.log
