#!/bin/bash
# Same-box A/B of the TabTransformer step prologue folded into the first fused block (default) vs the
# ag_step_prologue launch (the model's folds_batch_gather switched off).  tools/gather_fold_ab.sh OUT [ROUNDS]
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
ARGS="--model tabtransformer --rows 1000000 --steps 200 --warmup 20 --no-epoch"
for r in $(seq ${2:-3}); do
  for v in prologue folded; do
    if [ $v = folded ]; then
      timeout -k 10 300 python bench.py $ARGS > $O/${v}_$r.log 2>&1 || exit 1
    else
      timeout -k 10 300 python -c "import runpy, sys; sys.argv = ['bench.py'] + sys.argv[1:]; import dct_amd.models.tabtransformer as t; t.TabTransformer.folds_batch_gather = False; runpy.run_path('bench.py', run_name='__main__')" $ARGS > $O/${v}_$r.log 2>&1 || exit 1
    fi
    python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(f\"{sys.argv[2]:10s} {d['ms_per_step']*1e3:8.3f} us/step\")" $O/${v}_$r.log $v
  done
done
