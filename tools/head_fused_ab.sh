#!/bin/bash
# Same-box A/B of the TabTransformer classifier head: backward folded into the training forward launch
# (default, ops/nn.py unit_loss_seed) vs the head's forward + backward launches (the engine's
# unit_loss_seed replaced by a null context).  tools/head_fused_ab.sh OUT [ROUNDS]
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
ARGS="--model tabtransformer --rows 1000000 --steps 200 --warmup 20 --no-epoch"
for r in $(seq ${2:-3}); do
  for v in twolaunch fused; do
    if [ $v = fused ]; then
      timeout -k 10 300 python bench.py $ARGS > $O/${v}_$r.log 2>&1 || exit 1
    else
      timeout -k 10 300 python -c "import contextlib, runpy, sys; sys.argv = ['bench.py'] + sys.argv[1:]; import dct_amd.trainer.engines as e; e.unit_loss_seed = contextlib.nullcontext; runpy.run_path('bench.py', run_name='__main__')" $ARGS > $O/${v}_$r.log 2>&1 || exit 1
    fi
    python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(f\"{sys.argv[2]:10s} {d['ms_per_step']*1e3:8.3f} us/step\")" $O/${v}_$r.log $v
  done
done
