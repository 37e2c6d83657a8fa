#!/bin/bash
# CU reservation A/B for the DDP bucket reducer: the step on a stream masked to all
# CUs but N, the collectives (or a payload-sized stand-in) on a stream masked to those N.
#   tools/reserve_ab.sh OUT ROUNDS  - runs the tabular / TabTransformer matrix below, alternating
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAB="--model tabular-mlp-4x1024 --steps 200 --warmup 20 --rows 4000000 --no-reference-model"
TT="--model tabtransformer --steps 200 --warmup 20 --no-reference-model"
run() {  # name env... -- bench args
  local name=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py "$@" > $O/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "fail $name rc=$rc"; tail -20 $O/$name.log; exit 1; fi
  python - "$name" $O/$name.log <<'PY'
import json,sys
for l in open(sys.argv[2]):
    if l.startswith('{'):
        d=json.loads(l); e=d['extra']
        print(f"{sys.argv[1]:34s} {d['ms_per_step']:8.4f} ms/step  {d['config']['engine']}  reserved={e.get('reserved_cus')}")
PY
}
for r in $(seq ${2:-1}); do
  run tab_plain_$r X=1 -- $TAB
  run tab_res8_$r X=1 -- $TAB --reserve-cus 8
  run tab_res8hi_$r X=1 -- $TAB --reserve-cus 8 --reserve-pattern high
  run tab_ddp85_comm_$r DCT_FORCE_DDP=1 DCT_REDUCER_STANDIN_US=85 -- $TAB
  run tab_ddp85_comm_res8_$r DCT_FORCE_DDP=1 DCT_REDUCER_STANDIN_US=85 -- $TAB --reserve-cus 8
  run tab_ddp85_inline_$r DCT_FORCE_DDP=1 DCT_REDUCER_STANDIN_US=85 DCT_REDUCER_INLINE=1 -- $TAB
  run tt_plain_$r X=1 -- $TT
  run tt_res8_$r X=1 -- $TT --reserve-cus 8
  run tt_ddp35_inline_$r DCT_FORCE_DDP=1 DCT_REDUCER_STANDIN_US=35 -- $TT
  run tt_ddp35_branch_$r DCT_FORCE_DDP=1 DCT_REDUCER_STANDIN_US=35 DCT_REDUCER_INLINE=0 -- $TT
  run tt_ddp35_branch_res8_$r DCT_FORCE_DDP=1 DCT_REDUCER_STANDIN_US=35 DCT_REDUCER_INLINE=0 -- $TT --reserve-cus 8
done
