#!/bin/bash
# A/B of an env setting on the shared-GPU DDP rehearsal (N ranks of bench.py on ONE GPU, torchrun;
# N = 1 runs bench.py directly):
#   [BENCH_ARGS="--model tabular-mlp-4x1024"] tools/reh_ab.sh OUT "N_LIST" "STEPS WARMUP" "ENV_A" "ENV_B" [ROUNDS]
# prints one line per run: env, N, us/step, engine, replicas in sync
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
read -r K W <<< "$3"
for r in $(seq ${6:-1}); do for n in $2; do for e in "$4" "$5"; do
  tag=$(echo "$e" | tr ' =' '_-')
  if [ $n = 1 ]; then
    env $e timeout -k 10 200 python bench.py --steps $K --warmup $W --no-epoch --no-reference-model $BENCH_ARGS \
      > $O/b_${n}_${tag}_$r.log 2>&1 || { echo "fail n=$n env=$e"; tail -30 $O/b_${n}_${tag}_$r.log; exit 1; }
  else
    env $e timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29500+n)) bench.py --gpus $n --steps $K --warmup $W --no-epoch $BENCH_ARGS \
      > $O/b_${n}_${tag}_$r.log 2>&1 || { echo "fail n=$n env=$e"; tail -30 $O/b_${n}_${tag}_$r.log; exit 1; }
  fi
  python - "$e" $n $O/b_${n}_${tag}_$r.log <<'PY'
import json,sys
for l in open(sys.argv[3]):
    if l.startswith('{'):
        d=json.loads(l); e=d['extra']
        print(f"{sys.argv[1]:24s} N={sys.argv[2]} {d['ms_per_step']*1e3:8.3f} us/step  {d['config']['engine']}  sync={e['params_in_sync']} xg={e['xgmi_exchange_ok']}")
PY
done; done; done
