#!/bin/bash
# Same-box A/B of two builds of the native extension on the shared-GPU DDP rehearsal:
#   [BENCH_ARGS="--model tabtransformer"] tools/so_ab.sh OUT "N_LIST" "STEPS WARMUP" SO_A SO_B [ROUNDS]
# Each run copies SO_A / SO_B over the in-tree _dct_native*.so (separate processes, alternating),
# then runs bench.py through torchrun (N ranks on ONE GPU; N = 1 runs bench.py directly).
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
read -r K W <<< "$3"
SO=$(ls distributed-continuous-training-with-airflow-pytorch-distributed-ddp-_amd/_dct_native*.so)
cp "$SO" $O/orig.so
for r in $(seq ${6:-1}); do for n in $2; do for v in "$4" "$5"; do
  cp "$v" "$SO"
  tag=$(basename $v .so)
  if [ $n = 1 ]; then
    timeout -k 10 200 python bench.py --steps $K --warmup $W --no-epoch --no-reference-model $BENCH_ARGS > $O/b_${n}_${tag}_$r.log 2>&1
  else
    timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29500+n)) bench.py --gpus $n --steps $K --warmup $W --no-epoch $BENCH_ARGS > $O/b_${n}_${tag}_$r.log 2>&1
  fi
  rc=$?
  if [ $rc -ne 0 ]; then cp $O/orig.so "$SO"; echo "fail n=$n so=$v rc=$rc"; tail -30 $O/b_${n}_${tag}_$r.log; exit 1; fi
  python - "$tag" $n $O/b_${n}_${tag}_$r.log <<'PY'
import json,sys
for l in open(sys.argv[3]):
    if l.startswith('{'):
        d=json.loads(l); e=d['extra']
        print(f"{sys.argv[1]:10s} N={sys.argv[2]} {d['ms_per_step']*1e3:8.3f} us/step  {d['config']['engine']}  sync={e['params_in_sync']} xg={e['xgmi_exchange_ok']}")
PY
done; done; done
cp $O/orig.so "$SO"
