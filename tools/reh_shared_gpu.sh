set -o pipefail
O=gpurun_out/r4_reh; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/b_1_20.log 2>&1 || { tail -30 $O/b_1_20.log; exit 1; }
tail -1 $O/b_1_20.log
for n in 2 4 8; do for k in "20 5" "2000 200" "20000 2000"; do
  set -- $k
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500+n)) bench.py --gpus $n --steps $1 --warmup $2 > $O/b_${n}_$1.log 2>&1 || { echo "fail n=$n k=$1"; tail -30 $O/b_${n}_$1.log; exit 1; }
  python - $O/b_${n}_$1.log <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); e=d['extra']
        print(sys.argv[1].split('/')[-1], json.dumps({k:d[k] for k in ('value','n_gpus','steps','warmup','ms_per_step')}), json.dumps({'engine':d['config']['engine'],'rpd':e.get('ranks_per_device'),'sync':e.get('params_in_sync'),'xg':e.get('xgmi_exchange_ok')}))
PY
done; done
