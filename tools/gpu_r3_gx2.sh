#!/bin/bash
# Round 3: cost of the fused peer all-reduce + Adam step path.  W = 1 (DCT_FORCE_DDP=1): RCCL +
# flat Adam vs the exchange kernel; W = 2 / 4 ranks sharing the GPU (tools/gx_rehearsal.py);
# kernel trace of the W = 1 exchange path.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
: > $O/gx2.log
for g in 0 1 0 1; do
  DCT_FORCE_DDP=1 DCT_XG_GRAD=$g timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --no-reference-model > $O/bench_gx$g.json 2>&1 || exit $?
  python -c "import json; d=json.loads([l for l in open('$O/bench_gx$g.json') if l.startswith('{')][-1]); print('W1 force_ddp xg_grad=$g %.2f us/step mode %s' % (d['extra']['us_per_step'], d['extra'].get('engine')))" >> $O/gx2.log
done
for W in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$W --master-addr=127.0.0.1 \
    --master-port=$((29600 + W)) tools/gx_rehearsal.py 2000 200 >> $O/gx2.log 2> $O/gx_reh_$W.err || { tail -30 $O/gx_reh_$W.err; exit 1; }
done
cat $O/gx2.log
DCT_FORCE_DDP=1 DCT_XG_GRAD=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_gx -o run --output-format csv -- \
  python3 bench.py --steps 200 --warmup 20 --no-reference-model > $O/prof_gx.log 2>&1 || exit $?
python3 tools/kstats.py $O/prof_gx/run_kernel_stats.csv 220 12
echo done
