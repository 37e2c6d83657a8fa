#!/bin/bash
# Round 3: the 3x128 DDP step path at W = 1 (DCT_FORCE_DDP=1: block3 grad kernel per step + one-rank
# RCCL all-reduce + flat Adam, graph-replayed) - per-step cost and its kernel trace; wide models at HEAD.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
: > $O/ddp3.log
for i in 1 2; do
  DCT_FORCE_DDP=1 timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --no-reference-model > $O/bench_ddp3.json 2>&1 || exit $?
  python -c "import json; d=json.loads([l for l in open('$O/bench_ddp3.json') if l.startswith('{')][-1]); print('3x128 force_ddp %.2f us/step %.0f samples/s mode %s' % (d['extra']['us_per_step'], d['value'], d['extra'].get('engine')))" >> $O/ddp3.log
done
cat $O/ddp3.log
DCT_FORCE_DDP=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_ddp3 -o run --output-format csv -- \
  python3 bench.py --steps 200 --warmup 20 --no-reference-model > $O/prof_ddp3.log 2>&1 || exit $?
python3 tools/kstats.py $O/prof_ddp3/run_kernel_stats.csv 220 12
for m in tabular-mlp-4x1024 tabtransformer; do
  timeout -k 10 400 python bench.py --model $m > $O/bench_$m.json 2>&1 || exit $?
  python -c "import json; d=json.loads([l for l in open('$O/bench_$m.json') if l.startswith('{')][-1]); print('$m %.4f ms/step %.0f samples/s' % (d['ms_per_step'], d['value']))"
done
echo done
