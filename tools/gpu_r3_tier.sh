#!/bin/bash
# Round 3 pass at HEAD: full GPU test tier, smoke, the driver's bench command, a long run, rocprofv3
# kernel stats of the headline, hardware counters of the weather kernel.  Every GPU step under its own
# time limit, chained so the first failure ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > $O/pytest_gpu_tier.log 2>&1
rc=$?; tail -4 $O/pytest_gpu_tier.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_tier.log 2>&1 || exit $?
tail -2 $O/smoke_tier.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_tier_s20_$i.log 2>&1 || exit $?
  grep '^{' $O/bench_tier_s20_$i.log | cut -c1-300
done
timeout -k 10 300 python bench.py --steps 20000 --warmup 2000 > $O/bench_tier_long.log 2>&1 || exit $?
grep '^{' $O/bench_tier_long.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_tier_s20 -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 > $O/prof_tier_s20.log 2>&1 || exit $?
rocprofv3 -L > $O/rocprof_counters.txt 2>&1 || true
pmc() {  # pmc <tag> <counters> <bench args...>: only the counters this box lists
  local tag=$1 ctr="" c
  for c in $2; do grep -qw "$c" $O/rocprof_counters.txt && ctr="$ctr $c"; done
  shift 2
  echo "pass $tag:$ctr"
  [ -n "$ctr" ] || return 0
  timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $O/pmc_$tag -o run -- \
    python3 bench.py "$@" > $O/pmc_$tag.log 2>&1
}
W="--steps 4000 --warmup 200 --no-reference-model"
A="SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
V="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
pmc blk_A "$A" $W && pmc blk_V "$V" $W || exit $?
for t in blk_A blk_V; do
  echo "== $t"; python3 tools/pmc_summary.py $O/pmc_$t 20 6 2>&1 | head -10
done > $O/pmc_tier_summary.txt
cat $O/pmc_tier_summary.txt
for m in tabular-mlp-4x1024 tabtransformer; do
  timeout -k 10 300 python bench.py --model $m > $O/bench_tier_$m.log 2>&1 || exit $?
  grep '^{' $O/bench_tier_$m.log | cut -c1-200
done
echo done
