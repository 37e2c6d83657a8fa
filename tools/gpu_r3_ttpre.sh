#!/bin/bash
# Round 3: TabTransformer backward recomputes the FFN pre-activation instead of the forward storing it
# (DCT_TT_RECOMPUTE_PRE) - numerics tests, step A/B, kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest -q -rf -x --timeout 150 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_trainer_gpu.py tests/test_ddp_reducer_gpu.py -k "tt or tabtransformer" > $O/pytest_ttpre.log 2>&1
rc=$?; tail -3 $O/pytest_ttpre.log; [ $rc -eq 0 ] || exit 1
: > $O/ttpre_ab.log
for v in 1 0 1 0; do
  DCT_TT_RECOMPUTE_PRE=$v timeout -k 10 400 python bench.py --model tabtransformer > $O/bench_ttpre.json 2>&1 || exit $?
  python -c "import json; d=json.loads([l for l in open('$O/bench_ttpre.json') if l.startswith('{')][-1]); print('recompute_pre=$v %.4f ms/step %.0f samples/s' % (d['ms_per_step'], d['value']))" >> $O/ttpre_ab.log
done
cat $O/ttpre_ab.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_ttpre -o run --output-format csv -- \
  python3 bench.py --model tabtransformer --steps 20 --warmup 3 > $O/prof_ttpre.log 2>&1 || exit $?
python3 tools/kstats.py $O/prof_ttpre/run_kernel_stats.csv 23 12
echo done
