#!/bin/bash
# Wide models (BASELINE configs 4 / 5): step time with and without the DDP bucket reducer at W=1
# (DCT_FORCE_DDP=1: one-rank RCCL communicator + BucketReducer, the DDP=8 code path), and
# kernel-trace stats of each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
: > $O/wide_ab.log
for m in tabular-mlp-4x1024 tabtransformer; do
  for f in 0 1 0 1; do
    DCT_FORCE_DDP=$f timeout -k 10 400 python bench.py --model $m > $O/bench_${m}_ddp$f.json 2>&1 || exit $?
    python -c "import json; d=json.loads([l for l in open('$O/bench_${m}_ddp$f.json') if l.startswith('{')][-1]); print('$m force_ddp=$f %.4f ms/step %.0f samples/s engine %s' % (d['ms_per_step'], d['value'], d['config']['engine']))" >> $O/wide_ab.log
  done
done
for w8 in 1 0 1; do
  DCT_GEMM_8W=$w8 timeout -k 10 400 python bench.py --model tabular-mlp-4x1024 > $O/bench_tab_8w$w8.json 2>&1 || exit $?
  python -c "import json; d=json.loads([l for l in open('$O/bench_tab_8w$w8.json') if l.startswith('{')][-1]); print('tabular 8-wave=$w8 %.4f ms/step %.0f samples/s' % (d['ms_per_step'], d['value']))" >> $O/wide_ab.log
done
DCT_GEMM_8W=1 timeout -k 10 300 python -u -m pytest -q -rf --timeout 150 --timeout-method thread tests/test_kernels_gpu.py -k "gemm" > $O/pytest_gemm_8w.log 2>&1
tail -3 $O/pytest_gemm_8w.log
cat $O/wide_ab.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_tab -o run --output-format csv -- \
  python3 bench.py --model tabular-mlp-4x1024 --rows 2000000 --steps 50 --warmup 5 > $O/prof_tab.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_tt -o run --output-format csv -- \
  python3 bench.py --model tabtransformer --rows 1000000 --steps 50 --warmup 5 > $O/prof_tt.log 2>&1 || exit $?
echo done
