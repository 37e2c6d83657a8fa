#!/bin/bash
# Round 3: mlp_block5 prologue (early vector index loads, LDS-only barriers) - tests, stamps, benches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 500 python -u -m pytest -q -rf -x --timeout 150 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_trainer_gpu.py tests/test_ddp_reducer_gpu.py -k "fused_train or grad_mode or weight_decay or block_kernel or force or ddp" > $O/pytest_pro.log 2>&1
rc=$?; tail -3 $O/pytest_pro.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python tools/prof_block.py 4000 > $O/prof_b5_pro.log 2>&1 || exit $?
tail -6 $O/prof_b5_pro.log
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_pro_s20_$i.log 2>&1 || exit $?
  grep '^{' $O/bench_pro_s20_$i.log | cut -c1-200
done
timeout -k 10 200 python bench.py --steps 20000 --warmup 2000 --no-reference-model > $O/bench_pro_long.log 2>&1 || exit $?
grep '^{' $O/bench_pro_long.log | cut -c1-200
DCT_FORCE_DDP=1 timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --no-reference-model > $O/bench_pro_ddp.log 2>&1 || exit $?
grep '^{' $O/bench_pro_ddp.log | cut -c1-200
echo done
