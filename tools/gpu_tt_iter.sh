#!/bin/bash
# TabTransformer iteration: kernel + model + e2e tests, bench, kernel-trace profile (one GPU, one process at a time).
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_kernels_gpu.py tests/test_tabtransformer.py tests/test_e2e_gpu.py -q -rf -x \
  > gpurun_out/pytest_tt.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_tt.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --model tabtransformer > gpurun_out/bench_tt.log 2>&1 || { tail -20 gpurun_out/bench_tt.log; exit 4; }
grep -o '"ms_per_step": [0-9.]*\|"val_acc": [0-9.]*\|"value": [0-9.]*' gpurun_out/bench_tt.log
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tt -o run --output-format csv -- \
  python3 bench.py --model tabtransformer --rows 1000000 --steps 10 --warmup 5 > gpurun_out/prof_tt.log 2>&1
