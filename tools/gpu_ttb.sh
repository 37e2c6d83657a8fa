#!/bin/bash
# Fused TabTransformer block: numerics tests, A/B bench (fused fwd+bwd / fused fwd only / unfused), kernel profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_tabtransformer.py -m gpu -x -v \
  -k "tt_block or hip_path or hip_fit or prenorm or attention" --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_ttb.log 2>&1 || exit $?
DCT_TT_FUSED=0 timeout -k 10 300 python bench.py --model tabtransformer > gpurun_out/bench_tt_unfused.log 2>&1 || exit $?
DCT_TT_FUSED_BWD=0 timeout -k 10 300 python bench.py --model tabtransformer > gpurun_out/bench_tt_fwdonly.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --model tabtransformer > gpurun_out/bench_tt.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tt -o run --output-format csv -- \
  python3 bench.py --model tabtransformer --rows 1000000 --steps 50 --warmup 5 > gpurun_out/prof_tt.log 2>&1 || exit $?
