#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_tabtransformer.py -m gpu -x -q \
  -k "tt_ or hip_path or hip_fit" --timeout 120 --timeout-method thread > gpurun_out/pytest_tt4.log 2>&1 || exit $?
timeout -k 10 120 python tools/debug/tt_phase_prof.py 512 > gpurun_out/tt_phase.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --model tabtransformer > gpurun_out/bench_tt.log 2>&1 || exit $?
