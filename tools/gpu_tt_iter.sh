#!/bin/bash
# TabTransformer block-kernel iteration: numerics tests, phase profile, bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_tabtransformer.py -x -q --timeout 120 --timeout-method thread -k "tt or tabtransformer or TabTransformer" > gpurun_out/pytest_tt.log 2>&1 || exit $?
timeout -k 10 200 python tools/debug/tt_phase_prof.py 512 > gpurun_out/tt_phase.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --model tabtransformer > gpurun_out/bench_tt.log 2>&1 || exit $?
