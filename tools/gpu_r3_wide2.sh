#!/bin/bash
# VALU probe (with clock warm-up + realtime), 3x128 numerics subset, then the wide-model script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 60 ./tools/probes/valu_probe > $O/valu_probe2.log 2>&1 || exit $?
cat $O/valu_probe2.log
timeout -k 10 300 python -u -m pytest -q -rf --timeout 150 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_graph_engine_gpu.py -k "block or fused or grad_mode or dropout or eval or dw_slices" > $O/pytest_block5.log 2>&1
rc=$?; tail -3 $O/pytest_block5.log; [ $rc -le 1 ] || exit $rc
bash tools/gpu_r3_wide.sh
