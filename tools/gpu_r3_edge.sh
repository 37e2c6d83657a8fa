#!/bin/bash
# Round 3: mlp_block5 edge shapes (batch < 4, D0 = 1 / 3 / 8), weight decay, grad mode - numerics.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 500 python -u -m pytest -q -rf --timeout 150 --timeout-method thread tests/test_kernels_gpu.py \
  -k "fused_train or grad_mode or weight_decay or block_kernel" > $O/pytest_edge.log 2>&1
rc=$?; tail -6 $O/pytest_edge.log; exit $rc
