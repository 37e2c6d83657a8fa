#!/bin/bash
# Round 3: fused peer all-reduce + Adam kernel (csrc/xg_adam.hip) - kernel-level in-process
# rehearsal, timeout path, engine-level W = 2 / 4 processes sharing the GPU; regression of the
# in-kernel exchange and the W = 1 DDP step path.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_xg_adam_gpu.py \
  > $O/pytest_gx.log 2>&1 || { tail -60 $O/pytest_gx.log; exit 1; }
tail -12 $O/pytest_gx.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_xgmi_gpu.py \
  tests/test_trainer_gpu.py -k "xgmi or exchange or barrier or ddp_step_path" > $O/pytest_gx_reg.log 2>&1 \
  || { tail -60 $O/pytest_gx_reg.log; exit 1; }
tail -3 $O/pytest_gx_reg.log
echo done
