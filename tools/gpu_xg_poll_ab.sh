#!/bin/bash
# In-kernel exchange: plain sweep vs two pipelined sweeps (DCT_XG_POLL = 3 | stagger << 8), on the
# shared-GPU DDP rehearsal (2 / 4 / 8 ranks on one MI355X over IPC), long runs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_xgmi_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_xg_poll.log 2>&1 || exit $?
for w in 2 4 8; do
  for poll in 0 3 2051 4099; do
    DCT_XG_POLL=$poll timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$w \
      --master-addr 127.0.0.1 --master-port $((29700 + w)) bench.py --gpus $w --steps 20000 --warmup 2000 \
      > gpurun_out/xgpoll_w${w}_p${poll}.log 2>&1 || exit $?
  done
done
