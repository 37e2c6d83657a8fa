#!/bin/bash
# DDP rehearsal: 2, 4 and 8 ranks sharing ONE GPU (gloo control plane, in-kernel exchange over IPC
# mappings of the same device - no xGMI links involved), long run and driver-shaped window.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in ${WS:-2 4 8}; do
  for s in "20000 2000" "20 5"; do
    set -- $s
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$w --master-addr 127.0.0.1 \
      --master-port $((29600 + w)) bench.py --gpus $w --steps $1 --warmup $2 > gpurun_out/bench_dp${w}_shared_s$1.log 2>&1 || exit $?
  done
done
