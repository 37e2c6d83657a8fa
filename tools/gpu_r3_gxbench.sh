#!/bin/bash
# Round 3: the driver's bench command at N = 2 / 4 as ranks SHARING the one GPU (gloo control plane,
# IPC-mapped exchange buffers): the 3x128 DDP step path with the fused peer all-reduce + Adam kernel
# end to end through bench.py (warmup verify, graph capture, device-barrier bracket, JSON line).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
for N in 2 4; do
  for K in 20 2000; do
    W=$([ $K = 20 ] && echo 5 || echo 200)
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$N --master-addr=127.0.0.1 \
      --master-port=$((29650 + N)) bench.py --gpus $N --steps $K --warmup $W > $O/gxbench_${N}_$K.log 2>&1 \
      || { tail -40 $O/gxbench_${N}_$K.log; exit 1; }
    grep '^{' $O/gxbench_${N}_$K.log | cut -c1-420
    grep -o '"engine": "[^"]*"\|"params_in_sync": [a-z]*\|"xgmi_exchange_ok": [a-z]*\|"ranks_per_device": [0-9.]*' $O/gxbench_${N}_$K.log | tr '\n' ' '; echo
  done
done
echo done
