#!/bin/bash
# A/B of the in-kernel all-reduce poll strategies on ONE GPU (ranks share the device; 2 and 4 ranks).
set -u
mkdir -p gpurun_out
timeout -k 10 300 python tools/prof_xg.py --steps 20000 > gpurun_out/prof_xg.log 2>&1 || exit 1
for m in 0 1 2; do
  for w in 2 4; do
    DCT_XG_POLL=$m timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$w \
      --master-addr=127.0.0.1 --master-port=295$m$w bench.py --gpus $w --steps 20000 --warmup 2000 \
      > gpurun_out/dp${w}_poll$m.log 2>&1 || exit 2
  done
done
