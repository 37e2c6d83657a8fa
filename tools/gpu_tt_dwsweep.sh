#!/bin/bash
# TT step time vs grouped-dW split target / pipeline depth
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for wg in 64 128 256 512; do for st in 2 4; do
  DCT_GEMM_SPLIT_WG=$wg DCT_GEMM_STAGES=$st timeout -k 10 200 python bench.py --model tabtransformer --steps 300 --warmup 30 \
    > gpurun_out/tt_sweep_wg${wg}_s${st}.log 2>&1 || exit $?
done; done
