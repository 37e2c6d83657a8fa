#!/bin/bash
# TT bench across dW split-K settings (min k-tiles per slice x split workgroup target).
set -o pipefail
mkdir -p gpurun_out
for cfg in "8 256" "8 128" "16 256" "16 128" "32 256" "8 64"; do
  set -- $cfg
  DCT_GEMM_DW_MINK=$1 DCT_GEMM_SPLIT_WG=$2 timeout -k 10 150 python bench.py --model tabtransformer \
    > gpurun_out/dw_sweep_k$1_wg$2.log 2>&1 || exit $?
  echo "mink=$1 wg=$2 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dw_sweep_k$1_wg$2.log)"
done
