#!/bin/bash
# Cost of the split-K atomics in the grouped dW launch: TT bench with and without the plain-store probe.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 150 python bench.py --model tabtransformer > gpurun_out/dw_probe_atomic.log 2>&1 || exit $?
DCT_GEMM_SPLIT_PROBE=1 timeout -k 10 150 python bench.py --model tabtransformer > gpurun_out/dw_probe_store.log 2>&1 || exit $?
for f in atomic store; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dw_probe_$f.log)"; done
