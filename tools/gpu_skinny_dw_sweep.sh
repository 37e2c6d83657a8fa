#!/bin/bash
# Row-split sweep of the skinny head dW kernel (csrc/skinny.hip, K=1024, C=2, B=4096) inside the
# tabular bench: per split count, the kernel's mean time from rocprofv3 --stats and the step time.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for s in ${SPLITS:-16 32 64 128 256}; do
  DCT_SKINNY_DW_SPLITS=$s timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/skdw_$s -o run -- python3 bench.py --model tabular-mlp-4x1024 --rows 1000000 --steps 100 --warmup 10 \
    > gpurun_out/skdw_$s.log 2>&1 || exit $?
  ms=$(grep -o '"ms_per_step": [0-9.]*' gpurun_out/skdw_$s.log)
  k=$(grep -h 'skinny_dw' $(find gpurun_out/skdw_$s -name '*kernel_stats.csv') | awk -F'",' '{print $2}' | cut -d, -f1-3)
  echo "splits=$s $ms skinny_dw(calls,total_ns,avg_ns)=$k"
done
