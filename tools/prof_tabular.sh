#!/bin/bash
# rocprofv3 kernel statistics of the tabular (graph engine) bench step.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tab -o run --output-format csv -- \
  python3 bench.py --model tabular-mlp-4x1024 --rows 2000000 --steps 30 --warmup 5 > gpurun_out/prof_tab.log 2>&1
