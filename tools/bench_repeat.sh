#!/bin/bash
# 3 back-to-back single-GPU headline benches (run-to-run spread)
set -u
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 300 python bench.py > gpurun_out/b$i.log 2>&1 || exit 1
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/b$i.log
done
