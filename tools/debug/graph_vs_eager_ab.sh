#!/bin/bash
set -u
for i in 1 2 3; do
  timeout -k 10 200 python tools/debug/graph_vs_eager2.py 2>&1 | grep -v amdgpu.ids || exit 1
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_graph_engine_gpu.py 2>&1 | tail -3
