#!/bin/bash
# Full GPU tier: tests, smoke, every bench config, kernel-trace profiles.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_weather_s20.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench_weather.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --model weather-mlp-3x128 > gpurun_out/bench_3x128.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --model tabular-mlp-4x1024 > gpurun_out/bench_tab.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --model tabtransformer > gpurun_out/bench_tt.log 2>&1 || exit $?
if [ "${PROF:-1}" = "1" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_weather -o run --output-format csv -- \
  python3 bench.py --steps 2000 --warmup 200 > gpurun_out/prof_weather.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tab -o run --output-format csv -- \
  python3 bench.py --model tabular-mlp-4x1024 --rows 2000000 --steps 50 --warmup 5 > gpurun_out/prof_tab.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tt -o run --output-format csv -- \
  python3 bench.py --model tabtransformer --rows 1000000 --steps 50 --warmup 5 > gpurun_out/prof_tt.log 2>&1 || exit $?
fi
