set -u
mkdir -p gpurun_out
timeout -k 10 300 python tools/prof_fused.py --steps 20000 > gpurun_out/prof_fused.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench_w.log 2>&1 || exit 2
grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_w.log
