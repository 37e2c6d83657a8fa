set -u
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_tabtransformer.py -q -rf -x -k "attention or hip" > gpurun_out/pytest_attn.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_attn.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --model tabtransformer > gpurun_out/bench_tt.log 2>&1 || { tail -20 gpurun_out/bench_tt.log; exit 4; }
grep "^{" gpurun_out/bench_tt.log | cut -c1-400; grep -o '"extra.*' gpurun_out/bench_tt.log
