set -u
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_tabtransformer.py -q -rf -x > gpurun_out/pytest_tt.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_tt.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --model tabtransformer > gpurun_out/bench_tt.log 2>&1 || { tail -20 gpurun_out/bench_tt.log; exit 4; }
grep "^{" gpurun_out/bench_tt.log | cut -c1-2000
