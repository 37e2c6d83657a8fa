#!/bin/bash
# One gpurun session: smoke, GPU tests, benches, rocprofv3 kernel stats.
# Stops at the first step that ends abnormally (fault/abort/timeout); test failures (rc=1) continue.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
STEPS="${STEPS:-smoke pytest bench}"
run() {
  local name=$1 tmo=$2; shift 2
  echo "== $name: $*" | tee -a gpurun_out/summary.txt
  timeout -k 10 "$tmo" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/summary.txt
  tail -3 "gpurun_out/$name.log" | tee -a gpurun_out/summary.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)" | tee -a gpurun_out/summary.txt; exit $rc; fi
}
for s in $STEPS; do
  case $s in
    smoke) run smoke 400 python -c "import __graft_entry__ as g; g.smoke()" ;;
    pytest) run pytest_gpu 1200 python -m pytest tests -m gpu -q -rf ;;
    bench) run bench_weather 300 python bench.py
           run bench_3x128 300 python bench.py --model weather-mlp-3x128 ;;
    xgtest) run pytest_xgmi 600 python -m pytest tests/test_xgmi_gpu.py -q -rf -x ;;
    xgbench2) run bench_dp2_shared 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
                  --master-addr=127.0.0.1 --master-port=29571 bench.py --gpus 2 --steps 20000 --warmup 2000 ;;
    xgbench4) run bench_dp4_shared 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=4 \
                  --master-addr=127.0.0.1 --master-port=29572 bench.py --gpus 4 --steps 20000 --warmup 2000 ;;
    prof) export TMPDIR=/tmp
          run prof_weather 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_weather -o run --output-format csv -- python3 bench.py --steps 5000 --warmup 500 ;;
    *) run "$s" 900 bash -c "$s" ;;
  esac
done
