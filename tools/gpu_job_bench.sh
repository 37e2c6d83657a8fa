#!/bin/bash
# Whole reference training job (ETL'd parquet, 10 epochs, validation, checkpoints, MLflow file
# store) on the MI355X (fused engine) and, for comparison, the same job on the box's CPU
# (autograd engine, the reference's execution model); plus the trainer GPU tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_trainer_gpu.py tests/test_e2e_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_trainer_job.log 2>&1 || exit $?
timeout -k 10 300 python tools/bench_job.py --rows 100000 --epochs 10 > gpurun_out/job_gpu.log 2>&1 || exit $?
timeout -k 10 600 python tools/bench_job.py --rows 100000 --epochs 2 --accelerator cpu > gpurun_out/job_cpu.log 2>&1 || exit $?
