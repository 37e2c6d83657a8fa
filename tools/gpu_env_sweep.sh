#!/bin/bash
# HIP/HSA runtime settings vs the launch+sync floor and the driver-shaped weather window:
#   HIP_FORCE_DEV_KERNARG=1  kernel arguments copied into device memory at enqueue (the kernel's
#                            first argument loads do not cross PCIe to host memory)
#   HSA_ENABLE_INTERRUPT=0   completion signals are polled instead of waited on with an interrupt
# Each setting: tools/sync_floor.py, then 3 x `bench.py --steps 20 --warmup 5` (fresh processes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/env_sweep.log
: > $out
for envs in "X=0" "HIP_FORCE_DEV_KERNARG=1" "HSA_ENABLE_INTERRUPT=0" "HIP_FORCE_DEV_KERNARG=1 HSA_ENABLE_INTERRUPT=0"; do
  echo "=== $envs" >> $out
  env $envs timeout -k 10 120 python tools/sync_floor.py >> $out 2>&1 || exit $?
  for i in 1 2 3; do
    env $envs timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/env_b.json 2>&1 || exit $?
    python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/env_b.json') if l.startswith('{')][-1]); print('  bench s20: %.0f samples/s  %.3f us/step' % (d['value'], d['extra']['us_per_step']))" >> $out
  done
  env $envs timeout -k 10 120 python bench.py --steps 20000 --warmup 2000 > gpurun_out/env_b.json 2>&1 || exit $?
  python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/env_b.json') if l.startswith('{')][-1]); print('  bench long: %.0f samples/s  %.3f us/step' % (d['value'], d['extra']['us_per_step']))" >> $out
done
