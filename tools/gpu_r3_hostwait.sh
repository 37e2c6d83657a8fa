#!/bin/bash
# Round 3: host completion wait in the driver's 20-step window - runtime default (DCT_HOST_SPIN=0)
# vs hipDeviceScheduleSpin (bench default), alternating processes on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out
: > $O/hostwait.log
for i in 1 2 3 4; do
  for sp in 0 1; do
    DCT_HOST_SPIN=$sp timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/hw_$sp.log 2>&1 || exit 1
    python3 -c "import json; d=json.loads([l for l in open('$O/hw_$sp.log') if l.startswith('{')][-1]); print('spin=$sp run $i: 3x128 %.2f us/step (%.0f samples/s), 5-64-2 %.2f us/step' % (d['extra']['us_per_step'], d['value'], d['extra']['reference_model_us_per_step']))" >> $O/hostwait.log
  done
done
cat $O/hostwait.log
