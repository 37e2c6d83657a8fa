#!/bin/bash
# One parametrized GPU-box runner (replaces the per-experiment gpu_*.sh scripts):
#   tools/gpu.sh NAME 'command 1' 'command 2' ...
# Each command runs under its own `timeout -k 10 ${STEP_TIMEOUT:-300}`, its output goes to
# gpurun_out/NAME/stepN.log (merged back by gpurun), the tail is echoed, and the first failing
# step ends the run (no retries, nothing more touches the GPU after a fault / abort / timeout).
set -o pipefail
name=$1
shift
out=gpurun_out/$name
mkdir -p "$out"
export HSA_ENABLE_IPC_MODE_LEGACY=0
i=0
for c in "$@"; do
  i=$((i + 1))
  echo "[$i] $c" | tee -a "$out/steps.log"
  t0=$(date +%s)
  timeout -k 10 "${STEP_TIMEOUT:-300}" bash -c "$c" > "$out/step$i.log" 2>&1
  rc=$?
  tail -n "${TAIL:-8}" "$out/step$i.log"
  echo "[$i] rc=$rc $(( $(date +%s) - t0 ))s" | tee -a "$out/steps.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
