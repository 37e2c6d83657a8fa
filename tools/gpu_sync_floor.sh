set -u
mkdir -p gpurun_out
timeout -k 10 120 python tools/sync_floor.py > gpurun_out/sync_floor.log 2>&1 &&
timeout -k 10 120 python tools/sync_floor.py --spin >> gpurun_out/sync_floor.log 2>&1 &&
ROC_ACTIVE_WAIT_TIMEOUT=200 timeout -k 10 120 python tools/sync_floor.py >> gpurun_out/sync_floor.log 2>&1
