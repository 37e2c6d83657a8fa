set -e
export TMPDIR=/tmp
bash tools/gpu.sh r5_g6 "python tools/debug_ride.py 1024"
