set -e
export TMPDIR=/tmp
bash tools/gpu.sh r5_g40 "python tools/probes/skinny_head_atomics_probe.py"
