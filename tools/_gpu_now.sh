set -e
export TMPDIR=/tmp
bash tools/gpu.sh r5_g28 "python tools/probes/ffn_dw_probe.py"
