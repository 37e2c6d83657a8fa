set -e
export TMPDIR=/tmp
bash tools/gpu.sh r5_g24 "python tools/tt_pooled_head_ab.py"
