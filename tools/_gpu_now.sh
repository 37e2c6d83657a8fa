set -e
export TMPDIR=/tmp
bash tools/gpu.sh r5_g44 "python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'tt_embed_and_head or head_loss'" "python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_tabtransformer.py" "python tools/tt_pooled_head_ab.py native.tt_head_pooled_mode"
