set -e
export TMPDIR=/tmp
bash tools/gpu.sh r5_g49 "python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'tt_ or grouped'" "python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_tabtransformer.py tests/test_determinism_gpu.py tests/test_ddp_reducer_gpu.py" "python tools/tt_pooled_head_ab.py nn._TT_EMBED_RIDE"
