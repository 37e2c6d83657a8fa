set -e
export TMPDIR=/tmp
bash tools/gpu.sh r5_g52 "python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ddp_reducer_gpu.py tests/test_tabtransformer.py tests/test_multigpu.py tests/test_trainer_gpu.py"
