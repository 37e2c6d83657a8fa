set -e
export TMPDIR=/tmp
bash tools/gpu.sh r5_g47 "python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_xgmi_gpu.py tests/test_xg_block5_gpu.py"
