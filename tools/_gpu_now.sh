set -e
export TMPDIR=/tmp
bash tools/gpu.sh r5_g34 "python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'tt_dw'" "python tools/probes/tt_dw_probe.py"
