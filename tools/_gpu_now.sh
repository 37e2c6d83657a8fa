set -e
export TMPDIR=/tmp
export STEP_TIMEOUT=900
bash tools/gpu.sh r5_g54 "python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests" "python -c 'import __graft_entry__ as g; g.smoke()'" "python bench.py --steps 20 --warmup 5" "python bench.py --model tabtransformer --no-reference-model" "python bench.py --model tabular-mlp-4x1024 --no-reference-model"
