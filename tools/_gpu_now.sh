set -e
export TMPDIR=/tmp
B="python bench.py --model tabtransformer --steps 600 --warmup 100 --no-reference-model"
bash tools/gpu.sh r5_g30 "python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_tabtransformer.py" "DCT_AB_HEAD4=1 $B" "$B" "DCT_AB_HEAD4=1 $B" "$B"
