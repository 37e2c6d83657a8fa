set -e
export TMPDIR=/tmp
B="python bench.py --model tabtransformer --steps 600 --warmup 100 --no-reference-model"
bash tools/gpu.sh r5_g38 "python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'tt_embed_and_head or head_loss'" "DCT_AB_HEADFENCE=1 $B" "$B" "DCT_AB_HEADFENCE=1 $B" "$B" "DCT_AB_HEADFENCE=1 $B" "$B"
