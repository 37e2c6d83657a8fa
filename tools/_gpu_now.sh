set -e
export TMPDIR=/tmp
B="python bench.py --model tabtransformer --steps 600 --warmup 100 --no-reference-model"
bash tools/gpu.sh r5_g55 "$B" "DCT_AB_HEAD8=1 $B" "$B" "DCT_AB_HEAD8=1 $B" "$B" "DCT_AB_HEAD8=1 $B"
