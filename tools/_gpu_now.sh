set -e
export TMPDIR=/tmp
B="python bench.py --model tabtransformer --steps 600 --warmup 100 --no-reference-model"
bash tools/gpu.sh r5_g53 "$B" "DCT_AB_TWOPASS=64 $B" "$B" "DCT_AB_TWOPASS=64 $B" "$B" "DCT_AB_TWOPASS=64 $B"
