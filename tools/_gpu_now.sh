set -e
export TMPDIR=/tmp
B="python bench.py --model tabtransformer --steps 600 --warmup 100 --no-reference-model"
bash tools/gpu.sh r5_g43 "$B" "DCT_AB_DWCAP=8 $B" "DCT_AB_DWCAP=16 $B" "$B" "DCT_AB_DWCAP=8 $B" "DCT_AB_DWCAP=16 $B"
