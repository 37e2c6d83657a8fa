set -e
export TMPDIR=/tmp
B="python bench.py --rows 2000000 --no-epoch --warmup 10 --model tabular-mlp-4x1024 --steps 200"
F="DCT_FORCE_DDP=1"
S="DCT_FORCE_DDP=1 DCT_REDUCER_STANDIN_US=60"
TT="python bench.py --no-epoch --model tabtransformer --steps 200 --warmup 20"
bash tools/gpu.sh r5_g11 \
 "$B" "$F $B" "$S $B" "$S DCT_REDUCER_FLAG_EDGES=0 $B" "$S DCT_REDUCER_INLINE=1 $B" "$S DCT_REDUCER_TIMING=1 $B" \
 "$B" "$F $B" "$S $B" "$S DCT_REDUCER_FLAG_EDGES=0 $B" "$S DCT_REDUCER_INLINE=1 $B" "$S DCT_REDUCER_TIMING=1 $B" \
 "$TT" "$S $TT" "$S DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 $TT" "$S DCT_REDUCER_INLINE=1 $TT" "$F $TT"
