export TMPDIR=/tmp
T="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
B="python bench.py --rows 2000000 --no-epoch --warmup 10"
bash tools/gpu.sh r5_dp2 \
 "$T --nproc-per-node 2 --master-port 29621 tools/prof_b5x.py 4000" \
 "DCT_XG_ONEHOP=0 $T --nproc-per-node 2 --master-port 29622 tools/prof_b5x.py 4000" \
 "$T --nproc-per-node 4 --master-port 29623 tools/prof_b5x.py 4000" \
 "DCT_XG_ONEHOP=1 $T --nproc-per-node 4 --master-port 29624 tools/prof_b5x.py 4000" \
 "$T --nproc-per-node 8 --master-port 29625 tools/prof_b5x.py 4000" \
 "python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_xg_block5_gpu.py" \
 "DCT_FORCE_DDP=1 $B --model tabular-mlp-4x1024 --steps 100" \
 "DCT_FORCE_DDP=1 DCT_REDUCER_STANDIN_US=60 $B --model tabular-mlp-4x1024 --steps 100" \
 "DCT_FORCE_DDP=1 DCT_REDUCER_STANDIN_US=60 DCT_REDUCER_INLINE=1 $B --model tabular-mlp-4x1024 --steps 100" \
 "$B --model tabtransformer --steps 50" \
 "DCT_FORCE_DDP=1 $B --model tabtransformer --steps 50" \
 "DCT_FORCE_DDP=1 DCT_REDUCER_STANDIN_US=60 $B --model tabtransformer --steps 50" \
 "DCT_FORCE_DDP=1 DCT_REDUCER_STANDIN_US=60 DCT_REDUCER_INLINE=1 $B --model tabtransformer --steps 50"
