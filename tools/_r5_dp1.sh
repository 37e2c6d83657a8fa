export TMPDIR=/tmp
T="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
bash tools/gpu.sh r5_dp1 \
 "$T --nproc-per-node 2 --master-port 29621 tools/prof_b5x.py 4000" \
 "$T --nproc-per-node 4 --master-port 29622 tools/prof_b5x.py 4000" \
 "$T --nproc-per-node 8 --master-port 29623 tools/prof_b5x.py 4000" \
 "python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_ddp_reducer_gpu.py -s" \
 "DCT_FORCE_DDP=1 python bench.py --model tabular-mlp-4x1024 --rows 2000000 --steps 100 --warmup 10 --no-epoch" \
 "DCT_FORCE_DDP=1 DCT_REDUCER_STANDIN_US=60 python bench.py --model tabular-mlp-4x1024 --rows 2000000 --steps 100 --warmup 10 --no-epoch" \
 "DCT_FORCE_DDP=1 DCT_REDUCER_STANDIN_US=60 DCT_REDUCER_INLINE=1 python bench.py --model tabular-mlp-4x1024 --rows 2000000 --steps 100 --warmup 10 --no-epoch" \
 "DCT_FORCE_DDP=1 python bench.py --model tabtransformer --rows 1000000 --steps 50 --warmup 10 --no-epoch" \
 "DCT_FORCE_DDP=1 DCT_REDUCER_STANDIN_US=60 python bench.py --model tabtransformer --rows 1000000 --steps 50 --warmup 10 --no-epoch" \
 "DCT_FORCE_DDP=1 DCT_REDUCER_STANDIN_US=60 DCT_REDUCER_INLINE=1 python bench.py --model tabtransformer --rows 1000000 --steps 50 --warmup 10 --no-epoch"
