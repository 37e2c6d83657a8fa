export TMPDIR=/tmp
T="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
B="python bench.py --rows 2000000 --no-epoch --warmup 10"
bash tools/gpu.sh r5_dp3 \
 "python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_xg_block5_gpu.py" \
 "$T --nproc-per-node 2 --master-port 29631 bench.py --gpus 2 --steps 20000 --warmup 2000 --no-epoch" \
 "$T --nproc-per-node 4 --master-port 29632 bench.py --gpus 4 --steps 20000 --warmup 2000 --no-epoch" \
 "$T --nproc-per-node 6 --master-port 29636 bench.py --gpus 6 --steps 20000 --warmup 2000 --no-epoch" \
 "$T --nproc-per-node 8 --master-port 29633 bench.py --gpus 8 --steps 20000 --warmup 2000 --no-epoch" \
 "$T --nproc-per-node 2 --master-port 29634 bench.py --gpus 2 --steps 20 --warmup 5" \
 "DCT_FORCE_DDP=1 DCT_REDUCER_TIMING=1 DCT_REDUCER_STANDIN_US=60 $B --model tabular-mlp-4x1024 --steps 100" \
 "DCT_FORCE_DDP=1 DCT_REDUCER_STANDIN_US=60 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_dp3/prof_tab_standin -o run --output-format csv -- python3 bench.py --rows 2000000 --no-epoch --warmup 10 --model tabular-mlp-4x1024 --steps 20" \
 "DCT_GRAPH=0 $B --model tabtransformer --steps 50" \
 "DCT_GRAPH=0 DCT_FORCE_DDP=1 DCT_REDUCER_STANDIN_US=60 $B --model tabtransformer --steps 50" \
 "DCT_GRAPH=0 DCT_FORCE_DDP=1 DCT_REDUCER_STANDIN_US=60 DCT_REDUCER_INLINE=1 $B --model tabtransformer --steps 50"
