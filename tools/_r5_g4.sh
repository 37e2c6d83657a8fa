set -e
export TMPDIR=/tmp
T="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
B="python bench.py --rows 2000000 --no-epoch --warmup 10"
bash tools/gpu.sh r5_g4 \
 "python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_graph_engine_gpu.py tests/test_kernels_gpu.py tests/test_tabtransformer.py" \
 "$B --model tabular-mlp-4x1024 --steps 200" \
 "python tools/ride_ab.py" \
 "python tools/probes/gemm_chain.py" \
 "$T --nproc-per-node 2 --master-port 29641 tools/prof_b5x.py 4000" \
 "$T --nproc-per-node 8 --master-port 29642 tools/prof_b5x.py 4000" \
 "rocprofv3 --kernel-trace --stats -d gpurun_out/r5_g4/prof_tab -o run --output-format csv -- python3 bench.py --rows 2000000 --no-epoch --warmup 10 --model tabular-mlp-4x1024 --steps 20"
bash tools/gpu.sh r5_g4b \
 "python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_ddp_reducer_gpu.py" \
 "DCT_FORCE_DDP=1 DCT_REDUCER_STANDIN_US=60 $B --model tabular-mlp-4x1024 --steps 100" \
 "DCT_FORCE_DDP=1 DCT_REDUCER_STANDIN_US=60 DCT_REDUCER_INLINE=1 $B --model tabular-mlp-4x1024 --steps 100" \
 "DCT_FORCE_DDP=1 DCT_REDUCER_STANDIN_US=60 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_g4b/prof_tab_standin -o run --output-format csv -- python3 bench.py --rows 2000000 --no-epoch --warmup 10 --model tabular-mlp-4x1024 --steps 20"
