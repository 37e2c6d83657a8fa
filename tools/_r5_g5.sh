set -e
export TMPDIR=/tmp
B="python bench.py --rows 2000000 --no-epoch --warmup 10"
bash tools/gpu.sh r5_g5 \
 "python tools/debug_ride.py 1024" \
 "python tools/debug_ride.py 4096" \
 "python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_ddp_reducer_gpu.py" \
 "DCT_FORCE_DDP=1 DCT_REDUCER_STANDIN_US=60 $B --model tabular-mlp-4x1024 --steps 100" \
 "DCT_FORCE_DDP=1 DCT_REDUCER_STANDIN_US=60 DCT_REDUCER_INLINE=1 $B --model tabular-mlp-4x1024 --steps 100" \
 "DCT_FORCE_DDP=1 DCT_REDUCER_STANDIN_US=60 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_g5/prof_tab_standin -o run --output-format csv -- python3 bench.py --rows 2000000 --no-epoch --warmup 10 --model tabular-mlp-4x1024 --steps 20" \
 "DCT_GRAPH=0 python tools/probes/tt_copy_attrib.py"
