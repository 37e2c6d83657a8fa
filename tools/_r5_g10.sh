set -e
export TMPDIR=/tmp
B="python bench.py --rows 2000000 --no-epoch --warmup 10"
bash tools/gpu.sh r5_g10 \
 "DCT_FORCE_DDP=1 DCT_REDUCER_STANDIN_US=60 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_g10/prof_tab_standin -o run --output-format csv -- python3 bench.py --rows 2000000 --no-epoch --warmup 10 --model tabular-mlp-4x1024 --steps 20" \
 "rocprofv3 --kernel-trace --stats -d gpurun_out/r5_g10/prof_tab -o run --output-format csv -- python3 bench.py --rows 2000000 --no-epoch --warmup 10 --model tabular-mlp-4x1024 --steps 20" \
 "$B --model tabular-mlp-4x1024 --steps 200" \
 "python tools/ride_ab.py" \
 "DCT_FORCE_DDP=1 DCT_REDUCER_STANDIN_US=60 $B --model tabular-mlp-4x1024 --steps 100" \
 "python tools/probes/gemm_chain.py" \
 "DCT_GRAPH=0 python tools/probes/tt_copy_attrib.py" \
 "python bench.py --no-epoch --model tabtransformer --steps 200 --warmup 20"
