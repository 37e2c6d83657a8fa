set -e
export TMPDIR=/tmp
B="python bench.py --model tabular-mlp-4x1024 --steps 200 --no-reference-model"
E="DCT_FORCE_DDP=1 DCT_REDUCER_STANDIN_US=60"
bash tools/gpu.sh r5_g41 "$E DCT_AB_SIGREL=1 $B" "$E $B" "$E DCT_AB_SIGREL=1 $B" "$E $B" "$E DCT_AB_SIGREL=1 $B" "$E $B" "python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ddp_reducer_gpu.py"
