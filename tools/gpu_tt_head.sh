#!/bin/bash
# TabTransformer head kernels (tt_io.hip): numerics, then the TT bench with 16 vs 4 samples per
# workgroup x dW GEMMs on a side stream or not (two rounds), then a kernel-stat profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_tabtransformer.py "tests/test_kernels_gpu.py::test_tt_embed_and_head_loss_match_fp32_reference" > gpurun_out/pytest_tt_head.log 2>&1 || exit $?
out=gpurun_out/tt_head_ab.log
: > $out
for cfg in "16 1" "4 1" "16 0" "4 0" "16 1" "4 1" "16 0" "4 0"; do
  set -- $cfg
  DCT_TT_HEAD_SPB=$1 DCT_TT_DW_SIDE=$2 timeout -k 10 300 python bench.py --model tabtransformer > gpurun_out/tt_b.json 2>&1 || exit $?
  python -c "import json; d=json.loads([l for l in open('gpurun_out/tt_b.json') if l.startswith('{')][-1]); print('DCT_TT_HEAD_SPB=$1 DCT_TT_DW_SIDE=$2 TT %.4f ms/step  %.3fM samples/s  loss %s -> %s' % (d['ms_per_step'], d['value']/1e6, d['extra']['loss_first'], d['extra']['loss_last']))" >> $out
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tt -o run --output-format csv -- \
  python3 bench.py --model tabtransformer --rows 1000000 --steps 50 --warmup 5 > gpurun_out/prof_tt.log 2>&1 || exit $?
