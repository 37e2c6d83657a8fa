#!/bin/bash
# TabTransformer: every block's dW GEMMs deferred to ONE grouped launch after backward
# (DCT_TT_DW_DEFER=1) vs one grouped launch per block; also with half the split-K workgroup target.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_tabtransformer.py \
  tests/test_kernels_gpu.py::test_gemm_dw_grouped > gpurun_out/pytest_tt_defer.log 2>&1 || exit $?
out=gpurun_out/tt_defer_ab.log
: > $out
for cfg in "1 256" "0 256" "1 128" "0 128" "1 256" "0 256"; do
  set -- $cfg
  DCT_TT_DW_DEFER=$1 DCT_GEMM_SPLIT_WG=$2 timeout -k 10 300 python bench.py --model tabtransformer > gpurun_out/td_b.json 2>&1 || exit $?
  python -c "import json; d=json.loads([l for l in open('gpurun_out/td_b.json') if l.startswith('{')][-1]); print('DCT_TT_DW_DEFER=$1 DCT_GEMM_SPLIT_WG=$2 TT %.4f ms/step  %.3fM samples/s  loss %s -> %s' % (d['ms_per_step'], d['value']/1e6, d['extra']['loss_first'], d['extra']['loss_last']))" >> $out
done
