#!/bin/bash
# TabTransformer deferred grouped dW: k-tiles per split-K slice (DCT_GEMM_DW_MINK; default 8).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/tt_mink_ab.log
: > $out
for mk in ${MKS:-32 64 128 32 64 128}; do
  DCT_GEMM_DW_MINK=$mk timeout -k 10 300 python bench.py --model tabtransformer > gpurun_out/tm_b.json 2>&1 || exit $?
  python -c "import json; d=json.loads([l for l in open('gpurun_out/tm_b.json') if l.startswith('{')][-1]); print('DCT_GEMM_DW_MINK=$mk TT %.4f ms/step  %.3fM samples/s' % (d['ms_per_step'], d['value']/1e6))" >> $out
done
