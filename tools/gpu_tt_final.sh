#!/bin/bash
# TabTransformer after the adaptive grouped-dW slice length: tests, then the bench in deferred
# (default) and per-block (DCT_TT_DW_DEFER=0) modes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_tabtransformer.py \
  tests/test_kernels_gpu.py -k "dw_grouped or tt_ or tabtransformer or hip_path or side_stream or device_loop or fit" \
  > gpurun_out/pytest_tt_final.log 2>&1 || exit $?
out=gpurun_out/tt_final_ab.log
: > $out
for f in 1 0 1 0; do
  DCT_TT_DW_DEFER=$f timeout -k 10 300 python bench.py --model tabtransformer > gpurun_out/tf_b.json 2>&1 || exit $?
  python -c "import json; d=json.loads([l for l in open('gpurun_out/tf_b.json') if l.startswith('{')][-1]); print('DCT_TT_DW_DEFER=$f TT %.4f ms/step  %.3fM samples/s  loss %s -> %s' % (d['ms_per_step'], d['value']/1e6, d['extra']['loss_first'], d['extra']['loss_last']))" >> $out
done
