#!/bin/bash
# VALU issue probe (loop overhead amortised, 1-16 waves) + kernel traces of the forced-DDP wide models.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 60 ./tools/probes/valu_probe > $O/valu_probe3.log 2>&1 || exit $?
cat $O/valu_probe3.log
DCT_FORCE_DDP=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_tab_ddp -o run --output-format csv -- \
  python3 bench.py --model tabular-mlp-4x1024 --rows 2000000 --steps 50 --warmup 5 > $O/prof_tab_ddp.log 2>&1 || exit $?
DCT_FORCE_DDP=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_tt_ddp -o run --output-format csv -- \
  python3 bench.py --model tabtransformer --rows 1000000 --steps 50 --warmup 5 > $O/prof_tt_ddp.log 2>&1 || exit $?
echo done
