#!/bin/bash
# Instruction-mix counter pass over the TabTransformer bench (one rocprofv3 --pmc run, SQ block only)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
C="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"
timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_tt_insts -o run -- \
  python3 bench.py --model tabtransformer --steps 20 --warmup 3 > gpurun_out/pmc_tt_insts.log 2>&1
