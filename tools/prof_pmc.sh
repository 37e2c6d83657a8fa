#!/bin/bash
# Hardware-counter passes (rocprofv3 --pmc, one counter group per run) over the two bf16 MFMA
# benches: tabular MLP 4x1024 (BASELINE config 4) and TabTransformer (config 5).
#   pass A: MFMA busy cycles, wave cycles, LDS bank conflicts vs LDS activity, GPU-active cycles
#   pass B: FETCH_SIZE (HBM/fabric read bytes; on gfx950 it reports half of a wide streaming read)
# Summarise with: python tools/pmc_summary.py gpurun_out/pmc_<model>_<pass> <steps>
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
A="SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
B="FETCH_SIZE"
run() {  # run <tag> <counters> <bench args...>
  local tag=$1 ctr=$2
  shift 2
  timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d gpurun_out/pmc_$tag -o run -- \
    python3 bench.py "$@" > gpurun_out/pmc_$tag.log 2>&1
}
TAB="--model tabular-mlp-4x1024 --rows 1000000 --steps 20 --warmup 3"
TT="--model tabtransformer --steps 20 --warmup 3"
run tab_A "$A" $TAB && run tab_B "$B" $TAB && run tt_A "$A" $TT && run tt_B "$B" $TT
