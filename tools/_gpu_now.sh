set -e
export TMPDIR=/tmp
O=gpurun_out/r5_g35
mkdir -p $O
export STEP_TIMEOUT=900
bash tools/gpu.sh r5_g35 "python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests" "python -c 'import __graft_entry__ as g; g.smoke()'" "python bench.py --steps 20 --warmup 5" "python bench.py --model tabular-mlp-4x1024 --no-reference-model" "python bench.py --model tabtransformer --no-reference-model"
A="SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
C="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"
timeout -s KILL 150 rocprofv3 --pmc $A --kernel-trace --output-format csv -d $O/pmc_tt_A -o run -- python3 bench.py --model tabtransformer --steps 20 --warmup 3 --no-reference-model > $O/pmc_tt_A.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/pmc_tt_C -o run -- python3 bench.py --model tabtransformer --steps 20 --warmup 3 --no-reference-model > $O/pmc_tt_C.log 2>&1
python3 tools/pmc_summary.py $O/pmc_tt_A 23 12 > $O/pmc_tt_A.txt
python3 tools/pmc_summary.py $O/pmc_tt_C 23 12 > $O/pmc_tt_C.txt
rm -rf $O/pmc_tt_A $O/pmc_tt_C
cat $O/pmc_tt_A.txt $O/pmc_tt_C.txt
