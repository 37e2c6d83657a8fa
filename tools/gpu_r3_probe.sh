#!/bin/bash
# 4x4x1 fp32 MFMA probe + hardware counters of the 3x128 step (one counter group per pass)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 60 ./tools/probes/mfma4x4_probe > $O/mfma4x4_probe.log 2>&1 || exit $?
tail -12 $O/mfma4x4_probe.log
B="python3 bench.py --steps 4000 --warmup 200 --no-reference-model"
rocprofv3 -L > $O/rocprof_counters.txt 2>&1 || true
pmc() {  # pmc <tag> <counters>: only the counters this box lists (an unknown name aborts the pass)
  local ok=""
  for c in $2; do grep -qw "$c" $O/rocprof_counters.txt && ok="$ok $c"; done
  echo "pass $1:$ok"
  [ -n "$ok" ] || return 0
  timeout -s KILL 90 rocprofv3 --pmc $ok --kernel-trace --output-format csv -d $O/pmc_$1 -o run -- $B > $O/pmc_$1.log 2>&1
}
pmc blkA "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" || exit $?
pmc blkB "SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" || exit $?
python3 tools/pmc_summary.py $O/pmc_blkA 4200 4 > $O/pmc_blk_summary.txt 2>&1
python3 - <<'PY' >> $O/pmc_blk_summary.txt 2>&1
import csv, glob, collections
for tag in ("blkA", "blkB"):
    tot = collections.defaultdict(float)
    for p in glob.glob(f"gpurun_out/pmc_{tag}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            if "mlp_block2" in r["Kernel_Name"]:
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
    print(tag, {k: f"{v:.4g}" for k, v in sorted(tot.items())})
PY
cat $O/pmc_blk_summary.txt
echo done
