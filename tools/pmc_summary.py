"""Per-kernel summary of a rocprofv3 --pmc + --kernel-trace CSV run (tools/prof_pmc.sh).

python tools/pmc_summary.py <run dir> <steps> [top]

Counters are summed over every dispatch of a kernel name and divided by the number of timed +
warmup steps passed in (so the per-step figure is approximate: the bench's warmup and eval
dispatches are counted too). Derived columns:
  mfma%   SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs): busy-cycle share
          of the chip's matrix pipes while the kernel ran. GRBM_GUI_ACTIVE sums the 8 XCDs and
          SQ_VALU_MFMA_BUSY_CYCLES sums all 1024 SIMDs (checked: a 4096x1024x1024 bf16 GEMM
          reads 8.39M busy cycles = 2*M*N*K / 1024 flop per SIMD-cycle). Counter collection
          stretches the active cycles, so this is a lower bound.
  GF/st   dense bf16 MFMA work implied by the busy cycles: busy * 1024 flop, per step (GFLOP)
  TF/s    that work divided by the kernel's time per step in the same run (TFLOP/s; a lower
          bound, counter collection stretches the kernels)
  ldsc%   SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE  (extra cycles lost to bank conflicts)
  GB/s    2 * FETCH_SIZE (KB) / kernel time  (gfx950 FETCH_SIZE counts half of a wide read)
  V/M     SQ_INSTS_VALU / SQ_INSTS_MFMA (instruction-mix pass, tools/pmc_tt_insts.sh)
Kernel time comes from the same run's trace, which counter collection serialises, so it is an
upper bound; use the --stats profiles in profiles/ for timing.
"""
import collections
import csv
import glob
import os
import sys


def _rows(d, suffix):
    out = []
    for p in glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True):
        out.extend(csv.DictReader(open(p)))
    return out


def main():
    d, steps = sys.argv[1], float(sys.argv[2])
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 15
    ctr = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in _rows(d, "counter_collection.csv"):
        ctr[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"])
    dur = collections.defaultdict(float)
    calls = collections.Counter()
    for r in _rows(d, "kernel_trace.csv"):
        dur[r["Kernel_Name"]] += (float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
        calls[r["Kernel_Name"]] += 1
    names = sorted(set(ctr) | set(dur), key=lambda n: -dur.get(n, 0.0))[:top]
    print(f"{'us/step':>9} {'calls':>6} {'mfma%':>6} {'GF/st':>7} {'TF/s':>7} {'ldsc%':>6} {'GB/s':>7} {'V/M':>6}  kernel")
    for n in names:
        c = ctr.get(n, {})
        t_ns = dur.get(n, 0.0)
        mf = c.get("SQ_VALU_MFMA_BUSY_CYCLES")
        ga = c.get("GRBM_GUI_ACTIVE")
        mfma = f"{100 * mf * 8 / (ga * 1024):6.1f}" if mf is not None and ga else "     -"
        gf = f"{mf * 1024 / 1e9 / steps:7.2f}" if mf is not None else "      -"
        tf = f"{mf * 1024 / t_ns / 1e3:7.1f}" if (mf is not None and t_ns) else "      -"
        bc, la = c.get("SQ_LDS_BANK_CONFLICT"), c.get("SQ_LDS_IDX_ACTIVE")
        ldsc = f"{100 * bc / la:6.1f}" if bc is not None and la else "     -"
        fs = c.get("FETCH_SIZE")
        bw = f"{2 * fs * 1024 / t_ns:7.0f}" if fs is not None and t_ns else "      -"
        va, mi = c.get("SQ_INSTS_VALU"), c.get("SQ_INSTS_MFMA")
        vm = f"{va / mi:6.1f}" if va is not None and mi else "     -"
        print(f"{t_ns / 1e3 / steps:9.1f} {calls[n] / steps:6.1f} {mfma} {gf} {tf} {ldsc} {bw} {vm}  {n[:100]}")


if __name__ == "__main__":
    main()
