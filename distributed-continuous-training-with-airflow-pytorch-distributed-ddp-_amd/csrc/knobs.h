// Process-wide tuning / A-B knobs of the native launchers.  Every DCT_* environment variable the
// C++ side honours is read HERE, into one struct, at plan / bind time (dct_knobs_reload: the
// Python plan constructors call it - FusedMLPKernel, the step executors, the engines), never on a
// launch path: launchers only read the struct.  Defaults are the measured-best settings; the
// knobs exist for A/B runs, tests and debugging (README "Environment knobs"); variants that measured
// slower were deleted with their knobs (their A/B logs stay in profiles/).
#pragma once

namespace dct {

struct Knobs {
  // fused MLP trainers (mlp_fused.hip dispatch, bindings.cpp plan)
  int mlp_force_lds = 0;    // DCT_MLP_KERNEL=lds: the LDS/block kernels even where the wave kernel fits
  int mlp_block = -1;       // DCT_MLP_BLOCK: -1 auto, 0 generic LDS trainer, 3 force mlp_block3, 8 mlp_block5's
                            // two-micro-batch kernels at every batch (tests: == the one-micro-batch kernels at B <= 4)
  // wide-MLP step executor (mlp_executor.cpp; copied into each executor at construction)
  int fused_head = 1;       // DCT_FUSED_HEAD=0: the four-kernel head chain
  int dw_into_adam = 1;     // DCT_DW_INTO_ADAM=0: dW through g and the reduce pass
  // bucket reducer (runtime.cpp; copied into each reducer at construction)
  int reducer_inline = -2;  // DCT_REDUCER_INLINE: -2 auto (compute stream for a one-rank communicator without a
                            // stand-in and for real peers - RCCL's packed-fp32 reduce kernels must not share CUs
                            // with LDS-DMA GEMM tiles, runtime.cpp - else the comm stream), 1 compute stream,
                            // 0 comm stream, -1 inline under capture
  int reducer_standin_us = 0;   // DCT_REDUCER_STANDIN_US: test-only stand-in collective - a busy kernel of this many us
                                // per step (split over the buckets by size) on the collective's stream
  int reducer_standin_wgs = 16; // DCT_REDUCER_STANDIN_WGS: its workgroups (one wave each, no LDS)
  int reducer_flag_edges = 1;   // DCT_REDUCER_FLAG_EDGES: eager fork / join edges as device counters (1) or events (0)
  int rccl_one_rank = 0;    // DCT_RCCL_ONE_RANK=1: call RCCL for one-rank in-place collectives too
};

const Knobs& knobs();
void knobs_reload();

}  // namespace dct
