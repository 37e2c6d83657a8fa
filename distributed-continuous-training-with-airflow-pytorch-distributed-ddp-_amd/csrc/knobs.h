// Process-wide tuning / A-B knobs of the native launchers.  Every DCT_* environment variable the
// C++ side honours is read HERE, into one struct, at plan / bind time (dct_knobs_reload: the
// Python plan constructors call it - FusedMLPKernel, the step executors, the engines), never on a
// launch path: launchers only read the struct.  Defaults are the measured-best settings; the
// knobs exist for A/B runs and debugging (README "Environment knobs").
#pragma once

namespace dct {

struct Knobs {
  // fused MLP trainers (mlp_fused.hip dispatch, bindings.cpp plan)
  int mlp_force_lds = 0;    // DCT_MLP_KERNEL=lds: the LDS/block kernels even where the wave kernel fits
  int mlp_block = -1;       // DCT_MLP_BLOCK: -1 auto, 0 generic LDS trainer, 3 force mlp_block3
  int mlp_block_mf = 1;     // DCT_MLP_BLOCK_MF=0: mlp_block3's VALU layer-1 instead of the 4x4x1 MFMA
  int b3_prio = -1;         // DCT_B3_PRIO: mlp_block3 wave-priority split (-1: the launch's own)
  int mlp_rows = 1;         // DCT_MLP_ROWS=0: no row-parallel 2-layer kernel
  // bf16 GEMM (gemm_bf16.hip)
  int gemm_v1 = 0;          // DCT_GEMM_V1: the v1 register-staged GEMM
  int gemm_split_ws = 0;    // DCT_GEMM_SPLIT_WS: split-K through the tile-counter workspace
  int gemm_two_pass = -1;   // DCT_GEMM_SPLIT_TWO_PASS: -1 auto, 0 never, 1 always
  int gemm_stages = 0;      // DCT_GEMM_STAGES: 0 auto (2), 4 = four LDS stages where they fit
  int gemm_split_wg = 0;    // DCT_GEMM_SPLIT_WG: split-K workgroup target (0: one per CU)
  int gemm_splits = 0;      // DCT_GEMM_SPLITS: fixed split-K slice count (0: auto)
  int gemm_8w = -1;         // DCT_GEMM_8W=0: no 8-wave 128-deep-k tiles for <= 1 tile per CU
  int gemm_split_8w = 1;    // DCT_GEMM_SPLIT_8W=0: 4-wave split-K dW tiles (the 8-wave ones are the default)
  int gemm_bm128 = 0;       // DCT_GEMM_BM128: no half-height tiles
  int gemm_bm64_nk = 4;     // DCT_GEMM_BM64_NK: half-height tiles up to this many k-tiles
  int gemm_no_group = 0;    // DCT_GEMM_NO_GROUP: grouped dW as one launch per problem
  int gemm_dw_mink = 0;     // DCT_GEMM_DW_MINK: k-tiles per grouped dW slice (0: auto from 8)
  // skinny head / dW (skinny.hip), TabTransformer io (tt_io.hip), attention
  int skinny_head_rpw = 0;  // DCT_SKINNY_HEAD_RPW: rows per wave (0: auto)
  int skinny_head_waves = 0;// DCT_SKINNY_HEAD_WAVES: waves per block (0: auto)
  int skinny_dw_splits = 0; // DCT_SKINNY_DW_SPLITS: row splits (0: auto)
  int tt_head_spb = 4;      // DCT_TT_HEAD_SPB: samples per head workgroup (4 or 16)
  int attn_scalar = 0;      // DCT_ATTN_SCALAR: scalar attention instead of the MFMA kernels
  // wide-MLP step executor (mlp_executor.cpp), bucket reducer (runtime.cpp)
  int fused_head = 1;       // DCT_FUSED_HEAD=0: the four-kernel head chain
  int dw_into_adam = 1;     // DCT_DW_INTO_ADAM=0: dW through g and the reduce pass
  int reducer_inline = -2;  // DCT_REDUCER_INLINE: -2 auto (compute stream only for a one-rank communicator without
                            // a stand-in, else the comm stream), 1 compute stream, 0 comm stream, -1 inline under capture
  int reducer_standin_us = 0;   // DCT_REDUCER_STANDIN_US: test-only stand-in collective - a busy kernel of this many us
                                // per step (split over the buckets by size) on the collective's stream
  int reducer_standin_wgs = 16; // DCT_REDUCER_STANDIN_WGS: its workgroups (one wave each, no LDS)
  int rccl_one_rank = 0;    // DCT_RCCL_ONE_RANK=1: call RCCL for one-rank in-place collectives too
};

const Knobs& knobs();
void knobs_reload();

}  // namespace dct
