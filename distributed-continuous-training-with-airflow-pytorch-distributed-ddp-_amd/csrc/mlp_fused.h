// Host/device-shared descriptors of the fused MLP kernels (see mlp_fused_impl.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "knobs.h"

namespace dct {

constexpr int MLP_MAXL = 4;

// Everything a launch needs about one MLP architecture, computed once on the host
// (dct_mlp_make_shape): LDS layout, per-layer work split of the forward / dX phases and
// the ownership of weight blocks for the dW + Adam phase.
struct MlpShape {
  int L;
  int dims[MLP_MAXL + 1];
  int rows4[MLP_MAXL];  // round4(out_l)
  int cols4[MLP_MAXL];  // round4(in_l)
  int ldw[MLP_MAXL];    // LDS row stride of W_l (floats)
  int w_lds[MLP_MAXL];  // LDS offsets (floats)
  int b_lds[MLP_MAXL];
  int a_lds[MLP_MAXL + 1];  // activations A_l [BMAX][lda_l] for l >= 1; A_L = logits
  int a0_lds[2];            // double-buffered input batch (next batch is written during a step)
  int lab_lds[2];           // double-buffered labels (int)
  int lda[MLP_MAXL + 1];
  int dz_lds[MLP_MAXL];  // dZ_l [BMAX][rows4_l]
  int woff[MLP_MAXL];    // torch flat offsets of W_l / b_l
  int boff[MLP_MAXL];
  // forward split: items = (rows4/4 output groups) << f_ksl k-splits, f_kc float4s per split
  int f_ksl[MLP_MAXL], f_kc[MLP_MAXL], f_items[MLP_MAXL];
  // dX split: items = (cols4/4 column groups) << d_osl o-splits, d_oc o-groups per split
  int d_osl[MLP_MAXL], d_oc[MLP_MAXL], d_items[MLP_MAXL];
  int br;                        // rows per owned weight block: 1 (small models) or 4
  int blk_start[MLP_MAXL + 1];   // prefix count of weight blocks per layer
  int blk_cols[MLP_MAXL];        // column blocks per row (cols4/4)
  int bias_start[MLP_MAXL + 1];  // prefix count of biases
  int nblk;
  int nbias;
  int P;
  int red_lds;  // reduction scratch
  int lds_floats;
  int bmax;
  int nt;        // threads per workgroup
  int maxq;      // weight blocks per thread
  int fuse_loss; // loss computed inside the last forward layer (classes <= 4)
  int supported;
  int mlp_block;  // plan-time copy of DCT_MLP_BLOCK (MlpPlan, bindings.cpp): the launch path reads this, never
                  // the process-wide knob struct
};

struct MlpArgs {
  float* p;  // flat params (torch state_dict order): W0,b0,W1,b1,...
  float* m;  // Adam exp_avg (same layout)
  float* v;  // Adam exp_avg_sq
  float* grad_out;  // GRAD mode: [P] grads + [P] = batch loss
  const float* X;
  int ldx;
  const int* Y;
  const int* idx;
  int n_items;  // indices available to this launch
  int B;        // batch size (<= BMAX)
  int steps;
  int t0;  // Adam steps already taken (bias correction uses t0+s+1)
  float lr, b1, b2, eps, wd;
  float dropout;
  uint32_t seed;
  uint32_t step_base;
  float* loss_out;  // [steps]
  int mode;         // 0 = train (Adam fused), 1 = grad only
  int loss_kind;    // 0 = CE, 1 = MSE vs one-hot
  // eval outputs
  float* eval_acc;   // [2]: sum loss, sum correct (atomic)
  float* logits_out; // optional [n_items][C]
  // optional device step counter (Adam steps taken so far): when set it overrides t0 and
  // step_base, and the kernel advances it by `steps` -> launches are graph-replayable.
  int* step_counter;
  // optional (GRAD mode): device batch cursor into idx. The kernel uses batch *cursor, first
  // stores the previous step's (all-reduced) loss grad_out[P] into loss_out[*cursor - 1], and
  // advances the cursor -> one captured step graph replays over a whole epoch.
  int* cursor;
  // diagnostic only: per-phase cycle sums (s_memtime deltas, thread 0) + [30]/[31] realtime
  // start/end (100 MHz) when non-null; never set in production launches.
  unsigned long long* prof;
  // optional (GRAD mode, single-wave kernel): "update-then-grad". If *pending != 0 the
  // kernel first applies Adam with the (all-reduced) gradients still in grad_out, then
  // computes the new gradients; p/m/v are written back and *pending is set to 1.
  int* pending;
  // optional (single-wave kernel): tagged staging buffer for the next launch's batch,
  // [0] = batch index of the staged data, [64..) = one dword per lane per prefetch slot.
  // A launch whose cursor equals the tag reads its batch from here (one round trip, issued
  // with the parameter loads) instead of the dependent idx -> x gather.
  uint32_t* stage;
  // optional (single-wave kernel, train mode): in-kernel data-parallel gradient averaging
  // across GPUs.  Every rank pushes its step gradients as 8-byte {tag, value} granules
  // straight into each peer's receive buffer (peer-mapped over xGMI via IPC) and sums the
  // peers' granules in rank order, so all ranks apply bit-identical Adam updates with no
  // host round trip, no RCCL launch and no kernel boundary per step.  See mlp_wave_impl.h.
  unsigned long long* xg_recv;              // own receive buffer, [2][W][KX][64] granules
  unsigned long long* const* xg_peers;      // device array [W]: every rank's receive buffer
  int xg_world;                             // 0/1 = off
  int xg_rank;
  unsigned int* xg_status;                  // [0]: 0 ok, else (global step + 1) of a timeout
  long long xg_timeout;                     // spin limit in s_memrealtime ticks (100 MHz)
  int xg_poll;                              // 0 full sweeps, 1 probe-then-sweep, 2 sequential; rows kernel:
                                            // 3 | stagger << 8 = two pipelined sweeps in flight
  // optional (row-parallel kernel): wave 0 adds the s_memrealtime ticks (100 MHz) its exchange
  // took over the launch - the allreduce_ms metric of the fused DDP step
  unsigned long long* xg_ticks;
  // kernel-specific A/B knob (mlp_block3.hip: wave priority split), 0 = the kernel's default
  int tune;
  // launch constants derived on the host (bindings.cpp make_train_args): mlp_block5 reads them from
  // the kernarg segment (scalar registers) instead of deriving them in the kernel, where the compiler
  // re-materialised the divisions / logarithms inside the step loop to save vector registers
  float k_drop_scale;  // 1 / (1 - dropout), or 1 without dropout
  float k_l2b1, k_l2b2;  // log2(b1), log2(b2) (Adam bias corrections as one exp2 each)
  float k_rc1, k_rc2;  // 1 / (1 - b1), 1 / (1 - b2) (scaled-moment Adam)
  float k_sqc2;        // sqrt(1 - b2)
};

constexpr int XG_MAXW = 8;  // ranks of the in-kernel exchange (one node)

hipError_t mlp_launch_train_L2(const MlpShape& sh, const MlpArgs& a, hipStream_t st);
hipError_t mlp_launch_train_L3(const MlpShape& sh, const MlpArgs& a, hipStream_t st);
hipError_t mlp_launch_train_L4(const MlpShape& sh, const MlpArgs& a, hipStream_t st);
// register-resident 8-wave two-barrier trainer for D0 <= 32 -> 128 -> 128 -> C <= 4, train and
// grad mode (mlp_block3.hip): every 3x128 shape mlp_block5 does not take
bool mlp_block3_ok(const MlpShape& sh, const MlpArgs& a);
hipError_t mlp_launch_block3(const MlpShape& sh, const MlpArgs& a, hipStream_t st);
// lean two-barrier trainer for the exact weather shape D0<=8 -> 128 -> 128 -> 2, train mode, the
// one-step grad mode and the in-kernel data-parallel launches (mlp_block5.hip, the default there);
// DCT_MLP_BLOCK=3 selects mlp_block3, DCT_MLP_BLOCK=0 the generic LDS trainer
bool mlp_block5_ok(const MlpShape& sh, const MlpArgs& a);
hipError_t mlp_launch_block5(const MlpShape& sh, const MlpArgs& a, hipStream_t st);
// its shape (D0 <= 8 -> 128 -> 128 -> 2, batch <= 4) and the exchange buffer of its in-kernel
// data-parallel launches at `world` = 2 / 4 / 8 ranks (0: not supported)
bool mlp_block5_shape_ok(const int* dims, int L, int B);
size_t mlp_block5_xg_bytes(int world);
hipError_t mlp_launch_eval_L2(const MlpShape& sh, const MlpArgs& a, int grid, hipStream_t st);
hipError_t mlp_launch_eval_L3(const MlpShape& sh, const MlpArgs& a, int grid, hipStream_t st);
hipError_t mlp_launch_eval_L4(const MlpShape& sh, const MlpArgs& a, int grid, hipStream_t st);

}  // namespace dct

extern "C" {
int dct_mlp_shape_size();
int dct_mlp_make_shape(void* out, const int* dims, int L, int bmax);
int dct_mlp_select(const dct::MlpShape* sh, int* nt, int* maxblk);
int dct_mlp_train(const void* shape, const dct::MlpArgs* a, void* stream);
int dct_mlp_eval(const void* shape, const dct::MlpArgs* a, int grid, void* stream);
int dct_mlp_wave_supported(const int* dims, int L, int B);
int dct_mlp_wave_train(const int* dims, int L, const dct::MlpArgs* a, void* stream);
size_t dct_mlp_xg_slab_granules(const int* dims, int L);
int dct_adam_flat(float* p, const float* g, float* m, float* v, uint16_t* p_bf16, int64_t n, float lr,
                  float b1, float b2, float eps, float wd, int64_t t, float grad_scale, int decoupled,
                  const int* step_counter, void* stream);
int dct_f32_to_bf16(const float* in, uint16_t* out, int64_t n, void* stream);
int dct_zero_f32(float* p, int64_t n, void* stream);
int dct_adam_flat_step(float* p, const float* g, float* m, float* v, uint16_t* p_bf16, int64_t n, float lr,
                       float b1, float b2, float eps, float wd, int64_t t, float grad_scale, int decoupled,
                       const int* step_counter, int* cursor, const float* loss_slot, float* loss_out, int loss_cap,
                       void* stream);
int dct_ag_step_prologue(const void* X, int row_bytes, const int64_t* Y, const int64_t* idx, const int* cursor, int B,
                         int64_t n_items, void* xdst, int64_t* ydst, int* step_counter, float* zero, int64_t zero_n,
                         void* stream);
}
