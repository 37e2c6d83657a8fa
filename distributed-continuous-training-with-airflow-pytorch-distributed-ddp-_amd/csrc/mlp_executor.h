// Native graph-capturable training step for wide MLPs (see mlp_executor.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

namespace dct {

class BucketReducer;

class MlpStepExecutor {
 public:
  // dims: [d0, d1, ..., dL]; buffers are device pointers owned by the caller:
  //   p/g/m/v fp32 flat (g has P+1 entries: grads + the loss slot), p_bf16 bf16 flat shadow,
  //   acts[l] bf16 [batch][d_l] (acts[0] = gathered input, acts[L] = logits),
  //   pre[l] bf16 [batch][d_l] pre-activations (GELU only), dz0/dz1 bf16 [batch][max d],
  //   ybuf int32 [batch], stats fp32 [2].
  MlpStepExecutor(const std::vector<int>& dims, int batch, int act, int loss_kind, uintptr_t p, uintptr_t p_bf16,
                  uintptr_t g, uintptr_t m, uintptr_t v, const std::vector<uintptr_t>& acts,
                  const std::vector<uintptr_t>& pre, uintptr_t dz0, uintptr_t dz1, uintptr_t ybuf, uintptr_t stats,
                  BucketReducer* reducer);
  void set_adam(float lr, float b1, float b2, float eps, float wd, int decoupled);
  void set_adam_ride(bool on) { adam_ride_ = on; }
  bool adam_ride() const { return adam_ride_; }
  // full-batch steps gather the batch inside the first forward GEMM (dct_gemm_bf16_gather_fwd) instead
  // of a gather launch before it; gather_fused_steps() counts the steps that did
  void set_gather_fuse(bool on) { gather_fuse_ = on; }
  int64_t gather_fused_steps() const { return gather_fused_steps_; }
  // One optimizer step on batch *cursor of idx (rows <= batch); advances *cursor and *step_counter.
  void step(uintptr_t X, int row_bytes, uintptr_t Y, uintptr_t idx, int n_items, uintptr_t cursor,
            uintptr_t step_counter, uintptr_t loss_out, int loss_cap, int rows, uintptr_t stream);
  // Forward + loss/accuracy sums (added into stats[0..1]) on batch *cursor; advances *cursor.
  void eval_batch(uintptr_t X, int row_bytes, uintptr_t Y, uintptr_t idx, int n_items, uintptr_t cursor, int rows,
                  uintptr_t stats, uintptr_t stream);
  int64_t num_params() const { return P_; }
  int part_fallbacks() const { return part_fallbacks_; }
  // layers whose dW goes to Adam as split-K slices (no reducer): their weight range of g stays 0
  int partial_layers() const { return nparts_; }
  ~MlpStepExecutor();
  MlpStepExecutor(const MlpStepExecutor&) = delete;
  MlpStepExecutor& operator=(const MlpStepExecutor&) = delete;

 private:
  bool fused_head_knob_ = true, dw_into_adam_knob_ = true;  // DCT_FUSED_HEAD / DCT_DW_INTO_ADAM at construction
  bool adam_ride_ = true;  // Adam ranges riding in the dW launches (set_adam_ride)
  bool gather_fuse_ = true;  // set_gather_fuse
  int64_t gather_fused_steps_ = 0;
  int nzr_ = 0;                                   // gradient ranges a full-batch step zeroes (plan_partials)
  int64_t zr_off_[4] = {}, zr_cnt_[4] = {};
  int64_t zr_all_off_[1] = {0}, zr_all_cnt_[1] = {0};  // the whole buffer (set in the constructor)
  void forward(int rows, hipStream_t st, int layers = -1, int first = 0);  // layers first .. layers-1 (default all)
  bool fused_head() const;
  void plan_partials();
  int part_slot(int l) const;  // partial-buffer slot of layer l's dW, or -1
  // layers with <= 8 outputs run as bandwidth kernels (csrc/skinny.hip)
  bool skinny(int l) const { return dims_[l + 1] <= 8 && dims_[l] % 8 == 0 && woff_[l] % 8 == 0; }
  std::vector<int> dims_;
  int L_ = 0, B_ = 0, act_ = 1, loss_kind_ = 0;
  float* p_ = nullptr;
  uint16_t* pb_ = nullptr;
  float* g_ = nullptr;
  float* m_ = nullptr;
  float* v_ = nullptr;
  std::vector<uint16_t*> acts_, pre_;
  uint16_t* dz_[2] = {nullptr, nullptr};
  int* y_ = nullptr;
  float* stats_ = nullptr;
  std::vector<int64_t> woff_, boff_;
  int64_t P_ = 0;
  BucketReducer* reducer_ = nullptr;
  float lr_ = 1e-3f, b1_ = 0.9f, b2_ = 0.999f, eps_ = 1e-8f, wd_ = 0.f;
  int decoupled_ = 0;
  // split-K dW slices handed to Adam (plan_partials): device buffers [splits][M][N]
  float* part_[3] = {nullptr, nullptr, nullptr};
  int part_layer_[3] = {-1, -1, -1}, part_splits_[3] = {1, 1, 1};
  int nparts_ = 0;
  int part_fallbacks_ = 0;  // steps whose planned split-K slices went through g instead (short batch)
  // W^T (bf16, [din][dout]) of every hidden layer whose dX is a GEMM, written by that layer's forward
  // GEMM from its LDS B images (dct_gemm_bf16_bt): the dX GEMM then reads it in the forward's NT layout
  std::vector<uint16_t*> wt_;
  std::vector<char> wt_ok_;  // this step's forward wrote wt_[l]
};

}  // namespace dct
