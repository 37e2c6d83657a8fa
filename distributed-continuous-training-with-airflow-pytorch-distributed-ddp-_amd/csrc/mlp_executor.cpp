// Native step executor for wide MLPs (the BASELINE "100M x 256, 4-layer MLP-1024h" family):
// one data-parallel training step issued from C++ with no Python and no autograd on the path,
// designed to be captured ONCE into a hipGraph and replayed for every step of an epoch.
//
// Reference step (jobs/train_lightning_ddp.py:66-71,88,136 through Lightning/torch DDP):
//   collate -> forward (Linear/ReLU) -> loss -> autograd backward -> DDP bucket all-reduce -> Adam.
// MI355X step (all on one compute stream, the all-reduce on the reducer's comm stream):
//   gather_batch          HBM-resident bf16 dataset rows idx[cursor*B + r] -> X_b (16-B copies);
//                         the same grid zeroes the flat gradient buffer + loss slot g[P] and its
//                         first thread bumps the device Adam step counter
//   L x gemm_bf16         A_{l+1} = act(A_l W_l^T + b_l): MFMA GEMM, bias+ReLU/GELU epilogue, bf16 out
//   loss_fwd_bwd          CE / MSE + dlogits (scaled 1/rows); the batch-mean loss is accumulated
//                         straight into g[P] (all-reduced with the grads: sync_dist for free)
//                         [ReLU MLPs with a <= 8-class head: head forward, loss, head dW/db and the
//                          layer below's dZ are ONE kernel, skinny_head (csrc/skinny.hip)]
//   for l = L-1 .. 0:     bias_act_bwd (dZ = dA * act', db = colsum) ; dW_l = dZ^T A_l (fp32 straight
//                         into the flat gradient buffer = the DDP bucket views) ; mark params ready
//                         (the reducer launches each full bucket's ncclAvg on its comm stream while
//                         the earlier layers' backward GEMMs keep running) ; dA_l = dZ W_l
//   finalize              compute stream waits for the last bucket
//   adam_flat             fp32 master update + bf16 shadow weights for the next forward's GEMMs;
//                         [no reducer: the 2-8-way split-K slices of up to three layers' dW are
//                          summed here, in slice order, instead of by a reduce pass or fp32
//                          atomics into g]
//                         its first thread writes loss_out[cursor] = reduced loss, cursor += 1
// (the step prologue, gradient zeroing, loss slot and epilogue ride inside the gather, loss and
// Adam kernels instead of a memset node and three single-thread launches)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <vector>

#include "kernels.h"
#include "mlp_executor.h"
#include "mlp_fused.h"
#include "runtime.h"

#ifndef EXEC_DX_NT
#define EXEC_DX_NT 1
#endif

extern "C" {
int dct_gather_batch(const void* X, int row_bytes, const int* Y, const int* idx, const int* cursor, int stride,
                     int B, int n_items, void* xdst, int* ydst, void* stream);
int dct_gather_batch_step(const void* X, int row_bytes, const int* Y, const int* idx, const int* cursor, int stride,
                          int B, int n_items, void* xdst, int* ydst, int* step_counter, float* zero,
                          int64_t zero_n, void* stream);
int dct_gather_batch_step_ranges(const void* X, int row_bytes, const int* Y, const int* idx, const int* cursor,
                                 int stride, int B, int n_items, void* xdst, int* ydst, int* step_counter, float* zero,
                                 int nr, const int64_t* off, const int64_t* cnt, void* stream);
int dct_loss_fwd_bwd_ex(const void* logits, int logits_bf16, const int* labels, void* dlogits, float* loss_sum,
                        float* correct_sum, int M, int C, float grad_scale, int loss_kind, float loss_scale,
                        void* stream);
int dct_adam_flat_step(float* p, const float* g, float* m, float* v, uint16_t* p_bf16, int64_t n, float lr,
                       float b1, float b2, float eps, float wd, int64_t t, float grad_scale, int decoupled,
                       const int* step_counter, int* cursor, const float* loss_slot, float* loss_out, int loss_cap,
                       void* stream);
int dct_zero_f32(float* p, int64_t n, void* stream);
int dct_step_end(int* cursor, const float* slot, float* loss_out, int loss_cap, void* stream);
int dct_adam_flat_step_parts(float* p, const float* g, float* m, float* v, uint16_t* p_bf16, int64_t n, float lr,
                             float b1, float b2, float eps, float wd, float grad_scale, int decoupled,
                             const int* step_counter, int* cursor, const float* loss_slot, float* loss_out,
                             int loss_cap, int nparts, const int64_t* part_off, const int64_t* part_n,
                             const float* const* part, const int* part_splits, void* stream);
}

namespace dct {

static void ck(int e, const char* what) {
  if (e != 0) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString((hipError_t)e));
}

MlpStepExecutor::MlpStepExecutor(const std::vector<int>& dims, int batch, int act, int loss_kind, uintptr_t p,
                                 uintptr_t p_bf16, uintptr_t g, uintptr_t m, uintptr_t v,
                                 const std::vector<uintptr_t>& acts, const std::vector<uintptr_t>& pre,
                                 uintptr_t dz0, uintptr_t dz1, uintptr_t ybuf, uintptr_t stats,
                                 BucketReducer* reducer)
    : dims_(dims), B_(batch), act_(act), loss_kind_(loss_kind), reducer_(reducer) {
  knobs_reload();  // plan time: this executor keeps its own copy of the DCT_* knobs its launches read
  fused_head_knob_ = knobs().fused_head != 0;
  dw_into_adam_knob_ = knobs().dw_into_adam != 0;
  L_ = (int)dims.size() - 1;
  if (L_ < 1) throw std::invalid_argument("MlpStepExecutor: need at least one layer");
  if ((int)acts.size() != L_ + 1) throw std::invalid_argument("MlpStepExecutor: need L+1 activation buffers");
  if (act_ == ACT_GELU && (int)pre.size() != L_ + 1)
    throw std::invalid_argument("MlpStepExecutor: GELU needs L+1 pre-activation buffers");
  if (dims[0] % 8) throw std::invalid_argument("MlpStepExecutor: input width must be a multiple of 8");
  p_ = reinterpret_cast<float*>(p);
  pb_ = reinterpret_cast<uint16_t*>(p_bf16);
  g_ = reinterpret_cast<float*>(g);
  m_ = reinterpret_cast<float*>(m);
  v_ = reinterpret_cast<float*>(v);
  for (auto a : acts) acts_.push_back(reinterpret_cast<uint16_t*>(a));
  for (auto a : pre) pre_.push_back(reinterpret_cast<uint16_t*>(a));
  dz_[0] = reinterpret_cast<uint16_t*>(dz0);
  dz_[1] = reinterpret_cast<uint16_t*>(dz1);
  y_ = reinterpret_cast<int*>(ybuf);
  stats_ = reinterpret_cast<float*>(stats);
  int64_t off = 0;
  for (int l = 0; l < L_; ++l) {
    woff_.push_back(off);
    off += (int64_t)dims[l] * dims[l + 1];
    boff_.push_back(off);
    off += dims[l + 1];
  }
  P_ = off;
  zr_all_cnt_[0] = P_ + 1;
  plan_partials();
  wt_.assign(L_, nullptr);
  wt_ok_.assign(L_, 0);
#if EXEC_DX_NT
  for (int l = 1; l < L_; ++l)
    if (!skinny(l) && dims[l] % 8 == 0 && dims[l + 1] % 8 == 0)
      if (hipMalloc(&wt_[l], (size_t)dims[l] * dims[l + 1] * sizeof(uint16_t)) != hipSuccess) {
        (void)hipGetLastError();
        wt_[l] = nullptr;
      }
#endif
}

void MlpStepExecutor::set_adam(float lr, float b1, float b2, float eps, float wd, int decoupled) {
  lr_ = lr; b1_ = b1; b2_ = b2; eps_ = eps; wd_ = wd; decoupled_ = decoupled;
}

bool MlpStepExecutor::fused_head() const {
  // ReLU hidden layers only (GELU' needs the pre-activation: the unfused GEMM path); a skinny head
  // whose width fits the kernel's register budget; DCT_FUSED_HEAD=0 keeps the four-kernel chain
  const bool off = !fused_head_knob_;
  const int l = L_ - 1;
  return !off && act_ == ACT_RELU && skinny(l) && dct_skinny_head_supported(dims_[l], dims_[L_]);
}

void MlpStepExecutor::forward(int rows, hipStream_t st, int layers, int first) {
  if (layers < 0) layers = L_;
  for (int l = first; l < layers; ++l) {
    const int din = dims_[l], dout = dims_[l + 1];
    const bool last = l == L_ - 1;
    int epi = EPI_BIAS;
    void* aux = nullptr;
    if (!last) {
      if (act_ == ACT_RELU) epi = EPI_BIAS_RELU;
      else if (act_ == ACT_GELU) { epi = EPI_BIAS_GELU; aux = pre_[l + 1]; }
    }
    if (last && skinny(l)) {  // classifier head: a bandwidth kernel, not a 2-of-128-column MFMA tile
      ck(dct_skinny_fwd(acts_[l], pb_ + woff_[l], p_ + boff_[l], acts_[l + 1], rows, din, dout, st), "skinny fwd");
      continue;
    }
    // a hidden layer whose dX runs as a GEMM: the forward also leaves W^T for it (no extra reads)
    wt_ok_[l] = 0;
    if (wt_[l] && dct_gemm_bf16_bt(acts_[l], pb_ + woff_[l], acts_[l + 1], p_ + boff_[l], rows, dout, din, din, din,
                                   dout, epi, /*out_f32*/ 0, aux, wt_[l], dout, st) == 0) {
      wt_ok_[l] = 1;
      continue;
    }
    (void)hipGetLastError();
    ck(dct_gemm_bf16(acts_[l], pb_ + woff_[l], acts_[l + 1], p_ + boff_[l], rows, dout, din, din, din, dout,
                     /*trans_a*/ 0, /*trans_b*/ 1, epi, /*out_f32*/ 0, /*accumulate*/ 0, aux, st),
       "forward gemm");
  }
}

void MlpStepExecutor::step(uintptr_t X, int row_bytes, uintptr_t Y, uintptr_t idx, int n_items, uintptr_t cursor,
                           uintptr_t step_counter, uintptr_t loss_out, int loss_cap, int rows, uintptr_t stream) {
  if (rows < 1 || rows > B_) throw std::invalid_argument("rows must be in [1, batch]");
  if (row_bytes != dims_[0] * 2) throw std::invalid_argument("dataset row width does not match the model input");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int* cur = reinterpret_cast<int*>(cursor);
  int* sc = reinterpret_cast<int*>(step_counter);
  bool part_used[3] = {false, false, false};
  if (reducer_) reducer_->prepare();
  // gradient zeroing: the ranges of g this step accumulates into.  A full batch leaves the weights
  // of the split-K layers handed to Adam (part_) untouched in g, so those ranges are skipped (the
  // tabular step zeroed 13.6 MB per step for 5 k accumulated values); anything else zeroes all of g.
  const bool skip = rows == B_ && nzr_ > 0;
  // a full batch whose first layer is a hidden GEMM layer gathers inside that layer's forward GEMM
  // (labels, step counter and the gradient ranges riding along); anything else, or a shape the fused
  // kernel does not take, runs the gather launch first
  int first = 0;
  if (gather_fuse_ && skip && L_ > 1 && !skinny(0)) {
    GatherFwd ga{};
    ga.idx = reinterpret_cast<const int*>(idx); ga.cursor = cur; ga.stride = B_; ga.n_items = n_items;
    ga.a_out = acts_[0]; ga.Y = reinterpret_cast<const int*>(Y); ga.ydst = y_; ga.step_counter = sc;
    ga.zero = g_; ga.nz = nzr_;
    for (int q = 0; q < nzr_; ++q) { ga.zoff[q] = zr_off_[q]; ga.zcnt[q] = zr_cnt_[q]; }
    const int epi = act_ == ACT_GELU ? EPI_BIAS_GELU : EPI_BIAS_RELU;
    void* aux = act_ == ACT_GELU ? pre_[1] : nullptr;
    wt_ok_[0] = 0;
    if (dct_gemm_bf16_gather_fwd(reinterpret_cast<const uint16_t*>(X), row_bytes / 2, pb_ + woff_[0], acts_[1],
                                 p_ + boff_[0], rows, dims_[1], dims_[0], epi, aux, &ga, st) == 0) {
      first = 1;
      ++gather_fused_steps_;
    } else {
      (void)hipGetLastError();
    }
  }
  if (first == 0)
    ck(dct_gather_batch_step_ranges(reinterpret_cast<const void*>(X), row_bytes, reinterpret_cast<const int*>(Y),
                                    reinterpret_cast<const int*>(idx), cur, B_, rows, n_items, acts_[0], y_, sc, g_,
                                    skip ? nzr_ : 1, skip ? zr_off_ : zr_all_off_, skip ? zr_cnt_ : zr_all_cnt_, st),
       "gather_batch");
  // Adam riding in the dW launches (no reducer, full batch): when layer l's dW is launched every layer
  // above l has finished its backward (dW and dX), so Adam over those layers' range [woff[l+1], hi)
  // runs in extra workgroups of that dW launch (dct_gemm_bf16_dw_partials_adam) instead of all of it
  // in one HBM-bound launch at the end; only [0, woff[1]) is left for the final launch.  Same
  // arithmetic and slice-sum order as the one launch: bit-identical parameters.
  const bool ride = adam_ride_ && !reducer_ && rows == B_;
  int64_t adam_hi = P_;  // [adam_hi, P) already updated by a riding range
  auto adam_range = [&](int64_t lo, int64_t hi) {
    AdamRange r{};
    r.p = p_; r.g = g_; r.m = m_; r.v = v_; r.p_bf16 = pb_; r.n = P_;
    r.lr = lr_; r.b1 = b1_; r.b2 = b2_; r.eps = eps_; r.wd = wd_; r.grad_scale = 1.0f; r.decoupled = decoupled_;
    r.step_counter = sc;
    for (int q = 0; q < nparts_; ++q) {
      if (!part_used[q]) continue;
      const int lq = part_layer_[q];
      r.part_off[r.nparts] = woff_[lq]; r.part_n[r.nparts] = (int64_t)dims_[lq] * dims_[lq + 1];
      r.part[r.nparts] = part_[q]; r.part_splits[r.nparts] = part_splits_[q];
      ++r.nparts;
    }
    r.lo = lo; r.hi = hi;
    return r;
  };
  const int C = dims_[L_];
  int ci = 0;  // dz_[ci] holds dL/d(output of the current layer)
  int top = L_ - 1;  // highest layer the backward loop below still has to run
  if (fused_head()) {
    // classifier head fused (csrc/skinny.hip skinny_head_kernel): logits, loss (into the loss
    // slot g[P]), dlogits, dW/db of the head and the layer below's dZ in one pass over its input
    forward(rows, st, L_ - 1, first);
    const int l = L_ - 1;
    ck(dct_skinny_head(acts_[l], pb_ + woff_[l], p_ + boff_[l], y_, l > 0 ? dz_[1] : nullptr, g_ + woff_[l],
                       g_ + boff_[l], g_ + P_, rows, dims_[l], C, 1.0f / (float)rows, loss_kind_, 1.0f / (float)rows,
                       /*relu_mask*/ 1, st),
       "fused head");
    if (reducer_) {
      reducer_->mark_ready(2 * L_, stream);
      reducer_->mark_ready(2 * l + 1, stream);
      reducer_->mark_ready(2 * l, stream);
    }
    ci = 1;
    top = L_ - 2;
  } else {
    forward(rows, st, -1, first);
    ck(dct_loss_fwd_bwd_ex(acts_[L_], 1, y_, dz_[ci], g_ + P_, nullptr, rows, C, 1.0f / (float)rows, loss_kind_,
                           1.0f / (float)rows, st),
       "loss");
    if (reducer_) reducer_->mark_ready(2 * L_, stream);  // the loss slot rides in the last-layer bucket
  }
  // dz_[ci] = dL/dZ_l (pre-activation gradient of layer l): the loss kernel's dlogits for the
  // head, then each dX GEMM's activation-derivative epilogue (ReLU mask / GELU') for the layer below.
  for (int l = top; l >= 0; --l) {
    const int din = dims_[l], dout = dims_[l + 1];
    const int mask_epi = act_ == ACT_GELU ? EPI_GELU_GRAD : EPI_RELU_MASK;
    const void* mask_aux = act_ == ACT_GELU ? (const void*)(l > 0 ? pre_[l] : nullptr) : (const void*)acts_[l];
    if (skinny(l)) {
      // dW (+ fused db) and dX of a <= 8-output layer as bandwidth kernels
      ck(dct_skinny_dw(dz_[ci], acts_[l], g_ + woff_[l], g_ + boff_[l], rows, din, dout, st), "skinny dW");
      if (reducer_) {
        reducer_->mark_ready(2 * l + 1, stream);
        reducer_->mark_ready(2 * l, stream);
      }
      if (l > 0) {
        if (act_ == ACT_GELU) {  // GELU' needs the pre-activation: generic GEMM path
          ck(dct_gemm_bf16(dz_[ci], pb_ + woff_[l], dz_[ci ^ 1], nullptr, rows, din, dout, dout, din, din, 0, 0,
                           mask_epi, 0, 0, const_cast<void*>(mask_aux), st),
             "dX gemm");
        } else {
          ck(dct_skinny_dx(dz_[ci], pb_ + woff_[l], acts_[l], dz_[ci ^ 1], rows, din, dout, st), "skinny dX");
        }
        ci ^= 1;
      }
      continue;
    }
    // dW = dZ^T A_l (fp32 into the zeroed flat gradient buffer = a DDP bucket view), with the
    // bias gradient db = colsum(dZ) fused into the same GEMM.  Without a reducer, a layer planned
    // for it leaves its split-K slices in part_[r] for the Adam kernel to sum (no reduce pass, no
    // gradient write + re-read); the weight range of g stays zero and is not read.
    const int r = part_slot(l);
    const bool ride_here = ride && r >= 0 && adam_hi > woff_[l + 1];
    AdamRange rr{};
    if (ride_here) rr = adam_range(woff_[l + 1], adam_hi);
    if (r >= 0 && dct_gemm_bf16_dw_partials_adam(dz_[ci], acts_[l], part_[r], g_ + boff_[l], dout, din, rows,
                                                 part_splits_[r], ride_here ? &rr : nullptr, st) == 0) {
      part_used[r] = true;
      if (ride_here) adam_hi = woff_[l + 1];
    } else {
      if (r >= 0) {
        // the slice plan was made for a full batch; a shorter one (the epoch's partial last batch)
        // has too few k-tiles for it - the layer's dW then goes through g like with a reducer
        (void)hipGetLastError();
        ++part_fallbacks_;
        if (skip)  // this step did not zero the layer's weight range (full batch): zero it now
          ck(dct_zero_f32(g_ + woff_[l], (int64_t)din * dout, st), "zero dW range");
      }
      ck(dct_gemm_bf16_ex(dz_[ci], acts_[l], g_ + woff_[l], nullptr, dout, din, rows, dout, din, din,
                          /*trans_a*/ 1, /*trans_b*/ 0, EPI_NONE, /*out_f32*/ 1, /*accumulate*/ 1, nullptr,
                          g_ + boff_[l], st),
         "dW gemm");
    }
    if (reducer_) {
      reducer_->mark_ready(2 * l + 1, stream);
      reducer_->mark_ready(2 * l, stream);
    }
    if (l > 0) {  // dZ_{l-1} = (dZ_l W_l) * act'(.)  in the epilogue
      // NT on the forward's W^T when it wrote one this step (the NN form reads W through transposing
      // LDS loads), otherwise NN on W
      if (wt_ok_[l])
        ck(dct_gemm_bf16(dz_[ci], wt_[l], dz_[ci ^ 1], nullptr, rows, din, dout, dout, dout, din,
                         /*trans_a*/ 0, /*trans_b*/ 1, mask_epi, /*out_f32*/ 0, /*accumulate*/ 0,
                         const_cast<void*>(mask_aux), st),
           "dX gemm");
      else
        ck(dct_gemm_bf16(dz_[ci], pb_ + woff_[l], dz_[ci ^ 1], nullptr, rows, din, dout, dout, din, din,
                         /*trans_a*/ 0, /*trans_b*/ 0, mask_epi, /*out_f32*/ 0, /*accumulate*/ 0,
                         const_cast<void*>(mask_aux), st),
           "dX gemm");
      ci ^= 1;
    }
  }
  if (reducer_) reducer_->finalize(stream);
  if (adam_hi < P_) {  // the rest of Adam ([0, woff[1]) of a ridden step) + the step epilogue
    const AdamRange rr = adam_range(0, adam_hi);
    ck(dct_adam_range(&rr, cur, g_ + P_, reinterpret_cast<float*>(loss_out), loss_cap, st), "adam");
    return;
  }
  int np = 0;
  int64_t poff[3], pn[3];
  const float* pp[3];
  int psp[3];
  for (int q = 0; q < nparts_; ++q) {
    if (!part_used[q]) continue;
    const int l = part_layer_[q];
    poff[np] = woff_[l]; pn[np] = (int64_t)dims_[l] * dims_[l + 1]; pp[np] = part_[q]; psp[np] = part_splits_[q];
    ++np;
  }
  if (np)
    ck(dct_adam_flat_step_parts(p_, g_, m_, v_, pb_, P_, lr_, b1_, b2_, eps_, wd_, 1.0f, decoupled_, sc, cur, g_ + P_,
                                reinterpret_cast<float*>(loss_out), loss_cap, np, poff, pn, pp, psp, st),
       "adam");
  else
    ck(dct_adam_flat_step(p_, g_, m_, v_, pb_, P_, lr_, b1_, b2_, eps_, wd_, 1, 1.0f, decoupled_, sc, cur, g_ + P_,
                          reinterpret_cast<float*>(loss_out), loss_cap, st),
       "adam");
}

int MlpStepExecutor::part_slot(int l) const {
  if (!dw_into_adam_knob_) return -1;  // dW through g and the reduce pass
  for (int q = 0; q < nparts_; ++q)
    if (part_layer_[q] == l) return q;
  return -1;
}

void MlpStepExecutor::plan_partials() {
  // up to three layers whose dW the launcher would split 2..8 ways: their slices go straight to
  // Adam (no reduce pass for 2-4 slices, no fp32 atomics into g for 5-8 - the tabular input
  // layer's 1024 x 256 x 4096 dW, 8 slices on 128 workgroups).  Only without a DDP reducer (it
  // must all-reduce g), and not with DCT_DW_INTO_ADAM=0 (every dW then accumulates into g, which
  // must be zeroed whole each step).
  if (reducer_ || !dw_into_adam_knob_) return;
  for (int l = L_ - 1; l >= 0 && nparts_ < 3; --l) {
    if (skinny(l)) continue;
    const int M = dims_[l + 1], N = dims_[l];
    const int sp = dct_gemm_dw_auto_splits(M, N, B_);
    if (sp < 2 || sp > 8 || (woff_[l] & 3) || (((int64_t)M * N) & 3)) continue;
    float* buf = nullptr;
    if (hipMalloc(&buf, (size_t)sp * M * N * sizeof(float)) != hipSuccess) {
      (void)hipGetLastError();
      return;
    }
    part_[nparts_] = buf; part_layer_[nparts_] = l; part_splits_[nparts_] = sp;
    ++nparts_;
  }
  // zero ranges of a full-batch step: [0, P] minus the weight ranges of the part_ layers
  // (ascending), at most nparts_ + 1 <= 4 pieces; starts stay 16-B aligned (woff / counts % 4 == 0)
  int64_t skip_lo[3], skip_hi[3];
  int ns = 0;
  for (int q = 0; q < nparts_; ++q) {
    const int l = part_layer_[q];
    skip_lo[ns] = woff_[l];
    skip_hi[ns] = woff_[l] + (int64_t)dims_[l] * dims_[l + 1];
    ++ns;
  }
  for (int i = 0; i < ns; ++i)
    for (int j = i + 1; j < ns; ++j)
      if (skip_lo[j] < skip_lo[i]) { std::swap(skip_lo[i], skip_lo[j]); std::swap(skip_hi[i], skip_hi[j]); }
  int64_t pos = 0;
  nzr_ = 0;
  for (int i = 0; i < ns; ++i) {
    if (skip_lo[i] > pos) { zr_off_[nzr_] = pos; zr_cnt_[nzr_] = skip_lo[i] - pos; ++nzr_; }
    pos = skip_hi[i];
  }
  if (P_ + 1 > pos) { zr_off_[nzr_] = pos; zr_cnt_[nzr_] = P_ + 1 - pos; ++nzr_; }
  if (ns == 0) nzr_ = 0;  // nothing skipped: the full-buffer range below
}

MlpStepExecutor::~MlpStepExecutor() {
  for (int q = 0; q < nparts_; ++q) (void)hipFree(part_[q]);
  for (auto* w : wt_)
    if (w) (void)hipFree(w);
}

void MlpStepExecutor::eval_batch(uintptr_t X, int row_bytes, uintptr_t Y, uintptr_t idx, int n_items,
                                 uintptr_t cursor, int rows, uintptr_t stats, uintptr_t stream) {
  if (rows < 1 || rows > B_) throw std::invalid_argument("rows must be in [1, batch]");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int* cur = reinterpret_cast<int*>(cursor);
  ck(dct_gather_batch(reinterpret_cast<const void*>(X), row_bytes, reinterpret_cast<const int*>(Y),
                      reinterpret_cast<const int*>(idx), cur, B_, rows, n_items, acts_[0], y_, st),
     "gather_batch");
  forward(rows, st);
  float* s = reinterpret_cast<float*>(stats);
  ck(dct_loss_fwd_bwd(acts_[L_], 1, y_, nullptr, s, s + 1, rows, dims_[L_], 1.0f, loss_kind_, st), "eval loss");
  ck(dct_step_end(cur, s, nullptr, 0, st), "advance cursor");
}

}  // namespace dct
