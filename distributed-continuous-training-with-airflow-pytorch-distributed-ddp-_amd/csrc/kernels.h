// C API of the general NN kernels (GEMM, loss, norm, attention, gather).
#pragma once
#include <stdint.h>
#include "knobs.h"

namespace dct {

// EPI_RELU_MASK: z = aux[o] > 0 ? z : 0 with aux the layer's bf16 ReLU OUTPUT (backward dX GEMM
// producing the previous layer's dZ directly); EPI_GELU_GRAD: z *= gelu'(aux[o]), aux = the
// bf16 pre-activation.
enum Epilogue { EPI_NONE = 0, EPI_BIAS = 1, EPI_BIAS_RELU = 2, EPI_BIAS_GELU = 3, EPI_RELU_MASK = 4, EPI_GELU_GRAD = 5 };
enum Act { ACT_NONE = 0, ACT_RELU = 1, ACT_GELU = 2 };

struct GemmArgs {
  const uint16_t* A;
  const uint16_t* B;
  void* C;
  const float* bias;
  void* aux;
  int M, N, K, lda, ldb, ldc;
  int epilogue, out_f32, accumulate;
  int vec_a, vec_b;
  float alpha;
  float* colsum;  // optional: colsum[m] += sum_k op(A)[m][k] (the bias gradient of a dW GEMM)
  const float* residual;  // optional (fp32 out): C = residual + op(A) op(B) + bias, ld = ldc
  float* split_part;      // optional two-pass split-K: slice s plain-stores its partial C into
                          // split_part[s][M][N]; splitk_reduce_kernel sums the slices into C afterwards
  uint16_t* bt_out;       // optional (NT, no split-K): op(B)^T = B^T [K][N] (row stride bt_ld) written from
  int bt_ld;              // the LDS B images as they stream by - the wide MLP's forward leaves W^T for dX
};

// The wide-MLP step's batch gather folded into its first forward GEMM (dct_gemm_bf16_gather_fwd): A row
// m is dataset row idx[wrap(*cursor * stride + m)] (wrapping inside [0, n_items)), loaded straight
// into the LDS A images; the gathered rows are written once to a_out [M][K] (the dW GEMM's operand),
// and the rest of the step prologue rides along: labels ydst[m] = Y[row], *step_counter += 1, and
// up to 4 ranges [zoff, zoff + zcnt) of `zero` cleared (zoff % 4 == 0).
struct GatherFwd {
  const int* idx;
  const int* cursor;
  int stride, n_items;
  uint16_t* a_out;
  const int* Y;
  int* ydst;
  int* step_counter;
  float* zero;
  int nz;
  int64_t zoff[4], zcnt[4];
};

// An Adam range of the flat buffers, launched on its own or riding in another launch (the wide-MLP
// executor: each layer's Adam in the next lower layer's dW launch, csrc/mlp_executor.cpp).  Fields as
// AdamArgs (adam_impl.h); elements [lo, hi), lo % 4 == 0, hi % 4 == 0 or hi == n.
struct AdamRange {
  float* p;
  const float* g;
  float* m;
  float* v;
  uint16_t* p_bf16;
  int64_t n;
  float lr, b1, b2, eps, wd, grad_scale;
  int decoupled;
  const int* step_counter;
  int nparts;
  int64_t part_off[3], part_n[3];
  const float* part[3];
  int part_splits[3];
  int64_t lo, hi;
};

}  // namespace dct

extern "C" {
// dW = dZ^T X as split-K partials (dct_gemm_bf16_dw_partials) with Adam over r's range in extra
// workgroups of the same launch, co-resident with the GEMM tiles (r == nullptr: the GEMM alone)
int dct_gemm_bf16_dw_partials_adam(const uint16_t* dZ, const uint16_t* X, float* part, float* colsum, int M, int N,
                                   int K, int splits, const dct::AdamRange* r, void* stream);
// the same with the Adam body picked: f4 = 0 one element per thread (the executor's), 1 float4
int dct_gemm_bf16_dw_partials_adam_ex(const uint16_t* dZ, const uint16_t* X, float* part, float* colsum, int M, int N,
                                      int K, int splits, const dct::AdamRange* r, int f4, void* stream);
// Adam over r's range as its own launch (+ the step epilogue: loss_out[*cursor] = *loss_slot, cursor += 1)
int dct_adam_range(const dct::AdamRange* r, int* cursor, const float* loss_slot, float* loss_out, int loss_cap,
                   void* stream);
// reducer instrumentation (step_kernels.hip)
int dct_reducer_stamp(unsigned long long* dst, void* stream);
int dct_busy_spin(long long ticks, int wgs, void* stream);
int dct_flag_signal(int* flag, void* stream);
int dct_flag_wait(int* flag, int* consumed, int* status, void* stream);
int dct_reducer_close(unsigned long long* s, void* stream);
int dct_reducer_check(unsigned long long* s, void* stream);
int dct_phase_accum(unsigned long long* b, int n, void* stream);
int dct_gemm_bf16_bt(const uint16_t* A, const uint16_t* B, void* C, const float* bias, int M, int N, int K, int lda,
                     int ldb, int ldc, int epilogue, int out_f32, void* aux, uint16_t* bt_out, int bt_ld, void* stream);
int dct_gemm_bf16(const uint16_t* A, const uint16_t* B, void* C, const float* bias, int M, int N, int K, int lda,
                  int ldb, int ldc, int trans_a, int trans_b, int epilogue, int out_f32, int accumulate, void* aux,
                  void* stream);
// C [M][N] bf16 = act(gather(X) W^T + bias), X the dataset [rows][K] (row stride ldx), W [N][K]; see
// GatherFwd.  hipErrorInvalidValue (nothing launched) when the shape does not take the LDS-DMA kernels.
int dct_gemm_bf16_gather_fwd(const uint16_t* X, int ldx, const uint16_t* W, uint16_t* C, const float* bias, int M,
                             int N, int K, int epilogue, void* aux, const dct::GatherFwd* ga, void* stream);
// same, plus colsum[m] += sum over k of op(A)[m][k] (fused bias gradient; colsum accumulates)
int dct_gemm_bf16_ex(const uint16_t* A, const uint16_t* B, void* C, const float* bias, int M, int N, int K, int lda,
                     int ldb, int ldc, int trans_a, int trans_b, int epilogue, int out_f32, int accumulate, void* aux,
                     float* colsum, void* stream);
// fp32 C = residual + A W^T + bias (the residual-stream update of a transformer block)
int dct_gemm_bf16_residual(const uint16_t* A, const uint16_t* W, float* C, const float* bias, const float* residual,
                           int M, int N, int K, void* stream);
// Skinny layers (C <= 8 outputs, e.g. the classifier head) as bandwidth kernels:
//   fwd: Y[b][c] = sum_k X[b][k] W[c][k] + bias[c]            (bf16 X/W/Y)
//   dx : dX[b][k] = sum_c dZ[b][c] W[c][k], masked by aux[b][k] > 0 when aux (ReLU output)
//   dw : dW[c][k] += sum_b dZ[b][c] X[b][k] ; db[c] += sum_b dZ[b][c]   (fp32, accumulate)
int dct_skinny_fwd(const uint16_t* X, const uint16_t* W, const float* bias, uint16_t* Y, int B, int K, int C,
                   void* stream);
int dct_skinny_dx(const uint16_t* dZ, const uint16_t* W, const uint16_t* aux, uint16_t* dX, int B, int K, int C,
                  void* stream);
int dct_skinny_dw(const uint16_t* dZ, const uint16_t* X, float* dW, float* db, int B, int K, int C, void* stream);
int dct_skinny_head_supported(int K, int C);
int dct_gemm_bf16_dw_partials(const uint16_t* dZ, const uint16_t* X, float* part, float* colsum, int M, int N, int K,
                              int splits, void* stream);
int dct_gemm_dw_auto_splits(int M, int N, int K);
int dct_skinny_head(const uint16_t* H, const uint16_t* W, const float* bias, const int* labels, uint16_t* dH,
                    float* dW, float* db, float* loss_sum, int B, int K, int C, float grad_scale, int loss_kind,
                    float loss_scale, int relu_mask, void* stream);
// dZ = dY * act'(aux) (bf16 out); dbias[n] (+)= sum_m dZ[m][n]. dY is bf16. For RELU aux is
// the activation OUTPUT (bf16), for GELU the pre-activation (bf16), for NONE unused.
int dct_bias_act_bwd(const void* dY, const void* act_aux, uint16_t* dZ, float* dbias, int M, int N, int ldy, int act,
                     int accumulate_bias, void* stream);
// Row-wise CE (loss_kind 0) or MSE-vs-onehot (1): loss/correct sums (atomic fp32) and
// dlogits = dL/dz * grad_scale (bf16 if logits_bf16 else fp32).
int dct_loss_fwd_bwd(const void* logits, int logits_bf16, const int* labels, void* dlogits, float* loss_sum,
                     float* correct_sum, int M, int C, float grad_scale, int loss_kind, void* stream);
int dct_layernorm_fwd(const void* x, const float* w, const float* b, void* y, float* mean, float* rstd, int M, int N,
                      float eps, int in_bf16, int out_bf16, void* stream);
int dct_layernorm_bwd(const void* dy, const void* x, const float* w, const float* mean, const float* rstd, void* dx,
                      float* dw, float* db, int M, int N, int bf16_io, void* stream);
// narrow rows (N <= 256, N % 4 == 0, 16-B aligned): per-operand dtypes, + dres (fp32 residual
// gradient added into dx), optional bf16 copy dx2; dw/db ACCUMULATE (+=) through the slot
// workspace ws (dct_layernorm_bwd_ws_floats(N) floats, zeroed once, re-zeroed by the kernel).
int dct_layernorm_bwd_ex(const void* dy, int dy_bf16, const void* x, int x_bf16, const float* w, const float* mean,
                         const float* rstd, void* dx, int dx_bf16, uint16_t* dx2, const float* dres, float* dw,
                         float* db, float* ws, int M, int N, void* stream);
int dct_layernorm_bwd_ws_floats(int N);
// q/k/v: element (b, t, h, d) at ptr[(b*T + t)*ldq + h*D + d] (a packed QKV projection
// output); o/dout: at ptr[(b*T + t)*ldo + h*D + d]; lse fp32 [B*H*T].
int dct_attention_fwd(const uint16_t* q, const uint16_t* k, const uint16_t* v, uint16_t* o, float* lse, int Bsz, int H,
                      int T, int D, int ldq, int ldo, float scale, void* stream);
int dct_attention_bwd(const uint16_t* q, const uint16_t* k, const uint16_t* v, const uint16_t* o,
                      const uint16_t* dout, const float* lse, uint16_t* dq, uint16_t* dk, uint16_t* dv, int Bsz, int H,
                      int T, int D, int ldq, int ldo, float scale, void* stream);
int dct_tt_block_fwd(const uintptr_t* p, int n_ptrs, int Bsz, int T, int DM, int H, int FF, float eps, float scale,
                     void* stream);
int dct_tt_block_bwd(const uintptr_t* p, int n_ptrs, int Bsz, int T, int DM, int H, int FF, float scale,
                     void* stream);
int dct_tt_block_fwd_gx(const uintptr_t* p, int n_ptrs, int Bsz, int T, int DM, int H, int FF, float eps,
                        float scale, float* pool, const float* ex, const float* eE, const float* ec,
                        const uintptr_t* gx, int n_gx, void* stream);
int dct_tt_block_fwd_ex(const uintptr_t* p, int n_ptrs, int Bsz, int T, int DM, int H, int FF, float eps,
                        float scale, float* pool, const float* ex, const float* eE, const float* ec, void* stream);
int dct_tt_block_bwd_ex(const uintptr_t* p, int n_ptrs, int Bsz, int T, int DM, int H, int FF, float scale,
                        const float* dpool, uint16_t* dout16, const float* ex, const float* eE, const float* ec,
                        float* lnrep, unsigned* ticket, const uint16_t* a1, const uint16_t* wqkv,
                        const float* bqkv, void* stream);
int dct_tt_embed_fwd(const float* x, const float* E, const float* c, float* h, int B, int F, int Dm, void* stream);
int dct_tt_embed_bwd(const float* x, const float* dh, float* dE, float* dc, int B, int F, int Dm, void* stream);
int dct_tt_head_fwd(const uintptr_t* p, int n_ptrs, int B, int T, int Dm, int C, float eps, void* stream);
int dct_tt_head_bwd(const uintptr_t* p, int n_ptrs, int B, int T, int Dm, int C, float eps, void* stream);
int dct_tt_head_fused(const uintptr_t* p, int n_ptrs, int B, int T, int Dm, int C, float eps, void* stream);
int dct_gemm_bf16_dw_grouped(int n, const uint16_t* const* dZ, const uint16_t* const* X, float* const* C,
                             const int* M, const int* N, int K, float* const* colsum, int accumulate, void* stream);
int dct_gemm_bf16_dw_grouped_embed(int n, const uint16_t* const* dZ, const uint16_t* const* X, float* const* C,
                                   const int* M, const int* N, int K, float* const* colsum, int accumulate,
                                   const float* ex, const float* edh, float* edE, float* edc, int eB, int eF,
                                   void* stream);
int dct_gather_rows(const void* src, const int* idx, void* dst, int64_t n_rows, int row_bytes, void* stream);
// device-side barrier of the xGMI peer exchange (step_kernels.hip; barrier slots at byte offset off)
int dct_xg_barrier(void* recv, void* const* peers, int64_t off, unsigned* status, int world, int rank, unsigned tag,
                   long long timeout_ticks, void* stream);
// peer-to-peer gradient all-reduce + flat Adam over a PeerExchange (xg_adam.hip)
int64_t dct_xg_adam_buffer_bytes(int64_t n, int world);
int dct_xg_allreduce_adam(float* g, float* p, float* m, float* v, int64_t n, int64_t P, const int* step_counter,
                          float lr, float b1, float b2, float eps, float wd, void* recv, void* const* peers,
                          unsigned* status, int world, int rank, long long timeout_ticks, void* stream);
}
