// Whole-block fused forward of the TabTransformer layer (BASELINE.json config 5: 64 feature
// tokens, d_model 64, 4 heads of 16, FFN 256) - one workgroup per sample, every intermediate in LDS.
//
//   h1  = h  + Wo  Attn(Wqkv LN1(h) + bqkv) + bo
//   out = h1 + W2 gelu(W1 LN2(h1) + b1) + b2
//
// The unfused path is 7 kernels per layer (LN, QKV GEMM, attention, proj GEMM, LN, fc1, fc2), each
// a full HBM round trip of a [B*64, <=256] activation plus a launch: ~65 us per layer at batch 512
// on MI355X, of which the math is < 2 us.  Here a sample's 64 x 64 residual rows are read once,
// all seven stages run out of 68 KB of LDS (2 workgroups per CU), weights come from L2 (96 KB
// shared by every workgroup), and only the tensors the backward consumes are written - staged
// through LDS so every global store is a 16-byte coalesced chunk.  Same saved-tensor contract as
// the two unfused autograd nodes (ops/nn.py _PreNormAttnFn / _PreNormFFNFn), so the backward is
// unchanged.
//
// Work split (4 waves): LayerNorms and row-parallel GEMMs (proj, fc1, fc2) - wave w owns token
// rows 16w..16w+15; QKV GEMM + attention - wave w owns head w (its Q/K/V columns for all 64
// tokens), so attention never leaves the wave's registers and LDS rows.
// MFMA layouts: v_mfma_f32_16x16x32_bf16 (A: row = lane&15, k = 8*(lane>>4)+j; B likewise with
// col; C: col = lane&15, row = 4*(lane>>4)+r); attention uses the 16x16x16 form (head dim 16).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dct_common.h"

namespace dct {
namespace ttb {

// phase timestamps for tools/debug/tt_phase_prof.py (a.prof == nullptr in production)
#define TT_MARK(k) \
  if (a.prof && threadIdx.x == 0) a.prof[(size_t)blockIdx.x * 16 + (k)] = wall_clock64()

constexpr int T = 64, DM = 64, NH = 4, DH = 16, FF = 256;
constexpr int HS_LD = DM + 4;       // fp32 residual rows (272 B)
constexpr int AS_LD = DM + 8;       // bf16 LN output / attention output rows (144 B)
constexpr int QKV_LD = 3 * DM + 8;  // bf16 (400 B)
constexpr int F_LD = FF + 8;        // bf16 (528 B)
constexpr int HS_BYTES = T * HS_LD * 4;
constexpr int AS_BYTES = T * AS_LD * 2;
constexpr int R_BYTES = T * F_LD * 2;  // QKV (25.6 KB) then FFN hidden (33.8 KB)
constexpr int LDS_BYTES = HS_BYTES + 2 * AS_BYTES + R_BYTES;

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma32(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16(bf16x4 a, bf16x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float sum4g(float v) {  // over lanes l, l^16, l^32, l^48
  v += __shfl_xor(v, 16);
  v += __shfl_xor(v, 32);
  return v;
}
__device__ __forceinline__ float max4g(float v) {
  v = fmaxf(v, __shfl_xor(v, 16));
  v = fmaxf(v, __shfl_xor(v, 32));
  return v;
}
__device__ __forceinline__ bf16x4 pack4(f32x4 v) {
  bf16x4 r;
  r[0] = (short)f32_to_bf16(v[0]); r[1] = (short)f32_to_bf16(v[1]);
  r[2] = (short)f32_to_bf16(v[2]); r[3] = (short)f32_to_bf16(v[3]);
  return r;
}

// Optional feature-token embedding of the FIRST block (csrc/tt_io.hip embed_fwd_kernel, fused):
// the block input row of token f of sample b is  x[b, f] * E[f, :] + c[f, :]  (same fmaf as the
// standalone kernel, so bit-identical); computed where the kernels would read h, which is then never
// written to or read from HBM (8 MB at batch 512 each way)
struct Embed {
  const float* x;  // [B][T] features (null: the block input comes from h)
  const float* E;  // [T][DM]
  const float* c;  // [T][DM]
};

// Optional batch gather of the first block (the autograd engine's captured step, ops/nn.py
// fold_batch_gather): sample b's features are dataset row idx[wrap(*cursor * stride + b)] of X [rows][T],
// read where the embedding reads x; the workgroup also writes them to xdst (the backward's x) and the
// label to ydst, and the grid runs the rest of the step prologue (csrc/step_kernels.hip
// ag_prologue_kernel): Adam step counter += 1, zero[0, zero_n) cleared - one launch less per step
struct Gather {
  const float* X;
  const int64_t* idx;
  const int* cursor;
  int stride;
  int64_t n_items;
  float* xdst;
  const int64_t* Y;
  int64_t* ydst;
  int* step_counter;
  float* zero;
  int64_t zero_n;
};

struct Args {
  const float* h;
  const float *ln1_w, *ln1_b;
  const uint16_t* wqkv; const float* bqkv;
  const uint16_t* wo; const float* bo;
  const float *ln2_w, *ln2_b;
  const uint16_t* w1; const float* b1;
  const uint16_t* w2; const float* b2;
  uint16_t* a1; float* mean1; float* rstd1;
  uint16_t* qkv; uint16_t* o; float* lse;
  float* h1;
  uint16_t* a2; float* mean2; float* rstd2;
  uint16_t* f; uint16_t* pre;
  float* out;
  uint16_t* wT;  // transposed bf16 weights for the backward: W2^T | W1^T | Wo^T | Wqkv^T
  uint64_t* prof;  // optional phase timestamps (wall clock), 16 per workgroup
  float* pool;     // optional [B][DM]: the block output's mean over the sample's tokens (classifier head input)
  Embed em;        // optional: the first block's input computed from the features (h unused)
  Gather gx;       // optional (gx.X): those features gathered from the dataset (em.x is then the destination)
  int save;        // 0: inference (no_grad) - only `out` is written, no saved tensors / W^T
  int B;
  float eps, scale;
};


// 4 consecutive input columns 16 g + 4 q .. 16 g + 4 q + 3 of row r (token r) of the sample whose
// first global row is row0 (a multiple of T)
__device__ __forceinline__ float4 input_row4(const float* h, const Embed& em, int row0, int r, int g, int q) {
  // branch-free: (x, E row, c row) or (1, h row, +0) - fmaf(1, v, 0) == v for every non-zero v, and
  // the sign of a zero does not reach LayerNorm's (v - mean)
  const bool e = em.x != nullptr;
  const float xv = e ? em.x[row0 + r] : 1.f;
  const float* p = e ? em.E + r * DM : h + (size_t)(row0 + r) * DM;
  const float4 a = reinterpret_cast<const float4*>(p + 16 * g)[q];
  float4 cc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (e) cc = reinterpret_cast<const float4*>(em.c + r * DM + 16 * g)[q];
  return make_float4(fmaf(xv, a.x, cc.x), fmaf(xv, a.y, cc.y), fmaf(xv, a.z, cc.z), fmaf(xv, a.w, cc.w));
}

// 16 consecutive input columns 16 g .. 16 g + 15 of row r (token r) of the sample at row0 into v
__device__ __forceinline__ void input_row16(const float* h, const Embed& em, int row0, int r, int g, float* v) {
  const int row = row0 + r;
  if (em.x) {
    const float xv = em.x[row];
    const float4* ep = reinterpret_cast<const float4*>(em.E + r * DM + 16 * g);
    const float4* cp = reinterpret_cast<const float4*>(em.c + r * DM + 16 * g);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 e = ep[q], cc = cp[q];
      v[4 * q] = fmaf(xv, e.x, cc.x); v[4 * q + 1] = fmaf(xv, e.y, cc.y);
      v[4 * q + 2] = fmaf(xv, e.z, cc.z); v[4 * q + 3] = fmaf(xv, e.w, cc.w);
    }
  } else {
    const float4* p = reinterpret_cast<const float4*>(h + (size_t)row * DM + 16 * g);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 t = p[q];
      v[4 * q] = t.x; v[4 * q + 1] = t.y; v[4 * q + 2] = t.z; v[4 * q + 3] = t.w;
    }
  }
}

// offsets (elements) of the transposed weights in Args::wT / BwdArgs::wT
constexpr int WT_W2 = 0, WT_W1 = FF * DM, WT_WO = 2 * FF * DM, WT_QKV = 2 * FF * DM + DM * DM;
constexpr int WT_TOTAL = WT_QKV + 3 * DM * DM;

// wT <- transposes of this step's bf16 weights (grid-stride side task of the forward kernel:
// the backward's dX products need W^T rows as MFMA B fragments)
__device__ __forceinline__ void transpose_weights(const Args& a) {
  for (int e = blockIdx.x * 256 + threadIdx.x; e < WT_TOTAL; e += gridDim.x * 256) {
    uint16_t v;
    if (e < WT_W1) {            // W2 [DM][FF] -> W2^T [FF][DM]
      const int j = e / DM, n = e - j * DM;
      v = a.w2[n * FF + j];
    } else if (e < WT_WO) {     // W1 [FF][DM] -> W1^T [DM][FF]
      const int q = e - WT_W1, i = q / FF, j = q - i * FF;
      v = a.w1[j * DM + i];
    } else if (e < WT_QKV) {    // Wo [DM][DM] -> Wo^T
      const int q = e - WT_WO, i = q / DM, n = q - i * DM;
      v = a.wo[n * DM + i];
    } else {                    // Wqkv [3DM][DM] -> Wqkv^T [DM][3DM]
      const int q = e - WT_QKV, i = q / (3 * DM), j = q - i * (3 * DM);
      v = a.wqkv[j * DM + i];
    }
    a.wT[e] = v;
  }
}

// 64-row LDS tile -> contiguous global rows, 16-byte chunks over the whole workgroup.  All of a
// thread's LDS reads are issued before its stores (a rolled loop paid one LDS round trip each).
template <int ROW_BYTES, int LD_BYTES>
__device__ __forceinline__ void store_tile(void* g, const void* s) {
  constexpr int CPR = ROW_BYTES / 16, N = T * CPR / 256;
  static_assert(T * CPR % 256 == 0, "whole 16-byte chunks per thread");
  uint4 v[N];
#pragma unroll
  for (int it = 0; it < N; ++it) {
    const int idx = it * 256 + threadIdx.x, r = idx / CPR, c = idx - r * CPR;
    v[it] = *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(s) + r * LD_BYTES + c * 16);
  }
#pragma unroll
  for (int it = 0; it < N; ++it) {
    const int idx = it * 256 + threadIdx.x, r = idx / CPR, c = idx - r * CPR;
    *reinterpret_cast<uint4*>(reinterpret_cast<char*>(g) + r * ROW_BYTES + c * 16) = v[it];
  }
}

// LayerNorm of the wave's 16 rows: lane -> row 16w + (lane&15), columns 16g..16g+15.
// Input fp32 from `src` (global when from_global, else the LDS residual tile); the fp32 row is
// (re)written to HS, the bf16 normalised row to AS.
__device__ __forceinline__ void layer_norm_rows(const float* src, bool from_global, float* HS, uint16_t* AS,
                                                const float* w, const float* b, float* mean_out, float* rstd_out,
                                                int row0, float eps, const Embed& em) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r = 16 * wv + (lane & 15), g = lane >> 4;
  float v[16];
  if (from_global) {
    input_row16(src, em, row0, r, g, v);
  } else {
    const float* p = HS + r * HS_LD + 16 * g;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 t = reinterpret_cast<const float4*>(p)[q];
      v[4 * q] = t.x; v[4 * q + 1] = t.y; v[4 * q + 2] = t.z; v[4 * q + 3] = t.w;
    }
  }
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < 16; ++e) s += v[e];
  const float mean = sum4g(s) * (1.f / DM);
  float qv = 0.f;
#pragma unroll
  for (int e = 0; e < 16; ++e) { const float d = v[e] - mean; qv += d * d; }
  const float rstd = rsqrtf(sum4g(qv) * (1.f / DM) + eps);
  if (from_global) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      reinterpret_cast<float4*>(HS + r * HS_LD + 16 * g)[q] = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
  }
  float wv4[16], bv4[16];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 tw = reinterpret_cast<const float4*>(w + 16 * g)[q];
    const float4 tb = reinterpret_cast<const float4*>(b + 16 * g)[q];
    wv4[4 * q] = tw.x; wv4[4 * q + 1] = tw.y; wv4[4 * q + 2] = tw.z; wv4[4 * q + 3] = tw.w;
    bv4[4 * q] = tb.x; bv4[4 * q + 1] = tb.y; bv4[4 * q + 2] = tb.z; bv4[4 * q + 3] = tb.w;
  }
  bf16x8 o0, o1;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    o0[e] = (short)f32_to_bf16((v[e] - mean) * rstd * wv4[e] + bv4[e]);
    o1[e] = (short)f32_to_bf16((v[e + 8] - mean) * rstd * wv4[e + 8] + bv4[e + 8]);
  }
  *reinterpret_cast<bf16x8*>(AS + r * AS_LD + 16 * g) = o0;
  *reinterpret_cast<bf16x8*>(AS + r * AS_LD + 16 * g + 8) = o1;
  if (g == 0 && mean_out) {
    mean_out[row0 + r] = mean;
    rstd_out[row0 + r] = rstd;
  }
}

__global__ __launch_bounds__(256, 2) void tt_block_fwd_kernel(Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* HS = reinterpret_cast<float*>(smem);
  uint16_t* AS = reinterpret_cast<uint16_t*>(smem + HS_BYTES);
  uint16_t* OS = reinterpret_cast<uint16_t*>(smem + HS_BYTES + AS_BYTES);
  uint16_t* RS = reinterpret_cast<uint16_t*>(smem + HS_BYTES + 2 * AS_BYTES);
  const int bidx = blockIdx.x;
  const int row0 = bidx * T;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = lane & 15, g = lane >> 4;

  TT_MARK(0);
  Embed em = a.em;
  if (a.gx.X) {
    // this sample's dataset row; em.x rebased so that em.x[row0 + r] is its feature r
    int64_t q = (int64_t)a.gx.cursor[0] * a.gx.stride + bidx;
    q = q < a.gx.n_items ? q : (a.gx.n_items > 0 ? q % a.gx.n_items : 0);
    const int64_t drow = a.gx.idx[q];
    const float* xr = a.gx.X + drow * T;
    em.x = xr - row0;
    if (threadIdx.x < T) a.gx.xdst[row0 + threadIdx.x] = xr[threadIdx.x];
    if (threadIdx.x == 0) a.gx.ydst[bidx] = a.gx.Y[drow];
    if (bidx == 0 && threadIdx.x == 0 && a.gx.step_counter) a.gx.step_counter[0] += 1;
    if (a.gx.zero) {
      const int64_t n4 = a.gx.zero_n >> 2, t = (int64_t)bidx * blockDim.x + threadIdx.x;
      for (int64_t i = t; i < n4; i += (int64_t)gridDim.x * blockDim.x)
        reinterpret_cast<float4*>(a.gx.zero)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (t < a.gx.zero_n - (n4 << 2)) a.gx.zero[(n4 << 2) + t] = 0.f;
    }
  }
  // ---- P1: LN1 (rows of this wave)
  layer_norm_rows(a.h, true, HS, AS, a.ln1_w, a.ln1_b, a.mean1, a.rstd1, row0, a.eps, em);
  __syncthreads();
  TT_MARK(1);

  // ---- P2: a1 out; QKV = a1 Wqkv^T + bqkv for head wv (Q, K, V column tiles wv, 4+wv, 8+wv)
  if (a.save) store_tile<DM * 2, AS_LD * 2>(a.a1 + (size_t)row0 * DM, AS);
  {
    f32x4 acc[3][4];
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[t][i] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < DM / 32; ++ks) {
      bf16x8 bw[3], af[4];
#pragma unroll
      for (int t = 0; t < 3; ++t)
        bw[t] = *reinterpret_cast<const bf16x8*>(a.wqkv + (size_t)(t * DM + DH * wv + c) * DM + 32 * ks + 8 * g);
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const bf16x8*>(AS + (16 * i + c) * AS_LD + 32 * ks + 8 * g);
#pragma unroll
      for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[t][i] = mfma32(af[i], bw[t], acc[t][i]);
    }
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const int col = t * DM + DH * wv + c;
      const float bv = a.bqkv[col];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) RS[(16 * i + 4 * g + r) * QKV_LD + col] = f32_to_bf16(acc[t][i][r] + bv);
    }
  }
  __syncthreads();

  TT_MARK(2);
  // ---- P3: qkv out; attention of head wv over the 64 tokens (S^T = K Q^T; P V)
  if (a.save && a.qkv)  // null: the fused backward recomputes q, k, v from a1 (BwdArgs::wqkv)
    store_tile<3 * DM * 2, QKV_LD * 2>(a.qkv + (size_t)row0 * 3 * DM, RS);
  {
    const uint16_t* Qs = RS + DH * wv;
    const uint16_t* Ks = RS + DM + DH * wv;
    const uint16_t* Vs = RS + 2 * DM + DH * wv;
    f32x4 st[4][4];
    bf16x4 kf[4], qf[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      kf[i] = *reinterpret_cast<const bf16x4*>(Ks + (16 * i + c) * QKV_LD + 4 * g);
      qf[i] = *reinterpret_cast<const bf16x4*>(Qs + (16 * i + c) * QKV_LD + 4 * g);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) st[i][j] = mfma16(kf[i], qf[j], (f32x4){0.f, 0.f, 0.f, 0.f});
    bf16x4 pf[4][4];
    float lsev[4];
    // softmax in the exp2 domain: the scale carries log2(e), so each score is one fma + v_exp_f32
    // (__expf is fma, multiply by log2(e), v_exp_f32); lse leaves in natural-log units
    const float sl = a.scale * 1.4426950408889634f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float m = -3.402823466e+38f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) m = fmaxf(m, st[i][j][r]);
      m = max4g(m) * sl;
      float l = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = __builtin_amdgcn_exp2f(fmaf(st[i][j][r], sl, -m));
          st[i][j][r] = e;
          l += e;
        }
      l = sum4g(l);
      const float inv = 1.f / l;
#pragma unroll
      for (int i = 0; i < 4; ++i) pf[j][i] = pack4(st[i][j] * inv);
      lsev[j] = (m + __builtin_amdgcn_logf(l)) * 0.6931471805599453f;
    }
    bf16x4 vf[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint16_t* vp = Vs + (16 * i + 4 * g) * QKV_LD + c;
      vf[i][0] = (short)vp[0]; vf[i][1] = (short)vp[QKV_LD];
      vf[i][2] = (short)vp[2 * QKV_LD]; vf[i][3] = (short)vp[3 * QKV_LD];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 4; ++i) acc = mfma16(pf[j][i], vf[i], acc);
#pragma unroll
      for (int r = 0; r < 4; ++r) OS[(16 * j + 4 * g + r) * AS_LD + DH * wv + c] = f32_to_bf16(acc[r]);
    }
    if (g == 0 && a.save) {
#pragma unroll
      for (int j = 0; j < 4; ++j) a.lse[((size_t)bidx * NH + wv) * T + 16 * j + c] = lsev[j];
    }
  }
  __syncthreads();

  TT_MARK(3);
  // ---- P4: o out; h1 = h + o Wo^T + bo (rows of this wave); LN2 of the same rows
  if (a.save) store_tile<DM * 2, AS_LD * 2>(a.o + (size_t)row0 * DM, OS);
  // Row-parallel GEMMs split by COLUMNS across the waves (wave wv: column tile(s) wv for all 64
  // rows): each wave then streams only its quarter of the weight from L2 - the row split had
  // every wave fetch the whole matrix (4x the L2 traffic; fc1 was 10 us of a 30 us block).
  {  // proj: column tile wv
    f32x4 acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < DM / 32; ++ks) {
      const bf16x8 bw = *reinterpret_cast<const bf16x8*>(a.wo + (size_t)(16 * wv + c) * DM + 32 * ks + 8 * g);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        acc[i] = mfma32(*reinterpret_cast<const bf16x8*>(OS + (16 * i + c) * AS_LD + 32 * ks + 8 * g), bw, acc[i]);
    }
    const int col = 16 * wv + c;
    const float bv = a.bo[col];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) HS[(16 * i + 4 * g + r) * HS_LD + col] += acc[i][r] + bv;
  }
  __syncthreads();  // LN2 rows need every wave's columns
  layer_norm_rows(nullptr, false, HS, AS, a.ln2_w, a.ln2_b, a.mean2, a.rstd2, row0, a.eps, Embed{});
  __syncthreads();

  TT_MARK(4);
  // ---- P5: h1, a2 out; F = gelu(a2 W1^T + b1) for columns 64wv..64wv+63, pre-activation out
  if (a.save) {
    store_tile<DM * 4, HS_LD * 4>(a.h1 + (size_t)row0 * DM, HS);
    store_tile<DM * 2, AS_LD * 2>(a.a2 + (size_t)row0 * DM, AS);
  }
  {
    // Operands swapped (A = W1 rows, B = a2 rows): the C tile is [column][token], so each lane
    // holds 4 CONSECUTIVE columns of one token and the pre-activation / GELU outputs leave as
    // 8-byte stores (16 per lane instead of 64 two-byte ones, 8.6 -> see BASELINE.md)
    f32x4 acc[4][4];  // [token tile][column tile of this wave]
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[i][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < DM / 32; ++ks) {
      bf16x8 af[4], bw[4];
#pragma unroll
      for (int t = 0; t < 4; ++t)
        bw[t] = *reinterpret_cast<const bf16x8*>(a.w1 + (size_t)(64 * wv + 16 * t + c) * DM + 32 * ks + 8 * g);
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const bf16x8*>(AS + (16 * i + c) * AS_LD + 32 * ks + 8 * g);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[i][t] = mfma32(bw[t], af[i], acc[i][t]);
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int col0 = 64 * wv + 16 * t + 4 * g;
      const float4 bv = *reinterpret_cast<const float4*>(a.b1 + col0);
      const float bvs[4] = {bv.x, bv.y, bv.z, bv.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = 16 * i + c;
        uint16_t zp[4], fp[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float z = acc[i][t][r] + bvs[r];
          zp[r] = f32_to_bf16(z);
          fp[r] = f32_to_bf16(gelu_f(z));
        }
        if (a.save && a.pre)  // null: the fused backward recomputes pre from a2 (BwdArgs::a2)
          *reinterpret_cast<uint2*>(a.pre + (size_t)(row0 + row) * FF + col0) =
              make_uint2(zp[0] | ((uint32_t)zp[1] << 16), zp[2] | ((uint32_t)zp[3] << 16));
        *reinterpret_cast<uint2*>(RS + row * F_LD + col0) =
            make_uint2(fp[0] | ((uint32_t)fp[1] << 16), fp[2] | ((uint32_t)fp[3] << 16));
      }
    }
  }
  __syncthreads();

  TT_MARK(5);
  // ---- P6: f out; out = h1 + F W2^T + b2 for column tile wv
  if (a.save && a.f) store_tile<FF * 2, F_LD * 2>(a.f + (size_t)row0 * FF, RS);  // null: not stored
  {
    f32x4 acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < FF / 32; ++ks) {
      const bf16x8 bw = *reinterpret_cast<const bf16x8*>(a.w2 + (size_t)(16 * wv + c) * FF + 32 * ks + 8 * g);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        acc[i] = mfma32(*reinterpret_cast<const bf16x8*>(RS + (16 * i + c) * F_LD + 32 * ks + 8 * g), bw, acc[i]);
    }
    const int col = 16 * wv + c;
    const float bv = a.b2[col];
    float cs = 0.f;  // this lane's 16 rows of the output column (pool)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float* hp = HS + (16 * i + 4 * g + r) * HS_LD + col;
        const float v = *hp + (acc[i][r] + bv);
        *hp = v;
        cs += v;
      }
    if (a.pool) {
      // the last block hands the head its token mean (256 B per sample) instead of the 16-KB output
      // tile, which the head read twice (its forward and its backward recompute): the column's four
      // row groups (lanes c, c + 16, c + 32, c + 48) summed in registers
      cs += __shfl_xor(cs, 16);
      cs += __shfl_xor(cs, 32);
      if (g == 0) a.pool[(size_t)bidx * DM + col] = cs * (1.f / T);
    }
  }
  __syncthreads();
  TT_MARK(6);
  if (a.out) store_tile<DM * 4, HS_LD * 4>(a.out + (size_t)row0 * DM, HS);
  if (a.save) transpose_weights(a);
  TT_MARK(7);
}

// ============================================================================ backward
// dX chain of the same block for one sample per workgroup (the dW products stay split-K GEMMs
// over all B*64 rows, fed by the dZ tensors written here):
//   dF   = bf16(dout) W2 ; dpre = dF * gelu'(pre)              -> dpre (global, for dW1 / db1)
//   da2  = dpre W1 ; dh1 = dout + LN2_bwd(da2)                  -> bf16(dh1) (global, for dWo / dbo)
//   do   = bf16(dh1) Wo ; attention backward per head           -> dqkv (global, for dWqkv / dbqkv)
//   da1  = dqkv Wqkv ; dh = dh1 + LN1_bwd(da1)                  -> dh fp32 + bf16 copy
// LayerNorm weight/bias gradients: per-column partials reduced over the workgroup in LDS, one
// global atomic per column per workgroup.  LayerNorm backwards run directly on the MFMA C layout
// (row sums = 4 tiles in-lane + xor-shuffles over the 16 lanes of a row group).
// LDS (80 KB -> 2 workgroups per CU): G fp32 residual gradient rows; X bf16 A-operand rows;
// R pre/dpre, later qkv/dqkv (dq, dk, dv written in place over q, k, v of the wave's own head);
// O / dO for the attention backward.
struct BwdArgs {
  const float* dout;  // [M][DM] fp32
  const float* h; const float* mean1; const float* rstd1; const float* ln1_w;
  const uint16_t* qkv; const uint16_t* o; const float* lse;
  const float* h1; const float* mean2; const float* rstd2; const float* ln2_w;
  const uint16_t* pre;  // null: recompute pre = a2 W1^T + b1 (same MFMAs and roundings as the forward)
  const uint16_t* wT;
  const uint16_t* a2; const uint16_t* w1; const float* b1;  // the recompute's operands
  uint16_t* dpre; uint16_t* dh1_16; uint16_t* dqkv; float* dh; uint16_t* dh16;
  Embed em;            // optional: the first block's input recomputed from the features (h unused)
  const float* dpool;  // optional [B][DM]: the gradient of the token mean (pool) instead of dout rows;
  uint16_t* dout16;    // then bf16(dout) [M][DM] is written here for the W2 gradient GEMM
  float *dln1_w, *dln1_b, *dln2_w, *dln2_b;
  // optional: LN_REP replicas of the four LayerNorm gradient vectors [LN_REP][4][DM] and a ticket, both
  // zero between launches (the last workgroup folds the replicas into dln* and re-zeroes them)
  float* lnrep; unsigned* ticket;
  // optional: with qkv null, q / k / v are recomputed from a1 by the forward's QKV MFMAs (bit-identical)
  const uint16_t* a1; const uint16_t* wqkv; const float* bqkv;
  uint64_t* prof;
  float scale;
};
// The LayerNorm parameter gradients are per-workgroup column sums added into the same 4 x 64 floats
// by every workgroup: 512 adders on one 1 KB row run the memory-side float atomics ~14x below their
// rate (MI355X_MICROARCH.md 'Global float atomics', contention) - a ~5 us tail on every backward
// block kernel.  Workgroup b adds into replica b % LN_REP instead (32 adders per address at batch
// 512), and the workgroup that finishes last folds the replicas.
constexpr int LN_REP = 16;

constexpr int XB_LD = DM + 8;  // bf16 rows (144 B)
constexpr int G_BYTES = T * HS_LD * 4;
constexpr int X_BYTES = T * XB_LD * 2;
constexpr int BWD_LDS = G_BYTES + X_BYTES + R_BYTES + 2 * X_BYTES + 4 * DM * 4 + NH * T * 4;

__device__ __forceinline__ float rowsum16(float v) {  // over the 16 lanes of a row group
  v += __shfl_xor(v, 1);
  v += __shfl_xor(v, 2);
  v += __shfl_xor(v, 4);
  v += __shfl_xor(v, 8);
  return v;
}

// Copy this wave's 16 rows of an LDS bf16 tile to global rows (16-byte chunks).
template <int ROW_BYTES, int LD_BYTES>
__device__ __forceinline__ void store_rows16(void* gdst, const void* s, int wv, int lane) {
  constexpr int CPR = ROW_BYTES / 16;
  for (int idx = lane; idx < 16 * CPR; idx += 64) {
    const int r = 16 * wv + idx / CPR, c = idx % CPR;
    *reinterpret_cast<uint4*>(reinterpret_cast<char*>(gdst) + r * ROW_BYTES + c * 16) =
        *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(s) + r * LD_BYTES + c * 16);
  }
}
// global rows -> LDS tile (all 64 rows, whole workgroup).  Every global load of a thread is in
// flight before the first LDS write: the rolled loop was partly unrolled by the compiler and ran its
// remainder one HBM round trip per iteration (~2 us of a 3.5 us staging phase).
template <int ROW_BYTES, int LD_BYTES>
__device__ __forceinline__ void load_tile(void* s, const void* gsrc) {
  constexpr int CPR = ROW_BYTES / 16, N = T * CPR / 256;
  static_assert(T * CPR % 256 == 0, "whole 16-byte chunks per thread");
  uint4 v[N];
#pragma unroll
  for (int it = 0; it < N; ++it) {
    const int idx = it * 256 + threadIdx.x, r = idx / CPR, c = idx - r * CPR;
    v[it] = *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(gsrc) + r * ROW_BYTES + c * 16);
  }
#pragma unroll
  for (int it = 0; it < N; ++it) {
    const int idx = it * 256 + threadIdx.x, r = idx / CPR, c = idx - r * CPR;
    *reinterpret_cast<uint4*>(reinterpret_cast<char*>(s) + r * LD_BYTES + c * 16) = v[it];
  }
}

// LayerNorm backward of the wave's 16 rows in row layout (lane -> row 16w + (lane&15), columns
// 16g..16g+15): da from the fp32 scratch tile S (the column-split dX GEMM wrote it), x from global,
// dres / result in G.  dx = rstd (gw - mean(gw) - xhat mean(gw xhat)) + dres, gw = da * w;
// weight / bias partial column sums reduced over the wave's rows, then LDS atomics into red.
__device__ __forceinline__ void ln_bwd_rows(const float* S, const float* x, const float* mean, const float* rstd,
                                            const float* w, float* G, float* red_w, float* red_b, int row0, int wv,
                                            int lane, const Embed& em) {
  const int rl = 16 * wv + (lane & 15), g = lane >> 4;
  const float mu = mean[row0 + rl], rs = rstd[row0 + rl];
  float da[16], xh[16], s1 = 0.f, s2 = 0.f;  // gw = da * w recomputed below (16 fewer live VGPRs)
  const float4* sp = reinterpret_cast<const float4*>(S + rl * HS_LD + 16 * g);
  const float4* wp = reinterpret_cast<const float4*>(w + 16 * g);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 dv = sp[q], ww = wp[q], xv = input_row4(x, em, row0, rl, g, q);
    const float xs[4] = {xv.x, xv.y, xv.z, xv.w};
    const float ds[4] = {dv.x, dv.y, dv.z, dv.w}, ws[4] = {ww.x, ww.y, ww.z, ww.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = 4 * q + e;
      da[k] = ds[e];
      xh[k] = (xs[e] - mu) * rs;
      const float gw = ds[e] * ws[e];
      s1 += gw;
      s2 += gw * xh[k];
    }
  }
  s1 = sum4g(s1) * (1.f / DM);
  s2 = sum4g(s2) * (1.f / DM);
  float4* gp = reinterpret_cast<float4*>(G + rl * HS_LD + 16 * g);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float4 v = gp[q];
    const float4 ww = wp[q];
    v.x += rs * (da[4 * q] * ww.x - s1 - xh[4 * q] * s2);
    v.y += rs * (da[4 * q + 1] * ww.y - s1 - xh[4 * q + 1] * s2);
    v.z += rs * (da[4 * q + 2] * ww.z - s1 - xh[4 * q + 2] * s2);
    v.w += rs * (da[4 * q + 3] * ww.w - s1 - xh[4 * q + 3] * s2);
    gp[q] = v;
  }
  // column sums over the wave's 16 rows by recursive halving across the 16 lanes of a row group:
  // 15 shuffles per quantity (not 16 x 4), lane j ends with column 16g + j
  float vw[16], vb[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) { vw[k] = da[k] * xh[k]; vb[k] = da[k]; }
#pragma unroll
  for (int half = 8; half >= 1; half >>= 1) {
    const bool hi = (lane & half) != 0;
#pragma unroll
    for (int k = 0; k < half; ++k) {
      const float sw = hi ? vw[k] : vw[k + half], kw = hi ? vw[k + half] : vw[k];
      const float sb = hi ? vb[k] : vb[k + half], kb = hi ? vb[k + half] : vb[k];
      vw[k] = kw + __shfl_xor(sw, half);
      vb[k] = kb + __shfl_xor(sb, half);
    }
  }
  atomicAdd(red_w + 16 * g + (lane & 15), vw[0]);
  atomicAdd(red_b + 16 * g + (lane & 15), vb[0]);
}

// G own rows (row layout) -> bf16 X own rows
__device__ __forceinline__ void rows_to_bf16(const float* G, uint16_t* X, int wv, int lane) {
  const int rl = 16 * wv + (lane & 15), g = lane >> 4;
  const float4* gp = reinterpret_cast<const float4*>(G + rl * HS_LD + 16 * g);
  bf16x8 o[2];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 v = gp[q];
    o[q >> 1][4 * (q & 1)] = (short)f32_to_bf16(v.x);
    o[q >> 1][4 * (q & 1) + 1] = (short)f32_to_bf16(v.y);
    o[q >> 1][4 * (q & 1) + 2] = (short)f32_to_bf16(v.z);
    o[q >> 1][4 * (q & 1) + 3] = (short)f32_to_bf16(v.w);
  }
  *reinterpret_cast<bf16x8*>(X + rl * XB_LD + 16 * g) = o[0];
  *reinterpret_cast<bf16x8*>(X + rl * XB_LD + 16 * g + 8) = o[1];
}

// RECOMP: the forward did not store the FFN pre-activation (32 KB per sample written, then read back
// here); P1 recomputes it from the saved a2 (8 KB) and W1 in the dF tile's own lane layout instead
template <bool RECOMP>
__global__ __launch_bounds__(256, 2) void tt_block_bwd_kernel(BwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* G = reinterpret_cast<float*>(smem);
  uint16_t* X = reinterpret_cast<uint16_t*>(smem + G_BYTES);
  uint16_t* R = reinterpret_cast<uint16_t*>(smem + G_BYTES + X_BYTES);
  uint16_t* Os = reinterpret_cast<uint16_t*>(smem + G_BYTES + X_BYTES + R_BYTES);
  uint16_t* dOs = Os + T * XB_LD;
  float* S = reinterpret_cast<float*>(Os);  // fp32 [T][HS_LD] scratch over Os + dOs (free outside P4-P6)
  static_assert(T * HS_LD * 4 <= 2 * X_BYTES, "scratch must fit in Os + dOs");
  float* red = reinterpret_cast<float*>(smem + G_BYTES + 3 * X_BYTES + R_BYTES);  // [4][DM]
  float* sdl = red + 4 * DM;                                                       // [NH][T]
  const int bidx = blockIdx.x, row0 = bidx * T;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = lane & 15, g = lane >> 4;
  const uint16_t* W2T = a.wT + WT_W2;
  const uint16_t* W1T = a.wT + WT_W1;
  const uint16_t* WoT = a.wT + WT_WO;
  const uint16_t* WqT = a.wT + WT_QKV;

  TT_MARK(0);
  // ---- P0: pre -> R (whole tile); dout rows -> G (fp32) and X (bf16); zero the LN partials
  {
    // dout in row layout (lane -> row 16wv + (lane & 15), columns 16g..16g+15): 4 x 16-B loads
    // per lane issued with the pre tile's, then 16-B LDS writes (was 16 scalar loads + 32 stores)
    const int rl = 16 * wv + (lane & 15);
    // (with dpool: the head's gradient of the token mean, the same for every token, / T; x 1 is exact)
    const float4* dp = reinterpret_cast<const float4*>(a.dpool ? a.dpool + (size_t)bidx * DM + 16 * g
                                                                : a.dout + (size_t)(row0 + rl) * DM + 16 * g);
    const float dsc = a.dpool ? 1.f / T : 1.f;
    float4 dv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 v = dp[q];
      dv[q] = make_float4(v.x * dsc, v.y * dsc, v.z * dsc, v.w * dsc);
    }
    if constexpr (RECOMP) load_tile<DM * 2, XB_LD * 2>(Os, a.a2 + (size_t)row0 * DM);  // Os is free until P4
    else load_tile<FF * 2, F_LD * 2>(R, a.pre + (size_t)row0 * FF);
    red[threadIdx.x] = 0.f;
    float4* gp = reinterpret_cast<float4*>(G + rl * HS_LD + 16 * g);
    bf16x8 o[2];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      gp[q] = dv[q];
      o[q >> 1][4 * (q & 1)] = (short)f32_to_bf16(dv[q].x);
      o[q >> 1][4 * (q & 1) + 1] = (short)f32_to_bf16(dv[q].y);
      o[q >> 1][4 * (q & 1) + 2] = (short)f32_to_bf16(dv[q].z);
      o[q >> 1][4 * (q & 1) + 3] = (short)f32_to_bf16(dv[q].w);
    }
    *reinterpret_cast<bf16x8*>(X + rl * XB_LD + 16 * g) = o[0];
    *reinterpret_cast<bf16x8*>(X + rl * XB_LD + 16 * g + 8) = o[1];
  }
  __syncthreads();
  if (a.dout16) store_tile<DM * 2, XB_LD * 2>(a.dout16 + (size_t)row0 * DM, X);

  TT_MARK(1);
  // ---- P1: dpre = (bf16(dout) W2) * gelu'(pre) for columns 64wv..64wv+63 (all rows), in place over
  // pre in R.  The dX products are split by COLUMNS across the waves, so each wave streams a
  // quarter of the transposed weight from L2 (a row split fetches all of it per wave).
  {
    f32x4 acc[4][4];  // [row tile][column tile of this wave]
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[i][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < DM / 32; ++ks) {
      bf16x8 af[4], bw[4];
#pragma unroll
      for (int t = 0; t < 4; ++t)
        bw[t] = *reinterpret_cast<const bf16x8*>(W2T + (size_t)(64 * wv + 16 * t + c) * DM + 32 * ks + 8 * g);
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const bf16x8*>(X + (16 * i + c) * XB_LD + 32 * ks + 8 * g);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[i][t] = mfma32(bw[t], af[i], acc[i][t]);  // C = [column][token]
    }
    if constexpr (RECOMP) {
      // pre = a2 W1^T + b1 for the same (column, token) lanes: the forward's P5 MFMAs (A = W1 rows,
      // B = a2 rows, k-steps in the same order) and its bf16 rounding -> bit-identical pre
      f32x4 pz[4][4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int t = 0; t < 4; ++t) pz[i][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < DM / 32; ++ks) {
        bf16x8 af[4], bw[4];
#pragma unroll
        for (int t = 0; t < 4; ++t)
          bw[t] = *reinterpret_cast<const bf16x8*>(a.w1 + (size_t)(64 * wv + 16 * t + c) * DM + 32 * ks + 8 * g);
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const bf16x8*>(Os + (16 * i + c) * XB_LD + 32 * ks + 8 * g);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int t = 0; t < 4; ++t) pz[i][t] = mfma32(bw[t], af[i], pz[i][t]);
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float4 bv = *reinterpret_cast<const float4*>(a.b1 + 64 * wv + 16 * t + 4 * g);
        const float bvs[4] = {bv.x, bv.y, bv.z, bv.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          uint16_t dp[4];
#pragma unroll
          for (int r = 0; r < 4; ++r)
            dp[r] = f32_to_bf16(acc[i][t][r] * gelu_grad_f(bf16_to_f32(f32_to_bf16(pz[i][t][r] + bvs[r]))));
          *reinterpret_cast<uint2*>(R + (16 * i + c) * F_LD + 64 * wv + 16 * t + 4 * g) =
              make_uint2(dp[0] | ((uint32_t)dp[1] << 16), dp[2] | ((uint32_t)dp[3] << 16));
        }
      }
    } else {
      // each lane: 4 consecutive columns of one token -> one 8-byte LDS read-modify-write per tile
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          uint2* pp = reinterpret_cast<uint2*>(R + (16 * i + c) * F_LD + 64 * wv + 16 * t + 4 * g);
          const uint2 pv = *pp;
          const uint16_t pr[4] = {(uint16_t)(pv.x & 0xFFFF), (uint16_t)(pv.x >> 16), (uint16_t)(pv.y & 0xFFFF),
                                  (uint16_t)(pv.y >> 16)};
          uint16_t dp[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) dp[r] = f32_to_bf16(acc[i][t][r] * gelu_grad_f(bf16_to_f32(pr[r])));
          *pp = make_uint2(dp[0] | ((uint32_t)dp[1] << 16), dp[2] | ((uint32_t)dp[3] << 16));
        }
    }
    // dpre out: this wave's 64-column block of all 64 rows (128 B per row, 16-byte chunks); null: not stored
#pragma unroll
    for (int q = 0; q < (a.dpre ? 8 : 0); ++q) {
      const int idx = q * 64 + lane, rr = idx >> 3, cc = idx & 7;
      *reinterpret_cast<uint4*>(a.dpre + (size_t)(row0 + rr) * FF + 64 * wv + cc * 8) =
          *reinterpret_cast<const uint4*>(R + rr * F_LD + 64 * wv + cc * 8);
    }
  }
  __syncthreads();  // da2 reads every wave's dpre columns

  TT_MARK(2);
  // ---- P2/P3: da2 = dpre W1 (column tile wv, all rows) -> fp32 scratch S; dh1 = dout + LN2_bwd(da2)
  {
    f32x4 acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < FF / 32; ++ks) {
      const bf16x8 bw = *reinterpret_cast<const bf16x8*>(W1T + (size_t)(16 * wv + c) * FF + 32 * ks + 8 * g);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        acc[i] = mfma32(*reinterpret_cast<const bf16x8*>(R + (16 * i + c) * F_LD + 32 * ks + 8 * g), bw, acc[i]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) S[(16 * i + 4 * g + r) * HS_LD + 16 * wv + c] = acc[i][r];
  }
  __syncthreads();
  ln_bwd_rows(S, a.h1, a.mean2, a.rstd2, a.ln2_w, G, red + 2 * DM, red + 3 * DM, row0, wv, lane, Embed{});
  rows_to_bf16(G, X, wv, lane);
  store_rows16<DM * 2, XB_LD * 2>(a.dh1_16 + (size_t)row0 * DM, X, wv, lane);
  __syncthreads();  // do reads all rows of X; S (over Os / dOs) fully consumed

  TT_MARK(3);
  // ---- P4: do = bf16(dh1) Wo (column tile wv, all rows) -> dOs
  {
    f32x4 acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < DM / 32; ++ks) {
      const bf16x8 bw = *reinterpret_cast<const bf16x8*>(WoT + (size_t)(16 * wv + c) * DM + 32 * ks + 8 * g);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        acc[i] = mfma32(*reinterpret_cast<const bf16x8*>(X + (16 * i + c) * XB_LD + 32 * ks + 8 * g), bw, acc[i]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) dOs[(16 * i + 4 * g + r) * XB_LD + 16 * wv + c] = f32_to_bf16(acc[i][r]);
  }
  __syncthreads();  // every wave is done with R (dpre) and has written its dO columns

  TT_MARK(4);
  // ---- P5: qkv -> R (or a1 -> X and the forward's QKV GEMM), o -> Os
  if (a.qkv) load_tile<3 * DM * 2, QKV_LD * 2>(R, a.qkv + (size_t)row0 * 3 * DM);
  else load_tile<DM * 2, XB_LD * 2>(X, a.a1 + (size_t)row0 * DM);  // X is free until P7
  load_tile<DM * 2, XB_LD * 2>(Os, a.o + (size_t)row0 * DM);
  __syncthreads();
  if (!a.qkv) {
    // the forward's P2 for head wv - same operands (a1 as the forward staged it), k order and
    // rounding, so q, k, v are bit-identical to the ones it no longer stores (12 MB written and 12 MB
    // read back per block at batch 512)
    f32x4 acc[3][4];
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[t][i] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < DM / 32; ++ks) {
      bf16x8 bw[3], af[4];
#pragma unroll
      for (int t = 0; t < 3; ++t)
        bw[t] = *reinterpret_cast<const bf16x8*>(a.wqkv + (size_t)(t * DM + DH * wv + c) * DM + 32 * ks + 8 * g);
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const bf16x8*>(X + (16 * i + c) * XB_LD + 32 * ks + 8 * g);
#pragma unroll
      for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[t][i] = mfma32(af[i], bw[t], acc[t][i]);
    }
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const int col = t * DM + DH * wv + c;
      const float bv = a.bqkv[col];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) R[(16 * i + 4 * g + r) * QKV_LD + col] = f32_to_bf16(acc[t][i][r] + bv);
    }
    __syncthreads();
  }

  TT_MARK(5);
  // ---- P6: attention backward of head wv; dq, dk, dv overwrite q, k, v of the head in R
  {
    uint16_t* Qh = R + DH * wv;
    uint16_t* Kh = R + DM + DH * wv;
    uint16_t* Vh = R + 2 * DM + DH * wv;
    const uint16_t* Oh = Os + DH * wv;
    const uint16_t* Gh = dOs + DH * wv;
    const float* lb = a.lse + ((size_t)bidx * NH + wv) * T;
    float* dl = sdl + wv * T;
    {  // delta_q = rowsum(dO_q * O_q) over the head's 16 columns
      float sacc = 0.f;
#pragma unroll
      for (int d = 0; d < DH; d += 4) {
        const bf16x4 o4 = *reinterpret_cast<const bf16x4*>(Oh + lane * XB_LD + d);
        const bf16x4 g4 = *reinterpret_cast<const bf16x4*>(Gh + lane * XB_LD + d);
#pragma unroll
        for (int e = 0; e < 4; ++e) sacc += bf16_to_f32((uint16_t)o4[e]) * bf16_to_f32((uint16_t)g4[e]);
      }
      dl[lane] = sacc;
    }
    auto ld4 = [](const uint16_t* p) { return *reinterpret_cast<const bf16x4*>(p); };
    auto ld4col = [](const uint16_t* p, int ld) {
      bf16x4 r;
      r[0] = (short)p[0]; r[1] = (short)p[ld]; r[2] = (short)p[2 * ld]; r[3] = (short)p[3 * ld];
      return r;
    };
    bf16x4 qf[4], kf[4], gf[4], vf[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      qf[j] = ld4(Qh + (16 * j + c) * QKV_LD + 4 * g);
      kf[j] = ld4(Kh + (16 * j + c) * QKV_LD + 4 * g);
      vf[j] = ld4(Vh + (16 * j + c) * QKV_LD + 4 * g);
      gf[j] = ld4(Gh + (16 * j + c) * XB_LD + 4 * g);
    }
    f32x4 dv[4], dk[4], dq[4];
    {  // pass A: S = Q K^T, dP = dO V^T (C: row = query, col = key) -> dV = P^T dO, dK = dS^T Q
      f32x4 sc[4][4], dp[4][4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          sc[j][i] = mfma16(qf[j], kf[i], (f32x4){0.f, 0.f, 0.f, 0.f});
          dp[j][i] = mfma16(gf[j], vf[i], (f32x4){0.f, 0.f, 0.f, 0.f});
        }
      bf16x4 pa[4][4], dsa[4][4];
      const float sl = a.scale * 1.4426950408889634f;  // P recomputed in the exp2 domain (one fma + v_exp_f32)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int qi = 16 * j + 4 * g + r;
          const float lq = lb[qi] * 1.4426950408889634f, dq_ = dl[qi];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float p = __builtin_amdgcn_exp2f(fmaf(sc[j][i][r], sl, -lq));
            sc[j][i][r] = p;
            dp[j][i][r] = p * (dp[j][i][r] - dq_);
          }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) { pa[i][j] = pack4(sc[j][i]); dsa[i][j] = pack4(dp[j][i]); }
      }
      bf16x4 gcol[4], qcol[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        gcol[j] = ld4col(Gh + (16 * j + 4 * g) * XB_LD + c, XB_LD);
        qcol[j] = ld4col(Qh + (16 * j + 4 * g) * QKV_LD + c, QKV_LD);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        dv[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
        dk[i] = dv[i];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          dv[i] = mfma16(pa[i][j], gcol[j], dv[i]);
          dk[i] = mfma16(dsa[i][j], qcol[j], dk[i]);
        }
      }
    }
    {  // pass B: S^T = K Q^T, dP^T = V dO^T (C: row = key, col = query) -> dQ = dS K
      f32x4 st[4][4], dpt[4][4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          st[i][j] = mfma16(kf[i], qf[j], (f32x4){0.f, 0.f, 0.f, 0.f});
          dpt[i][j] = mfma16(vf[i], gf[j], (f32x4){0.f, 0.f, 0.f, 0.f});
        }
      bf16x4 dsq[4][4];
      const float sl = a.scale * 1.4426950408889634f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int qi = 16 * j + c;
        const float lq = lb[qi] * 1.4426950408889634f, dq_ = dl[qi];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          f32x4 tv;
#pragma unroll
          for (int r = 0; r < 4; ++r)
            tv[r] = __builtin_amdgcn_exp2f(fmaf(st[i][j][r], sl, -lq)) * (dpt[i][j][r] - dq_);
          dsq[j][i] = pack4(tv);
        }
      }
      bf16x4 kcol[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) kcol[i] = ld4col(Kh + (16 * i + 4 * g) * QKV_LD + c, QKV_LD);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        dq[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < 4; ++i) dq[j] = mfma16(dsq[j][i], kcol[i], dq[j]);
      }
    }
    // all of this head's reads of q, k, v are done (same wave, LDS in order) -> overwrite in place
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rr = (16 * i + 4 * g + r) * QKV_LD + c;
        Qh[rr] = f32_to_bf16(dq[i][r] * a.scale);
        Kh[rr] = f32_to_bf16(dk[i][r] * a.scale);
        Vh[rr] = f32_to_bf16(dv[i][r]);
      }
  }
  __syncthreads();

  TT_MARK(6);
  // ---- P7: dqkv out; da1 = dqkv Wqkv (column tile wv, all rows) -> S; dh = dh1 + LN1_bwd(da1)
  store_tile<3 * DM * 2, QKV_LD * 2>(a.dqkv + (size_t)row0 * 3 * DM, R);
  {
    f32x4 acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 3 * DM / 32; ++ks) {
      const bf16x8 bw = *reinterpret_cast<const bf16x8*>(WqT + (size_t)(16 * wv + c) * (3 * DM) + 32 * ks + 8 * g);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        acc[i] = mfma32(*reinterpret_cast<const bf16x8*>(R + (16 * i + c) * QKV_LD + 32 * ks + 8 * g), bw, acc[i]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) S[(16 * i + 4 * g + r) * HS_LD + 16 * wv + c] = acc[i][r];
  }
  __syncthreads();
  TT_MARK(7);
  ln_bwd_rows(S, a.h, a.mean1, a.rstd1, a.ln1_w, G, red, red + DM, row0, wv, lane, a.em);
  if (a.dh16) {  // null for the embedding block: only the fp32 dh feeds the embedding's gradient
    rows_to_bf16(G, X, wv, lane);
    store_rows16<DM * 2, XB_LD * 2>(a.dh16 + (size_t)row0 * DM, X, wv, lane);
  }
  store_rows16<DM * 4, HS_LD * 4>(a.dh + (size_t)row0 * DM, G, wv, lane);
  __syncthreads();
  float* dsts[4] = {a.dln1_w, a.dln1_b, a.dln2_w, a.dln2_b};
  if (!a.lnrep) {  // LayerNorm parameter gradients: one atomic per column per workgroup
    atomicAdd(dsts[threadIdx.x >> 6] + (threadIdx.x & 63), red[threadIdx.x]);
  } else {
    atomicAdd(a.lnrep + (blockIdx.x % LN_REP) * 4 * DM + threadIdx.x, red[threadIdx.x]);
    // the add has been performed (float atomics execute at the memory side, so completion is all the
    // ordering the fold needs - an agent-scope release fence here would write back the XCD's L2 in every
    // workgroup: 0.339 -> 0.556 ms per TabTransformer step).  Hardware assumptions of gfx950 this relies
    // on, outside the HIP memory model: vmcnt covers a no-return atomic until the memory side
    // has acknowledged it (gfx9: stores and atomics share vmcnt); device-scope float atomics, the ticket's
    // and the fold's read-and-zero exchanges all execute beyond the per-XCD L2; the asm's memory clobber
    // keeps the compiler from moving the add below the wait.  A late add would stay in its replica, so
    // tests/test_kernels_gpu.py::test_tt_ln_replica_fold_complete_and_matches_direct_atomics checks the
    // workspace is exactly zero after every launch at B = 512 / 1024 and the fold equals direct atomics.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // (every read of red is done: red[0] carries the verdict; no static LDS in this kernel)
    if (threadIdx.x == 0)
      red[0] = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1
                   ? 1.f : 0.f;
    __syncthreads();
    if (red[0] != 0.f) {  // every other workgroup's adds are done: fold (read-and-zero at the memory side)
      float v = 0.f;
#pragma unroll
      for (int r = 0; r < LN_REP; ++r) v += atomicExch(a.lnrep + r * 4 * DM + threadIdx.x, 0.f);
      atomicAdd(dsts[threadIdx.x >> 6] + (threadIdx.x & 63), v);
      if (threadIdx.x == 0) __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  TT_MARK(8);
}

}  // namespace ttb
}  // namespace dct

extern "C" {

// ptrs (27, in order): h, ln1_w, ln1_b, wqkv, bqkv, wo, bo, ln2_w, ln2_b, w1, b1, w2, b2,
//   a1, mean1, rstd1, qkv, o, lse, h1, a2, mean2, rstd2, f, pre, out, wT
// pool (optional): the last block's token mean for the classifier head; `out` (p[25]) may then be null.
// ex / eE / ec (optional): the first block's input embedded from the features x [B][T] (E, c [T][DM]);
// h (p[0]) is then not read and may be null
static int tt_block_fwd_impl(const uintptr_t* p, int n_ptrs, int Bsz, int T, int DM, int H, int FF, float eps,
                             float scale, float* pool, const float* ex, const float* eE, const float* ec,
                             const dct::ttb::Gather& gx, void* stream);

int dct_tt_block_fwd_ex(const uintptr_t* p, int n_ptrs, int Bsz, int T, int DM, int H, int FF, float eps,
                        float scale, float* pool, const float* ex, const float* eE, const float* ec, void* stream) {
  return tt_block_fwd_impl(p, n_ptrs, Bsz, T, DM, H, FF, eps, scale, pool, ex, eE, ec, dct::ttb::Gather{}, stream);
}

// gx (11 values): X, idx (int64), cursor (int32), stride, n_items, xdst (= ex), Y (int64), ydst (int64),
// step_counter (int32, may be 0), zero (fp32, may be 0), zero_n - see Gather; needs the embedding (ex, eE, ec)
int dct_tt_block_fwd_gx(const uintptr_t* p, int n_ptrs, int Bsz, int T, int DM, int H, int FF, float eps,
                        float scale, float* pool, const float* ex, const float* eE, const float* ec,
                        const uintptr_t* gx, int n_gx, void* stream) {
  if (n_gx != 11 || !ex || !gx[0] || !gx[1] || !gx[2] || gx[5] != (uintptr_t)ex || !gx[6] || !gx[7] ||
      (int64_t)gx[4] <= 0 || (gx[9] && (gx[9] & 15)))
    return (int)hipErrorInvalidValue;
  dct::ttb::Gather g{};
  g.X = (const float*)gx[0]; g.idx = (const int64_t*)gx[1]; g.cursor = (const int*)gx[2]; g.stride = (int)gx[3];
  g.n_items = (int64_t)gx[4]; g.xdst = (float*)gx[5]; g.Y = (const int64_t*)gx[6]; g.ydst = (int64_t*)gx[7];
  g.step_counter = (int*)gx[8]; g.zero = (float*)gx[9]; g.zero_n = (int64_t)gx[10];
  return tt_block_fwd_impl(p, n_ptrs, Bsz, T, DM, H, FF, eps, scale, pool, ex, eE, ec, g, stream);
}

static int tt_block_fwd_impl(const uintptr_t* p, int n_ptrs, int Bsz, int T, int DM, int H, int FF, float eps,
                             float scale, float* pool, const float* ex, const float* eE, const float* ec,
                             const dct::ttb::Gather& gx, void* stream) {
  using namespace dct::ttb;
  if ((n_ptrs != 27 && n_ptrs != 28) || T != dct::ttb::T || DM != dct::ttb::DM || H != NH || FF != dct::ttb::FF || Bsz <= 0)
    return (int)hipErrorInvalidValue;
  // inference (no saved tensors) when a1 (p[13]) is null: then only inputs, weights and out are used
  const bool save = p[13] != 0;
  uintptr_t any = 0;
  for (int i = 0; i < 27; ++i) {
    const bool needed = (i < 13 || (i == 25 && !pool) || save) && i != 24 && i != 23 && i != 16 && !(i == 25 && pool) &&
                        !(i == 0 && ex);
    if (needed && !p[i]) return (int)hipErrorInvalidValue;
    any |= p[i];
  }
  if (any & 15) return (int)hipErrorInvalidValue;  // 16-byte vector loads / stores everywhere
  Args a;
  a.h = (const float*)p[0]; a.ln1_w = (const float*)p[1]; a.ln1_b = (const float*)p[2];
  a.wqkv = (const uint16_t*)p[3]; a.bqkv = (const float*)p[4];
  a.wo = (const uint16_t*)p[5]; a.bo = (const float*)p[6];
  a.ln2_w = (const float*)p[7]; a.ln2_b = (const float*)p[8];
  a.w1 = (const uint16_t*)p[9]; a.b1 = (const float*)p[10];
  a.w2 = (const uint16_t*)p[11]; a.b2 = (const float*)p[12];
  a.a1 = (uint16_t*)p[13]; a.mean1 = (float*)p[14]; a.rstd1 = (float*)p[15];
  a.qkv = (uint16_t*)p[16]; a.o = (uint16_t*)p[17]; a.lse = (float*)p[18];
  a.h1 = (float*)p[19]; a.a2 = (uint16_t*)p[20]; a.mean2 = (float*)p[21]; a.rstd2 = (float*)p[22];
  a.f = (uint16_t*)p[23]; a.pre = (uint16_t*)p[24]; a.out = (float*)p[25]; a.wT = (uint16_t*)p[26];
  a.prof = n_ptrs == 28 ? (uint64_t*)p[27] : nullptr;
  a.pool = pool;
  if (pool && (((uintptr_t)pool) & 15)) return (int)hipErrorInvalidValue;
  if (ex && (!eE || !ec || ((((uintptr_t)eE) | ((uintptr_t)ec)) & 15))) return (int)hipErrorInvalidValue;
  a.em = Embed{ex, eE, ec};
  a.gx = gx;
  a.save = save ? 1 : 0;
  a.B = Bsz; a.eps = eps; a.scale = scale;
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)tt_block_fwd_kernel,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  hipLaunchKernelGGL(tt_block_fwd_kernel, dim3(Bsz), dim3(256), LDS_BYTES, reinterpret_cast<hipStream_t>(stream), a);
  return (int)hipGetLastError();
}

int dct_tt_block_fwd(const uintptr_t* p, int n_ptrs, int Bsz, int T, int DM, int H, int FF, float eps, float scale,
                     void* stream) {
  return dct_tt_block_fwd_ex(p, n_ptrs, Bsz, T, DM, H, FF, eps, scale, nullptr, nullptr, nullptr, nullptr, stream);
}

// ptrs (22, in order): dout, h, mean1, rstd1, ln1_w, qkv, o, lse, h1, mean2, rstd2, ln2_w, pre, wT,
//   dpre, dh1_16, dqkv, dh, dh16, dln1_w, dln1_b, dln2_w, dln2_b  (23 with the last four)
// dpool (optional): the head's gradient of the last block's token mean instead of dout (p[0] may then be
// null); bf16(dout) is then written to dout16 ([B*T][DM]) for the W2 gradient GEMM
// ex / eE / ec (optional): the block input is embedded from the features (h p[1] and dh16 p[18] may be null)
// lnrep / ticket (optional, together): zeroed [16][4][DM] floats + a zeroed uint32 the launch leaves zeroed
// (LayerNorm gradients through replicas, see LN_REP); null: direct atomics
// a1 / wqkv / bqkv (optional): with qkv (p[5]) null, q / k / v are recomputed from a1 [B*T][DM] bf16, the
// bf16 Wqkv [3DM][DM] and bqkv fp32, bit-identical to the forward's
int dct_tt_block_bwd_ex(const uintptr_t* p, int n_ptrs, int Bsz, int T, int DM, int H, int FF, float scale,
                        const float* dpool, uint16_t* dout16, const float* ex, const float* eE, const float* ec,
                        float* lnrep, unsigned* ticket, const uint16_t* a1, const uint16_t* wqkv,
                        const float* bqkv, void* stream) {
  using namespace dct::ttb;
  // 23 (+1 prof) pointers; 26 (+1 prof): + a2, w1 (bf16 [FF][DM]), b1 - with pre (p[12]) null the
  // kernel recomputes the pre-activation from them
  const bool ext = n_ptrs == 26 || n_ptrs == 27;
  if ((n_ptrs != 23 && n_ptrs != 24 && !ext) || T != dct::ttb::T || DM != dct::ttb::DM || H != NH ||
      FF != dct::ttb::FF || Bsz <= 0)
    return (int)hipErrorInvalidValue;
  const bool recomp = ext && p[12] == 0;
  uintptr_t any = 0;
  for (int i = 0; i < (ext ? 26 : 23); ++i) {
    if (!p[i] && !(i == 12 && recomp) && !(i >= 23 && !recomp) && !(i == 0 && dpool) && !((i == 1 || i == 18) && ex) &&
        !(i == 14 && recomp) && !(i == 5 && a1))
      return (int)hipErrorInvalidValue;
    if (i < 19 || i >= 23) any |= p[i];
  }
  if (any & 15) return (int)hipErrorInvalidValue;
  BwdArgs a;
  a.dout = (const float*)p[0]; a.h = (const float*)p[1]; a.mean1 = (const float*)p[2]; a.rstd1 = (const float*)p[3];
  a.ln1_w = (const float*)p[4]; a.qkv = (const uint16_t*)p[5]; a.o = (const uint16_t*)p[6]; a.lse = (const float*)p[7];
  a.h1 = (const float*)p[8]; a.mean2 = (const float*)p[9]; a.rstd2 = (const float*)p[10]; a.ln2_w = (const float*)p[11];
  a.pre = (const uint16_t*)p[12]; a.wT = (const uint16_t*)p[13];
  a.dpre = (uint16_t*)p[14]; a.dh1_16 = (uint16_t*)p[15]; a.dqkv = (uint16_t*)p[16]; a.dh = (float*)p[17];
  a.dh16 = (uint16_t*)p[18];
  a.dln1_w = (float*)p[19]; a.dln1_b = (float*)p[20]; a.dln2_w = (float*)p[21]; a.dln2_b = (float*)p[22];
  a.a2 = ext ? (const uint16_t*)p[23] : nullptr;
  a.w1 = ext ? (const uint16_t*)p[24] : nullptr;
  a.b1 = ext ? (const float*)p[25] : nullptr;
  a.prof = n_ptrs == 24 ? (uint64_t*)p[23] : (n_ptrs == 27 ? (uint64_t*)p[26] : nullptr);
  a.scale = scale;
  if (dpool && (!dout16 || ((((uintptr_t)dpool) | ((uintptr_t)dout16)) & 15))) return (int)hipErrorInvalidValue;
  a.dpool = dpool;
  a.dout16 = dpool ? dout16 : nullptr;
  if (ex && (!eE || !ec || ((((uintptr_t)eE) | ((uintptr_t)ec)) & 15))) return (int)hipErrorInvalidValue;
  a.em = Embed{ex, eE, ec};
  if ((lnrep == nullptr) != (ticket == nullptr)) return (int)hipErrorInvalidValue;
  a.lnrep = lnrep;
  a.ticket = ticket;
  if (!p[5] && (!a1 || !wqkv || !bqkv || ((((uintptr_t)a1) | ((uintptr_t)wqkv)) & 15))) return (int)hipErrorInvalidValue;
  a.a1 = p[5] ? nullptr : a1;
  a.wqkv = p[5] ? nullptr : wqkv;
  a.bqkv = p[5] ? nullptr : bqkv;
  static bool attr = false;
  if (!attr) {
    for (const void* k : {(const void*)tt_block_bwd_kernel<false>, (const void*)tt_block_bwd_kernel<true>}) {
      const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, BWD_LDS);
      if (e != hipSuccess) return (int)e;
    }
    attr = true;
  }
  if (recomp)
    hipLaunchKernelGGL(tt_block_bwd_kernel<true>, dim3(Bsz), dim3(256), BWD_LDS, reinterpret_cast<hipStream_t>(stream), a);
  else
    hipLaunchKernelGGL(tt_block_bwd_kernel<false>, dim3(Bsz), dim3(256), BWD_LDS, reinterpret_cast<hipStream_t>(stream), a);
  return (int)hipGetLastError();
}

int dct_tt_block_bwd(const uintptr_t* p, int n_ptrs, int Bsz, int T, int DM, int H, int FF, float scale,
                     void* stream) {
  return dct_tt_block_bwd_ex(p, n_ptrs, Bsz, T, DM, H, FF, scale, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                             nullptr, nullptr, nullptr, nullptr, stream);
}

}  // extern "C"
