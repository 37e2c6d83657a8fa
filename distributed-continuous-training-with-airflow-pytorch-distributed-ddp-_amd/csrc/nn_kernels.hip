// Memory-bound NN kernels for gfx950: fused loss fwd+bwd, bias+activation backward with the
// bias-gradient column reduction, LayerNorm fwd/bwd, and the on-device batch gather.
// All of them vectorise bf16 I/O to 16-B per lane where the layout allows (CDNA guide G13)
// and reduce per block before one atomic per (block, column) (G12).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdint.h>

#include "dct_common.h"
#include "kernels.h"

namespace dct {

__device__ __forceinline__ float gelu_grad(float z) { return gelu_grad_f(z); }

__device__ __forceinline__ float ld_any(const void* p, size_t i, int bf16) {
  return bf16 ? bf16_to_f32(reinterpret_cast<const uint16_t*>(p)[i]) : reinterpret_cast<const float*>(p)[i];
}
__device__ __forceinline__ void st_any(void* p, size_t i, float v, int bf16) {
  if (bf16) reinterpret_cast<uint16_t*>(p)[i] = f32_to_bf16(v);
  else reinterpret_cast<float*>(p)[i] = v;
}

// ------------------------------------------------------------------------------- loss
__global__ __launch_bounds__(256) void loss_kernel(const void* logits, int lbf16, const int* labels, void* dlogits,
                                                   float* loss_sum, float* correct_sum, int M, int C,
                                                   float grad_scale, int loss_kind, float loss_scale) {
  __shared__ float red[2][4];
  float l_acc = 0.f, c_acc = 0.f;
  for (int row = blockIdx.x * blockDim.x + threadIdx.x; row < M; row += gridDim.x * blockDim.x) {
    const size_t base = (size_t)row * C;
    const int y = labels[row];
    if (C <= 8) {
      // heads of <= 8 classes: the row's logits are loaded once, unconditionally (class slots past C
      // re-read column C-1 and are masked), then every pass runs from registers; the generic loop below
      // re-reads memory per pass and its guarded loads drain the load queue (s_waitcnt vmcnt(0)).
      float z[8];
      if (lbf16) {
        const uint16_t* lg = reinterpret_cast<const uint16_t*>(logits) + base;
#pragma unroll
        for (int c = 0; c < 8; ++c) z[c] = bf16_to_f32(lg[c < C ? c : C - 1]);
      } else {
        const float* lg = reinterpret_cast<const float*>(logits) + base;
#pragma unroll
        for (int c = 0; c < 8; ++c) z[c] = lg[c < C ? c : C - 1];
      }
      float mx = z[0], zy = z[0];
      int am = 0;
#pragma unroll
      for (int c = 1; c < 8; ++c)
        if (c < C && z[c] > mx) { mx = z[c]; am = c; }
#pragma unroll
      for (int c = 1; c < 8; ++c)
        if (c == y) zy = z[c];
      c_acc += (am == y) ? 1.f : 0.f;
      if (loss_kind == 0) {
        float e[8], s = 0.f;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          e[c] = c < C ? __expf(z[c] - mx) : 0.f;
          s += e[c];
        }
        l_acc += mx + __logf(s) - zy;
        if (dlogits) {
          const float rs = 1.f / s;
#pragma unroll
          for (int c = 0; c < 8; ++c)
            if (c < C) st_any(dlogits, base + c, (e[c] * rs - (c == y ? 1.f : 0.f)) * grad_scale, lbf16);
        }
      } else {
        float acc = 0.f;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          if (c < C) {
            const float d = z[c] - (c == y ? 1.f : 0.f);
            acc += d * d;
            if (dlogits) st_any(dlogits, base + c, 2.f * d * grad_scale / (float)C, lbf16);
          }
        }
        l_acc += acc / (float)C;
      }
      continue;
    }
    float mx = -3.402823466e+38f;
    int am = 0;
    for (int c = 0; c < C; ++c) {
      const float z = ld_any(logits, base + c, lbf16);
      if (z > mx) { mx = z; am = c; }
    }
    c_acc += (am == y) ? 1.f : 0.f;
    if (loss_kind == 0) {
      float s = 0.f;
      for (int c = 0; c < C; ++c) s += __expf(ld_any(logits, base + c, lbf16) - mx);
      const float lse = mx + __logf(s);
      l_acc += lse - ld_any(logits, base + y, lbf16);
      if (dlogits) {
        const float rs = 1.f / s;
        for (int c = 0; c < C; ++c) {
          const float pr = __expf(ld_any(logits, base + c, lbf16) - mx) * rs;
          st_any(dlogits, base + c, (pr - (c == y ? 1.f : 0.f)) * grad_scale, lbf16);
        }
      }
    } else {
      float acc = 0.f;
      for (int c = 0; c < C; ++c) {
        const float d = ld_any(logits, base + c, lbf16) - (c == y ? 1.f : 0.f);
        acc += d * d;
        if (dlogits) st_any(dlogits, base + c, 2.f * d * grad_scale / (float)C, lbf16);
      }
      l_acc += acc / (float)C;
    }
  }
  l_acc = wave_sum(l_acc);
  c_acc = wave_sum(c_acc);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { red[0][w] = l_acc; red[1][w] = c_acc; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = 0.f, b = 0.f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) { a += red[0][i]; b += red[1][i]; }
    if (loss_sum) atomicAdd(loss_sum, a * loss_scale);
    if (correct_sum) atomicAdd(correct_sum, b);
  }
}

// ------------------------------------------------------------------------ bias+act bwd
// block: 64 column-chunks (8 columns each) x 4 row lanes
template <bool VEC>
__global__ __launch_bounds__(256) void bias_act_bwd_kernel(const uint16_t* dY, const uint16_t* aux, uint16_t* dZ,
                                                           float* dbias, int M, int N, int ldy, int act,
                                                           int accumulate_bias) {
  __shared__ float part[4][64 * 8];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int cc = blockIdx.x * 64 + tx;
  const int c0 = cc * 8;
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  if (c0 < N) {
#pragma unroll 4
    for (int r = blockIdx.y * 4 + ty; r < M; r += gridDim.y * 4) {
      const size_t o = (size_t)r * ldy + c0;
      float dy[8], zz[8];
      if (VEC && c0 + 8 <= N) {
        const uint4 v = *reinterpret_cast<const uint4*>(dY + o);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) { dy[2 * j] = bf16_to_f32(w[j] & 0xffff); dy[2 * j + 1] = bf16_to_f32(w[j] >> 16); }
        if (act != ACT_NONE) {
          const uint4 a = *reinterpret_cast<const uint4*>(aux + o);
          const uint32_t u[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
          for (int j = 0; j < 4; ++j) { zz[2 * j] = bf16_to_f32(u[j] & 0xffff); zz[2 * j + 1] = bf16_to_f32(u[j] >> 16); }
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          dy[j] = (c0 + j < N) ? bf16_to_f32(dY[o + j]) : 0.f;
          zz[j] = (act != ACT_NONE && c0 + j < N) ? bf16_to_f32(aux[o + j]) : 0.f;
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float d = dy[j];
        if (act == ACT_RELU) d = zz[j] > 0.f ? d : 0.f;
        else if (act == ACT_GELU) d *= gelu_grad(zz[j]);
        dy[j] = d;
        acc[j] += d;
      }
      if (dZ) {
        if (VEC && c0 + 8 <= N) {
          uint4 v;
          v.x = f32_to_bf16(dy[0]) | ((uint32_t)f32_to_bf16(dy[1]) << 16);
          v.y = f32_to_bf16(dy[2]) | ((uint32_t)f32_to_bf16(dy[3]) << 16);
          v.z = f32_to_bf16(dy[4]) | ((uint32_t)f32_to_bf16(dy[5]) << 16);
          v.w = f32_to_bf16(dy[6]) | ((uint32_t)f32_to_bf16(dy[7]) << 16);
          *reinterpret_cast<uint4*>(dZ + o) = v;
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (c0 + j < N) dZ[o + j] = f32_to_bf16(dy[j]);
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) part[ty][tx * 8 + j] = acc[j];
  __syncthreads();
  if (ty == 0 && dbias && c0 < N) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (c0 + j < N) {
        const float s = part[0][tx * 8 + j] + part[1][tx * 8 + j] + part[2][tx * 8 + j] + part[3][tx * 8 + j];
        if (gridDim.y == 1 && !accumulate_bias) dbias[c0 + j] = s;
        else atomicAdd(&dbias[c0 + j], s);
      }
    }
  }
}

// --------------------------------------------------------------------------- layernorm
// one wave per row, N <= 64 * LN_MAX
constexpr int LN_MAX = 32;

__global__ __launch_bounds__(256) void layernorm_fwd_kernel(const void* x, const float* w, const float* b, void* y,
                                                            float* mean_out, float* rstd_out, int M, int N, float eps,
                                                            int in_bf16, int out_bf16) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= M) return;
  const size_t base = (size_t)row * N;
  float v[LN_MAX];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < LN_MAX; ++j) {
    const int c = lane + j * 64;
    v[j] = (c < N) ? ld_any(x, base + c, in_bf16) : 0.f;
    s += v[j];
  }
  const float mean = wave_sum(s) / (float)N;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < LN_MAX; ++j) {
    const int c = lane + j * 64;
    const float d = (c < N) ? v[j] - mean : 0.f;
    q += d * d;
  }
  const float rstd = rsqrtf(wave_sum(q) / (float)N + eps);
#pragma unroll
  for (int j = 0; j < LN_MAX; ++j) {
    const int c = lane + j * 64;
    if (c < N) st_any(y, base + c, (v[j] - mean) * rstd * (w ? w[c] : 1.f) + (b ? b[c] : 0.f), out_bf16);
  }
  if (lane == 0) {
    if (mean_out) mean_out[row] = mean;
    if (rstd_out) rstd_out[row] = rstd;
  }
}

__global__ __launch_bounds__(256) void layernorm_bwd_kernel(const void* dy, const void* x, const float* w,
                                                            const float* mean, const float* rstd, void* dx, float* dw,
                                                            float* db, int M, int N, int bf16_io) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;
  float dwa[LN_MAX], dba[LN_MAX];
#pragma unroll
  for (int j = 0; j < LN_MAX; ++j) { dwa[j] = 0.f; dba[j] = 0.f; }
  for (int row = blockIdx.x * nw + wave; row < M; row += gridDim.x * nw) {
    const size_t base = (size_t)row * N;
    const float mu = mean[row], rs = rstd[row];
    float g[LN_MAX], xh[LN_MAX];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < LN_MAX; ++j) {
      const int c = lane + j * 64;
      if (c < N) {
        const float d = ld_any(dy, base + c, bf16_io);
        xh[j] = (ld_any(x, base + c, bf16_io) - mu) * rs;
        g[j] = d * (w ? w[c] : 1.f);
        dwa[j] += d * xh[j];
        dba[j] += d;
      } else {
        xh[j] = 0.f;
        g[j] = 0.f;
      }
      s1 += g[j];
      s2 += g[j] * xh[j];
    }
    s1 = wave_sum(s1) / (float)N;
    s2 = wave_sum(s2) / (float)N;
#pragma unroll
    for (int j = 0; j < LN_MAX; ++j) {
      const int c = lane + j * 64;
      if (c < N) st_any(dx, base + c, rs * (g[j] - s1 - xh[j] * s2), bf16_io);
    }
  }
  __shared__ float red[4][64 * 2];
  // reduce dw/db across the block's waves, one atomic per column per block
#pragma unroll
  for (int j = 0; j < LN_MAX; ++j) {
    const int c = lane + j * 64;
    if (j * 64 >= N) break;
    red[wave][lane] = dwa[j];
    red[wave][64 + lane] = dba[j];
    __syncthreads();
    if (wave == 0 && c < N) {
      float a = 0.f, bsum = 0.f;
      for (int i = 0; i < nw; ++i) { a += red[i][lane]; bsum += red[i][64 + lane]; }
      if (dw) atomicAdd(&dw[c], a);
      if (db) atomicAdd(&db[c], bsum);
    }
    __syncthreads();
  }
}

// ----------------------------------------------------------- narrow LayerNorm (N <= 256)
// Transformer widths (d_model 32..256): one lane owns 4 consecutive columns of a row, a row
// takes LPR = pow2(N/4) lanes, a wave holds 64/LPR rows; statistics by xor-shuffles inside
// the lane group.  (The one-wave-per-row kernel above leaves 63/64 lanes idle at N = 64.)
template <int LPR>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = 1; o < LPR; o <<= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ void ld4any(const void* p, size_t i, int bf16, float (&v)[4]) {
  if (bf16) {
    const uint2 u = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(p) + i);
    v[0] = bf16_to_f32(u.x & 0xffff); v[1] = bf16_to_f32(u.x >> 16);
    v[2] = bf16_to_f32(u.y & 0xffff); v[3] = bf16_to_f32(u.y >> 16);
  } else {
    const float4 f = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(p) + i);
    v[0] = f.x; v[1] = f.y; v[2] = f.z; v[3] = f.w;
  }
}
__device__ __forceinline__ void st4any(void* p, size_t i, int bf16, const float (&v)[4]) {
  if (bf16) {
    uint2 u;
    u.x = f32_to_bf16(v[0]) | ((uint32_t)f32_to_bf16(v[1]) << 16);
    u.y = f32_to_bf16(v[2]) | ((uint32_t)f32_to_bf16(v[3]) << 16);
    *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(p) + i) = u;
  } else {
    *reinterpret_cast<float4*>(reinterpret_cast<float*>(p) + i) = make_float4(v[0], v[1], v[2], v[3]);
  }
}

template <int LPR>
__global__ __launch_bounds__(256) void layernorm_fwd_small(const void* x, const float* w, const float* b, void* y,
                                                           float* mean_out, float* rstd_out, int M, int N, float eps,
                                                           int in_bf16, int out_bf16) {
  constexpr int RPW = 64 / LPR;
  const int lane = threadIdx.x & 63, sub = lane / LPR, li = lane % LPR;
  const int c0 = li * 4;
  const bool act = c0 < N;
  float wv[4] = {1.f, 1.f, 1.f, 1.f}, bv[4] = {0.f, 0.f, 0.f, 0.f};
  if (act && w) { const float4 t = *reinterpret_cast<const float4*>(w + c0); wv[0] = t.x; wv[1] = t.y; wv[2] = t.z; wv[3] = t.w; }
  if (act && b) { const float4 t = *reinterpret_cast<const float4*>(b + c0); bv[0] = t.x; bv[1] = t.y; bv[2] = t.z; bv[3] = t.w; }
  const int wave_g = blockIdx.x * 4 + (threadIdx.x >> 6);
  for (int row = wave_g * RPW + sub; row < M; row += gridDim.x * 4 * RPW) {
    const size_t base = (size_t)row * N + c0;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (act) ld4any(x, base, in_bf16, v);
    const float mean = group_sum<LPR>(v[0] + v[1] + v[2] + v[3]) / (float)N;
    float q = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) { const float d = act ? v[e] - mean : 0.f; q += d * d; }
    const float rstd = rsqrtf(group_sum<LPR>(q) / (float)N + eps);
    if (act) {
      float o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (v[e] - mean) * rstd * wv[e] + bv[e];
      st4any(y, base, out_bf16, o);
    }
    if (li == 0) {
      if (mean_out) mean_out[row] = mean;
      if (rstd_out) rstd_out[row] = rstd;
    }
  }
}

// Backward of the narrow LayerNorm, fused for pre-norm residual blocks:
//   dx = rstd * (g - mean(g) - xhat * mean(g * xhat)) [+ dres],  g = dy * w
// with the residual-stream gradient dres folded in (saves the autograd add) and an optional
// bf16 copy of dx (the next GEMM's operand; saves a conversion pass).  dw/db column sums go
// through NSLOT striped slot rows of a persistent workspace (atomics spread over 16x the
// addresses: a 1024-way fan-in on N addresses serialised the old kernel to ~30 us at M=32k);
// layernorm_bwd_fold then adds the slots into dw/db and re-zeroes them.
struct LnBwdArgs {
  const void* dy; const void* x; const float* w; const float* mean; const float* rstd;
  void* dx; uint16_t* dx2; const float* dres; float* dw; float* db; float* ws;
  int M, N, dy_bf16, x_bf16, dx_bf16;
};
constexpr int LN_NSLOT = 16;

template <int LPR>
__global__ __launch_bounds__(256) void layernorm_bwd_small(LnBwdArgs a) {
  constexpr int RPW = 64 / LPR;
  __shared__ float red[2][256 * 4];
  const int N = a.N;
  const int lane = threadIdx.x & 63, sub = lane / LPR, li = lane % LPR;
  const int c0 = li * 4;
  const bool act = c0 < N;
  float wv[4] = {1.f, 1.f, 1.f, 1.f};
  if (act && a.w) { const float4 t = *reinterpret_cast<const float4*>(a.w + c0); wv[0] = t.x; wv[1] = t.y; wv[2] = t.z; wv[3] = t.w; }
  float aw[4] = {0.f, 0.f, 0.f, 0.f}, ab[4] = {0.f, 0.f, 0.f, 0.f};
  const int wave_g = blockIdx.x * 4 + (threadIdx.x >> 6);
  for (int row = wave_g * RPW + sub; row < a.M; row += gridDim.x * 4 * RPW) {
    const size_t base = (size_t)row * N + c0;
    float xv[4] = {0.f, 0.f, 0.f, 0.f}, gv[4] = {0.f, 0.f, 0.f, 0.f}, rv[4] = {0.f, 0.f, 0.f, 0.f};
    if (act) {
      ld4any(a.x, base, a.x_bf16, xv);
      ld4any(a.dy, base, a.dy_bf16, gv);
      if (a.dres) ld4any(a.dres, base, 0, rv);
    }
    const float mean = a.mean[row], rstd = a.rstd[row];
    float xh[4], gw[4], s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      xh[e] = act ? (xv[e] - mean) * rstd : 0.f;
      gw[e] = gv[e] * wv[e];
      s1 += gw[e];
      s2 += gw[e] * xh[e];
      aw[e] += gv[e] * xh[e];
      ab[e] += gv[e];
    }
    s1 = group_sum<LPR>(s1) / (float)N;
    s2 = group_sum<LPR>(s2) / (float)N;
    if (act) {
      float o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = rstd * (gw[e] - s1 - xh[e] * s2) + rv[e];
      st4any(a.dx, base, a.dx_bf16, o);
      if (a.dx2) st4any(a.dx2, base, 1, o);
    }
  }
  if (!a.dw && !a.db) return;
  // column partials: threads with the same li own the same 4 columns
#pragma unroll
  for (int e = 0; e < 4; ++e) { red[0][threadIdx.x * 4 + e] = aw[e]; red[1][threadIdx.x * 4 + e] = ab[e]; }
  __syncthreads();
  float* slot = a.ws + (size_t)(blockIdx.x % LN_NSLOT) * 2 * N;
  for (int cc = threadIdx.x; cc < LPR * 4; cc += blockDim.x) {
    const int l = cc / 4, e = cc % 4;
    if (l * 4 >= N) continue;
    float sw = 0.f, sb = 0.f;
    for (int t = l; t < 256; t += LPR) { sw += red[0][t * 4 + e]; sb += red[1][t * 4 + e]; }
    atomicAdd(slot + cc, sw);
    atomicAdd(slot + N + cc, sb);
  }
}

// folds the slot rows into dw/db (+=) and re-zeroes them (one block, after the row kernel).
// A last-block ticket inside the row kernel was tried: 1024 serialised ticket atomics plus an
// agent-scope release fence (L2 write-back) per block made it 3x slower than this extra launch.
__global__ __launch_bounds__(256) void layernorm_bwd_fold(float* ws, float* dw, float* db, int N) {
  for (int cc = threadIdx.x; cc < 2 * N; cc += blockDim.x) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < LN_NSLOT; ++k) {
      float* p = ws + (size_t)k * 2 * N + cc;
      s += *p;
      *p = 0.f;
    }
    float* dst = cc < N ? dw : db;
    if (dst) dst[cc < N ? cc : cc - N] += s;
  }
}

// ------------------------------------------------------------------------------ gather
__global__ __launch_bounds__(256) void gather_rows16_kernel(const uint4* src, const int* idx, uint4* dst,
                                                            int64_t n_rows, int row_vec) {
  const int64_t total = n_rows * row_vec;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / row_vec;
    const int c = (int)(e - r * row_vec);
    dst[e] = src[(int64_t)idx[r] * row_vec + c];
  }
}
__global__ __launch_bounds__(256) void gather_rows4_kernel(const uint32_t* src, const int* idx, uint32_t* dst,
                                                           int64_t n_rows, int row_words) {
  const int64_t total = n_rows * row_words;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / row_words;
    const int c = (int)(e - r * row_words);
    dst[e] = src[(int64_t)idx[r] * row_words + c];
  }
}

}  // namespace dct

static inline int grid_cap(int64_t work, int block, int cap = 2048) {
  int64_t g = (work + block - 1) / block;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (int)g;
}

extern "C" {

int dct_loss_fwd_bwd_ex(const void* logits, int logits_bf16, const int* labels, void* dlogits, float* loss_sum,
                        float* correct_sum, int M, int C, float grad_scale, int loss_kind, float loss_scale,
                        void* stream) {
  if (M <= 0) return 0;
  hipLaunchKernelGGL(dct::loss_kernel, dim3(grid_cap(M, 256, 1024)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     logits, logits_bf16, labels, dlogits, loss_sum, correct_sum, M, C, grad_scale, loss_kind,
                     loss_scale);
  return (int)hipGetLastError();
}

int dct_loss_fwd_bwd(const void* logits, int logits_bf16, const int* labels, void* dlogits, float* loss_sum,
                     float* correct_sum, int M, int C, float grad_scale, int loss_kind, void* stream) {
  return dct_loss_fwd_bwd_ex(logits, logits_bf16, labels, dlogits, loss_sum, correct_sum, M, C, grad_scale, loss_kind,
                             1.0f, stream);
}

int dct_bias_act_bwd(const void* dY, const void* act_aux, uint16_t* dZ, float* dbias, int M, int N, int ldy, int act,
                     int accumulate_bias, void* stream) {
  if (M <= 0 || N <= 0) return 0;
  const int ncc = (N + 7) / 8;
  // row blocks of >= 64 rows: few float atomics per column (a 512-way atomicAdd fan-in on the
  // same 1024 addresses serialised this kernel to ~100 us at M = 4096), enough blocks to fill
  // the chip (the row loop keeps 4 rows of loads in flight per thread)
  dim3 grid((ncc + 63) / 64, (unsigned)grid_cap((M + 63) / 64, 1, std::max(64, 512 / std::max(1, (ncc + 63) / 64))));
  const bool vec = (N % 8 == 0) && (ldy % 8 == 0) && ((((uintptr_t)dY) | ((uintptr_t)act_aux) | ((uintptr_t)dZ)) & 15) == 0;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (vec)
    hipLaunchKernelGGL(dct::bias_act_bwd_kernel<true>, grid, dim3(256), 0, st, (const uint16_t*)dY,
                       (const uint16_t*)act_aux, dZ, dbias, M, N, ldy, act, accumulate_bias);
  else
    hipLaunchKernelGGL(dct::bias_act_bwd_kernel<false>, grid, dim3(256), 0, st, (const uint16_t*)dY,
                       (const uint16_t*)act_aux, dZ, dbias, M, N, ldy, act, accumulate_bias);
  return (int)hipGetLastError();
}

static int ln_lpr(int N, const void* a, const void* b2, const void* c) {
  if (N % 4 || N > 256 || ((((uintptr_t)a) | ((uintptr_t)b2) | ((uintptr_t)c)) & 15)) return 0;
  int l = 1;
  while (l * 4 < N) l <<= 1;
  return l;
}

int dct_layernorm_fwd(const void* x, const float* w, const float* b, void* y, float* mean, float* rstd, int M, int N,
                      float eps, int in_bf16, int out_bf16, void* stream) {
  if (N > 64 * dct::LN_MAX) return (int)hipErrorInvalidValue;
  if (M <= 0) return 0;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (const int lpr = ln_lpr(N, x, y, w)) {
    const int rows_per_block = 4 * (64 / lpr);
    const int grid = grid_cap((M + rows_per_block - 1) / rows_per_block, 1, 4096);
#define LNF(L) hipLaunchKernelGGL(dct::layernorm_fwd_small<L>, dim3(grid), dim3(256), 0, st, x, w, b, y, mean, rstd, M, N, eps, in_bf16, out_bf16)
    switch (lpr) { case 1: LNF(1); break; case 2: LNF(2); break; case 4: LNF(4); break; case 8: LNF(8); break;
                   case 16: LNF(16); break; case 32: LNF(32); break; default: LNF(64); }
#undef LNF
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(dct::layernorm_fwd_kernel, dim3((M + 3) / 4), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     x, w, b, y, mean, rstd, M, N, eps, in_bf16, out_bf16);
  return (int)hipGetLastError();
}

int dct_layernorm_bwd_ex(const void* dy, int dy_bf16, const void* x, int x_bf16, const float* w, const float* mean,
                         const float* rstd, void* dx, int dx_bf16, uint16_t* dx2, const float* dres, float* dw,
                         float* db, float* ws, int M, int N, void* stream) {
  if (M <= 0) return 0;
  const int lpr = ln_lpr(N, dy, x, dx);
  if (!lpr || !ws || (dres && (((uintptr_t)dres) & 15)) || (dx2 && (((uintptr_t)dx2) & 7)))
    return (int)hipErrorInvalidValue;
  dct::LnBwdArgs a{dy, x, w, mean, rstd, dx, dx2, dres, dw, db, ws, M, N, dy_bf16, x_bf16, dx_bf16};
  const int rows_per_block = 4 * (64 / lpr);
  const int grid = grid_cap((M + rows_per_block - 1) / rows_per_block, 1, 1024);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
#define LNB(L) hipLaunchKernelGGL(dct::layernorm_bwd_small<L>, dim3(grid), dim3(256), 0, st, a)
  switch (lpr) { case 1: LNB(1); break; case 2: LNB(2); break; case 4: LNB(4); break; case 8: LNB(8); break;
                 case 16: LNB(16); break; case 32: LNB(32); break; default: LNB(64); }
#undef LNB
  if (dw || db) hipLaunchKernelGGL(dct::layernorm_bwd_fold, dim3(1), dim3(256), 0, st, ws, dw, db, N);
  return (int)hipGetLastError();
}

int dct_layernorm_bwd_ws_floats(int N) { return dct::LN_NSLOT * 2 * N; }

int dct_layernorm_bwd(const void* dy, const void* x, const float* w, const float* mean, const float* rstd, void* dx,
                      float* dw, float* db, int M, int N, int bf16_io, void* stream) {
  if (N > 64 * dct::LN_MAX) return (int)hipErrorInvalidValue;
  if (M <= 0) return 0;
  // generic one-wave-per-row kernel (any N <= 64 * LN_MAX, any alignment); the narrow fused
  // path needs the caller's slot workspace -> dct_layernorm_bwd_ex
  hipLaunchKernelGGL(dct::layernorm_bwd_kernel, dim3(grid_cap((M + 3) / 4, 1, 1024)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), dy, x, w, mean, rstd, dx, dw, db, M, N, bf16_io);
  return (int)hipGetLastError();
}

int dct_gather_rows(const void* src, const int* idx, void* dst, int64_t n_rows, int row_bytes, void* stream) {
  if (n_rows <= 0) return 0;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (row_bytes % 16 == 0 && ((((uintptr_t)src) | ((uintptr_t)dst)) & 15) == 0) {
    const int rv = row_bytes / 16;
    hipLaunchKernelGGL(dct::gather_rows16_kernel, dim3(grid_cap(n_rows * rv, 256)), dim3(256), 0, st,
                       (const uint4*)src, idx, (uint4*)dst, n_rows, rv);
  } else if (row_bytes % 4 == 0) {
    const int rw = row_bytes / 4;
    hipLaunchKernelGGL(dct::gather_rows4_kernel, dim3(grid_cap(n_rows * rw, 256)), dim3(256), 0, st,
                       (const uint32_t*)src, idx, (uint32_t*)dst, n_rows, rw);
  } else {
    return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

}  // extern "C"
