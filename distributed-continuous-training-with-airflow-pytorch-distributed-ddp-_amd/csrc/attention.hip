// Feature-token attention for the TabTransformer config (BASELINE.json config 5).
//
// Tokens are the tabular features (T <= 256), so one (batch, head) pair's
// whole K/V (T x D bf16, <= 32 KB each) fits in LDS: one workgroup per (b, h), one query row
// per thread, online softmax in registers, K/V rows read as LDS broadcasts (every lane of a
// wave reads the same key row -> one ds_read per 16 B per wave).  No sequence/context
// parallelism is needed at these lengths.
// Backward recomputes P from Q, K and the forward's log-sum-exp: phase A (thread = query)
// produces dQ, phase B (thread = key) produces dK and dV, so no atomics are needed.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "dct_common.h"
#include "kernels.h"

namespace dct {

constexpr int ATT_MAXD = 64;
constexpr int ATT_NT = 256;

__device__ __forceinline__ void load_row(const uint16_t* s, float* r, int D) {
#pragma unroll
  for (int d = 0; d < ATT_MAXD; ++d) r[d] = (d < D) ? bf16_to_f32(s[d]) : 0.f;
}

// LDS tile [T][D] bf16 <- global rows (b, t, h) with row stride ld
__device__ __forceinline__ void stage_tile(uint16_t* dst, const uint16_t* src, int T, int D, int ld) {
  for (int e = threadIdx.x; e < T * D; e += blockDim.x) {
    const int t = e / D, d = e - t * D;
    dst[e] = src[(size_t)t * ld + d];
  }
}

__global__ __launch_bounds__(ATT_NT) void attn_fwd_kernel(const uint16_t* q, const uint16_t* k, const uint16_t* v,
                                                          uint16_t* o, float* lse, int H, int T, int D, int ldq,
                                                          int ldo, float scale) {
  extern __shared__ __attribute__((aligned(16))) uint16_t sm[];
  uint16_t* Ks = sm;
  uint16_t* Vs = sm + T * D;
  const int bh = blockIdx.x;
  const int b = bh / H, h = bh % H;
  const size_t row0 = (size_t)b * T;
  stage_tile(Ks, k + row0 * ldq + h * D, T, D, ldq);
  stage_tile(Vs, v + row0 * ldq + h * D, T, D, ldq);
  __syncthreads();
  for (int i = threadIdx.x; i < T; i += blockDim.x) {
    float qr[ATT_MAXD], acc[ATT_MAXD];
    load_row(q + (row0 + i) * ldq + h * D, qr, D);
#pragma unroll
    for (int d = 0; d < ATT_MAXD; ++d) { qr[d] *= scale; acc[d] = 0.f; }
    float m = -3.402823466e+38f, l = 0.f;
    for (int j = 0; j < T; ++j) {
      const uint16_t* kr = Ks + j * D;
      float s = 0.f;
#pragma unroll
      for (int d = 0; d < ATT_MAXD; ++d)
        if (d < D) s += qr[d] * bf16_to_f32(kr[d]);
      const float mn = fmaxf(m, s);
      const float alpha = __expf(m - mn);
      const float p = __expf(s - mn);
      l = l * alpha + p;
      const uint16_t* vr = Vs + j * D;
#pragma unroll
      for (int d = 0; d < ATT_MAXD; ++d)
        if (d < D) acc[d] = acc[d] * alpha + p * bf16_to_f32(vr[d]);
      m = mn;
    }
    const float inv = 1.f / l;
    uint16_t* orow = o + (row0 + i) * ldo + h * D;
#pragma unroll
    for (int d = 0; d < ATT_MAXD; ++d)
      if (d < D) orow[d] = f32_to_bf16(acc[d] * inv);
    lse[(size_t)bh * T + i] = m + __logf(l);
  }
}

__global__ __launch_bounds__(ATT_NT) void attn_bwd_kernel(const uint16_t* q, const uint16_t* k, const uint16_t* v,
                                                          const uint16_t* o, const uint16_t* dout, const float* lse,
                                                          uint16_t* dq, uint16_t* dk, uint16_t* dv, int H, int T, int D,
                                                          int ldq, int ldo, float scale) {
  extern __shared__ __attribute__((aligned(16))) uint16_t sm[];
  uint16_t* Qs = sm;
  uint16_t* Ks = Qs + T * D;
  uint16_t* Vs = Ks + T * D;
  uint16_t* dOs = Vs + T * D;
  float* Ls = reinterpret_cast<float*>(dOs + T * D + ((4 * T * D) & 1));
  float* Dl = Ls + T;  // delta_i = rowsum(dO_i * O_i)
  const int bh = blockIdx.x;
  const int b = bh / H, h = bh % H;
  const size_t row0 = (size_t)b * T;
  stage_tile(Qs, q + row0 * ldq + h * D, T, D, ldq);
  stage_tile(Ks, k + row0 * ldq + h * D, T, D, ldq);
  stage_tile(Vs, v + row0 * ldq + h * D, T, D, ldq);
  stage_tile(dOs, dout + row0 * ldo + h * D, T, D, ldo);
  for (int i = threadIdx.x; i < T; i += blockDim.x) {
    Ls[i] = lse[(size_t)bh * T + i];
    float dl = 0.f;
    const uint16_t* orow = o + (row0 + i) * ldo + h * D;
    const uint16_t* drow = dout + (row0 + i) * ldo + h * D;
    for (int d = 0; d < D; ++d) dl += bf16_to_f32(orow[d]) * bf16_to_f32(drow[d]);
    Dl[i] = dl;
  }
  __syncthreads();
  // phase A: dQ_i = scale * sum_j dS_ij K_j
  for (int i = threadIdx.x; i < T; i += blockDim.x) {
    float qr[ATT_MAXD], dor[ATT_MAXD], acc[ATT_MAXD];
    load_row(Qs + i * D, qr, D);
    load_row(dOs + i * D, dor, D);
#pragma unroll
    for (int d = 0; d < ATT_MAXD; ++d) acc[d] = 0.f;
    const float li = Ls[i], di = Dl[i];
    for (int j = 0; j < T; ++j) {
      const uint16_t* kr = Ks + j * D;
      const uint16_t* vr = Vs + j * D;
      float s = 0.f, dp = 0.f;
#pragma unroll
      for (int d = 0; d < ATT_MAXD; ++d)
        if (d < D) { s += qr[d] * bf16_to_f32(kr[d]); dp += dor[d] * bf16_to_f32(vr[d]); }
      const float p = __expf(s * scale - li);
      const float ds = p * (dp - di);
#pragma unroll
      for (int d = 0; d < ATT_MAXD; ++d)
        if (d < D) acc[d] += ds * bf16_to_f32(kr[d]);
    }
    uint16_t* out = dq + (row0 + i) * ldq + h * D;
#pragma unroll
    for (int d = 0; d < ATT_MAXD; ++d)
      if (d < D) out[d] = f32_to_bf16(acc[d] * scale);
  }
  // phase B: dK_j = scale * sum_i dS_ij Q_i ; dV_j = sum_i P_ij dO_i
  for (int j = threadIdx.x; j < T; j += blockDim.x) {
    float kr[ATT_MAXD], vr[ATT_MAXD], ak[ATT_MAXD], av[ATT_MAXD];
    load_row(Ks + j * D, kr, D);
    load_row(Vs + j * D, vr, D);
#pragma unroll
    for (int d = 0; d < ATT_MAXD; ++d) { ak[d] = 0.f; av[d] = 0.f; }
    for (int i = 0; i < T; ++i) {
      const uint16_t* qr = Qs + i * D;
      const uint16_t* dor = dOs + i * D;
      float s = 0.f, dp = 0.f;
#pragma unroll
      for (int d = 0; d < ATT_MAXD; ++d)
        if (d < D) { s += bf16_to_f32(qr[d]) * kr[d]; dp += bf16_to_f32(dor[d]) * vr[d]; }
      const float p = __expf(s * scale - Ls[i]);
      const float ds = p * (dp - Dl[i]);
#pragma unroll
      for (int d = 0; d < ATT_MAXD; ++d)
        if (d < D) { ak[d] += ds * bf16_to_f32(qr[d]); av[d] += p * bf16_to_f32(dor[d]); }
    }
    uint16_t* ko = dk + (row0 + j) * ldq + h * D;
    uint16_t* vo = dv + (row0 + j) * ldq + h * D;
#pragma unroll
    for (int d = 0; d < ATT_MAXD; ++d)
      if (d < D) { ko[d] = f32_to_bf16(ak[d] * scale); vo[d] = f32_to_bf16(av[d]); }
  }
}


// ============================================================ MFMA path (T, D multiples of 16)
// One wave per (batch, head), 4 waves per workgroup; T <= 64 tokens, D <= 64.  All products
// are v_mfma_f32_16x16x16_bf16 (A: row = lane&15, k = 4*(lane>>4)+j; B: col = lane&15,
// k = 4*(lane>>4)+j; C: col = lane&15, row = 4*(lane>>4)+r).
// Forward computes S^T = K Q^T ("swapped QK^T"): its accumulator holds, per lane, 4 keys of one
// query, which is exactly the A-operand layout of P for O = P V - no LDS round trip, no
// transpose; the softmax row reduction is in-register + two xor-shuffles (lanes q, q+16, q+32, q+48).
// Backward recomputes P twice: in S layout (-> dV = P^T dO, dK = dS^T Q) and in S^T layout
// (-> dQ = dS K), each product again consuming accumulators as operands directly.
typedef short bf16x4v __attribute__((ext_vector_type(4)));
typedef float f32x4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4v mfma16(bf16x4v a, bf16x4v b, f32x4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
}
// 4 consecutive bf16 of a row (8-byte load)
__device__ __forceinline__ bf16x4v ld4(const uint16_t* p) { return *reinterpret_cast<const bf16x4v*>(p); }
// 4 bf16 down a column (rows r0..r0+3, stride ld)
__device__ __forceinline__ bf16x4v ld4col(const uint16_t* p, int ld) {
  bf16x4v r;
  r[0] = (short)p[0]; r[1] = (short)p[ld]; r[2] = (short)p[2 * ld]; r[3] = (short)p[3 * ld];
  return r;
}
__device__ __forceinline__ bf16x4v pack4(f32x4v v) {
  bf16x4v r;
  r[0] = (short)f32_to_bf16(v[0]); r[1] = (short)f32_to_bf16(v[1]);
  r[2] = (short)f32_to_bf16(v[2]); r[3] = (short)f32_to_bf16(v[3]);
  return r;
}
__device__ __forceinline__ float xsum16(float v) {  // sum over lanes l, l^16, l^32, l^48
  v += __shfl_xor(v, 16);
  v += __shfl_xor(v, 32);
  return v;
}
__device__ __forceinline__ float xmax16(float v) {
  v = fmaxf(v, __shfl_xor(v, 16));
  v = fmaxf(v, __shfl_xor(v, 32));
  return v;
}

template <int TT, int DT>
__global__ __launch_bounds__(256) void attn_fwd_mfma(const uint16_t* q, const uint16_t* k, const uint16_t* v,
                                                     uint16_t* o, float* lse, int BH, int H, int ldq, int ldo,
                                                     float scale) {
  constexpr int T = TT * 16, D = DT * 16;
  const int lane = threadIdx.x & 63;
  const int bh = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (bh >= BH) return;
  const int b = bh / H, h = bh - b * H;
  const size_t row0 = (size_t)b * T;
  const int c = lane & 15, g = lane >> 4;
  const uint16_t* qb = q + row0 * ldq + h * D;
  const uint16_t* kb = k + row0 * ldq + h * D;
  const uint16_t* vb = v + row0 * ldq + h * D;
  // S^T[key tile i][query tile j] = sum_kd K[i] . Q[j]^T
  f32x4v st[TT][TT];
#pragma unroll
  for (int i = 0; i < TT; ++i)
#pragma unroll
    for (int j = 0; j < TT; ++j) st[i][j] = (f32x4v){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kd = 0; kd < DT; ++kd) {
    bf16x4v kf[TT], qf[TT];
#pragma unroll
    for (int i = 0; i < TT; ++i) kf[i] = ld4(kb + (size_t)(16 * i + c) * ldq + 16 * kd + 4 * g);
#pragma unroll
    for (int j = 0; j < TT; ++j) qf[j] = ld4(qb + (size_t)(16 * j + c) * ldq + 16 * kd + 4 * g);
#pragma unroll
    for (int i = 0; i < TT; ++i)
#pragma unroll
      for (int j = 0; j < TT; ++j) st[i][j] = mfma16(kf[i], qf[j], st[i][j]);
  }
  // softmax over keys for query 16j + c: this lane holds keys 16i + 4g + r
  bf16x4v pf[TT][TT];  // [query tile j][key k-step i]
  float lsev[TT];
#pragma unroll
  for (int j = 0; j < TT; ++j) {
    float m = -3.402823466e+38f;
#pragma unroll
    for (int i = 0; i < TT; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) m = fmaxf(m, st[i][j][r]);
    m = xmax16(m) * scale;
    float l = 0.f;
#pragma unroll
    for (int i = 0; i < TT; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float e = __expf(st[i][j][r] * scale - m);
        st[i][j][r] = e;
        l += e;
      }
    }
    l = xsum16(l);
    const float inv = 1.f / l;
#pragma unroll
    for (int i = 0; i < TT; ++i) pf[j][i] = pack4(st[i][j] * inv);
    lsev[j] = m + __logf(l);
  }
  // O[query tile j][d tile n] = sum_i P[j][i] V[i][n]
#pragma unroll
  for (int n = 0; n < DT; ++n) {
    bf16x4v vf[TT];
#pragma unroll
    for (int i = 0; i < TT; ++i) vf[i] = ld4col(vb + (size_t)(16 * i + 4 * g) * ldq + 16 * n + c, ldq);
#pragma unroll
    for (int j = 0; j < TT; ++j) {
      f32x4v acc = (f32x4v){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < TT; ++i) acc = mfma16(pf[j][i], vf[i], acc);
#pragma unroll
      for (int r = 0; r < 4; ++r) o[(row0 + 16 * j + 4 * g + r) * ldo + h * D + 16 * n + c] = f32_to_bf16(acc[r]);
    }
  }
  if (g == 0) {
#pragma unroll
    for (int j = 0; j < TT; ++j) lse[(size_t)bh * T + 16 * j + c] = lsev[j];
  }
}

template <int TT, int DT>
__global__ __launch_bounds__(256) void attn_bwd_mfma(const uint16_t* q, const uint16_t* k, const uint16_t* v,
                                                     const uint16_t* o, const uint16_t* dout, const float* lse,
                                                     uint16_t* dq, uint16_t* dk, uint16_t* dv, int BH, int H, int ldq,
                                                     int ldo, float scale) {
  constexpr int T = TT * 16, D = DT * 16;
  __shared__ float sdl[4][T];  // delta_q = rowsum(dO_q * O_q) per wave
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int bh = blockIdx.x * 4 + w;
  const bool live = bh < BH;
  const int bhc = live ? bh : BH - 1;
  const int b = bhc / H, h = bhc - b * H;
  const size_t row0 = (size_t)b * T;
  const int c = lane & 15, g = lane >> 4;
  const uint16_t* qb = q + row0 * ldq + h * D;
  const uint16_t* kb = k + row0 * ldq + h * D;
  const uint16_t* vb = v + row0 * ldq + h * D;
  const uint16_t* ob = o + row0 * ldo + h * D;
  const uint16_t* gb = dout + row0 * ldo + h * D;
  for (int t = lane; t < T; t += 64) {
    float s = 0.f;
#pragma unroll
    for (int d = 0; d < D; d += 4) {
      const bf16x4v a = ld4(ob + (size_t)t * ldo + d), bb = ld4(gb + (size_t)t * ldo + d);
#pragma unroll
      for (int e = 0; e < 4; ++e) s += bf16_to_f32((uint16_t)a[e]) * bf16_to_f32((uint16_t)bb[e]);
    }
    sdl[w][t] = s;
  }
  __syncthreads();
  if (!live) return;
  const float* lb = lse + (size_t)bh * T;
  // ---------------- pass A: S layout (C: col = key, row = query) -> dV, dK
  {
    f32x4v sc[TT][TT], dp[TT][TT];  // [query tile j][key tile i]
#pragma unroll
    for (int j = 0; j < TT; ++j)
#pragma unroll
      for (int i = 0; i < TT; ++i) { sc[j][i] = (f32x4v){0.f, 0.f, 0.f, 0.f}; dp[j][i] = sc[j][i]; }
#pragma unroll
    for (int kd = 0; kd < DT; ++kd) {
      bf16x4v qf[TT], kf[TT], gf[TT], vf[TT];
#pragma unroll
      for (int j = 0; j < TT; ++j) {
        qf[j] = ld4(qb + (size_t)(16 * j + c) * ldq + 16 * kd + 4 * g);
        gf[j] = ld4(gb + (size_t)(16 * j + c) * ldo + 16 * kd + 4 * g);
      }
#pragma unroll
      for (int i = 0; i < TT; ++i) {
        kf[i] = ld4(kb + (size_t)(16 * i + c) * ldq + 16 * kd + 4 * g);
        vf[i] = ld4(vb + (size_t)(16 * i + c) * ldq + 16 * kd + 4 * g);
      }
#pragma unroll
      for (int j = 0; j < TT; ++j)
#pragma unroll
        for (int i = 0; i < TT; ++i) {
          sc[j][i] = mfma16(qf[j], kf[i], sc[j][i]);   // S = Q K^T
          dp[j][i] = mfma16(gf[j], vf[i], dp[j][i]);   // dP = dO V^T
        }
    }
    // P and dS (rows = queries 16j + 4g + r)
    bf16x4v pa[TT][TT], dsa[TT][TT];  // A fragments of P^T / dS^T: [key tile i][query k-step j]
#pragma unroll
    for (int j = 0; j < TT; ++j) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qi = 16 * j + 4 * g + r;
        const float lq = lb[qi], dq_ = sdl[w][qi];
#pragma unroll
        for (int i = 0; i < TT; ++i) {
          const float p = __expf(sc[j][i][r] * scale - lq);
          sc[j][i][r] = p;
          dp[j][i][r] = p * (dp[j][i][r] - dq_);
        }
      }
#pragma unroll
      for (int i = 0; i < TT; ++i) { pa[i][j] = pack4(sc[j][i]); dsa[i][j] = pack4(dp[j][i]); }
    }
    // dV[key tile i][d tile n] = sum_j P^T[i][j] dO[j][n] ; dK = scale * sum_j dS^T[i][j] Q[j][n]
#pragma unroll
    for (int n = 0; n < DT; ++n) {
      bf16x4v gcol[TT], qcol[TT];
#pragma unroll
      for (int j = 0; j < TT; ++j) {
        gcol[j] = ld4col(gb + (size_t)(16 * j + 4 * g) * ldo + 16 * n + c, ldo);
        qcol[j] = ld4col(qb + (size_t)(16 * j + 4 * g) * ldq + 16 * n + c, ldq);
      }
#pragma unroll
      for (int i = 0; i < TT; ++i) {
        f32x4v av = (f32x4v){0.f, 0.f, 0.f, 0.f}, ak = av;
#pragma unroll
        for (int j = 0; j < TT; ++j) {
          av = mfma16(pa[i][j], gcol[j], av);
          ak = mfma16(dsa[i][j], qcol[j], ak);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const size_t off = (row0 + 16 * i + 4 * g + r) * ldq + h * D + 16 * n + c;
          dv[off] = f32_to_bf16(av[r]);
          dk[off] = f32_to_bf16(ak[r] * scale);
        }
      }
    }
  }
  // ---------------- pass B: S^T layout (C: col = query, row = key) -> dQ
  {
    f32x4v st[TT][TT], dpt[TT][TT];  // [key tile i][query tile j]
#pragma unroll
    for (int i = 0; i < TT; ++i)
#pragma unroll
      for (int j = 0; j < TT; ++j) { st[i][j] = (f32x4v){0.f, 0.f, 0.f, 0.f}; dpt[i][j] = st[i][j]; }
#pragma unroll
    for (int kd = 0; kd < DT; ++kd) {
      bf16x4v qf[TT], kf[TT], gf[TT], vf[TT];
#pragma unroll
      for (int j = 0; j < TT; ++j) {
        qf[j] = ld4(qb + (size_t)(16 * j + c) * ldq + 16 * kd + 4 * g);
        gf[j] = ld4(gb + (size_t)(16 * j + c) * ldo + 16 * kd + 4 * g);
      }
#pragma unroll
      for (int i = 0; i < TT; ++i) {
        kf[i] = ld4(kb + (size_t)(16 * i + c) * ldq + 16 * kd + 4 * g);
        vf[i] = ld4(vb + (size_t)(16 * i + c) * ldq + 16 * kd + 4 * g);
      }
#pragma unroll
      for (int i = 0; i < TT; ++i)
#pragma unroll
        for (int j = 0; j < TT; ++j) {
          st[i][j] = mfma16(kf[i], qf[j], st[i][j]);    // S^T = K Q^T
          dpt[i][j] = mfma16(vf[i], gf[j], dpt[i][j]);  // dP^T = V dO^T
        }
    }
    bf16x4v dsq[TT][TT];  // A fragments of dS: [query tile j][key k-step i]
#pragma unroll
    for (int j = 0; j < TT; ++j) {
      const int qi = 16 * j + c;
      const float lq = lb[qi], dq_ = sdl[w][qi];
#pragma unroll
      for (int i = 0; i < TT; ++i) {
        f32x4v t;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = __expf(st[i][j][r] * scale - lq);
          t[r] = p * (dpt[i][j][r] - dq_);
        }
        dsq[j][i] = pack4(t);
      }
    }
#pragma unroll
    for (int n = 0; n < DT; ++n) {
      bf16x4v kcol[TT];
#pragma unroll
      for (int i = 0; i < TT; ++i) kcol[i] = ld4col(kb + (size_t)(16 * i + 4 * g) * ldq + 16 * n + c, ldq);
#pragma unroll
      for (int j = 0; j < TT; ++j) {
        f32x4v aq = (f32x4v){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < TT; ++i) aq = mfma16(dsq[j][i], kcol[i], aq);
#pragma unroll
        for (int r = 0; r < 4; ++r)
          dq[(row0 + 16 * j + 4 * g + r) * ldq + h * D + 16 * n + c] = f32_to_bf16(aq[r] * scale);
      }
    }
  }
}

template <int TT, int DT>
static hipError_t launch_attn_mfma(bool bwd, const uint16_t* q, const uint16_t* k, const uint16_t* v,
                                   const uint16_t* o, const uint16_t* dout, const float* lse_in, float* lse_out,
                                   uint16_t* out0, uint16_t* dk, uint16_t* dv, int BH, int H, int ldq, int ldo,
                                   float scale, hipStream_t st) {
  const int grid = (BH + 3) / 4;
  if (!bwd)
    hipLaunchKernelGGL((attn_fwd_mfma<TT, DT>), dim3(grid), dim3(256), 0, st, q, k, v, out0, lse_out, BH, H, ldq, ldo,
                       scale);
  else
    hipLaunchKernelGGL((attn_bwd_mfma<TT, DT>), dim3(grid), dim3(256), 0, st, q, k, v, o, dout, lse_in, out0, dk, dv,
                       BH, H, ldq, ldo, scale);
  return hipGetLastError();
}

template <int TT>
static hipError_t attn_mfma_d(int DT, bool bwd, const uint16_t* q, const uint16_t* k, const uint16_t* v,
                              const uint16_t* o, const uint16_t* dout, const float* lse_in, float* lse_out,
                              uint16_t* out0, uint16_t* dk, uint16_t* dv, int BH, int H, int ldq, int ldo, float scale,
                              hipStream_t st) {
  switch (DT) {
    case 1: return launch_attn_mfma<TT, 1>(bwd, q, k, v, o, dout, lse_in, lse_out, out0, dk, dv, BH, H, ldq, ldo, scale, st);
    case 2: return launch_attn_mfma<TT, 2>(bwd, q, k, v, o, dout, lse_in, lse_out, out0, dk, dv, BH, H, ldq, ldo, scale, st);
    case 4: return launch_attn_mfma<TT, 4>(bwd, q, k, v, o, dout, lse_in, lse_out, out0, dk, dv, BH, H, ldq, ldo, scale, st);
    default: return hipErrorInvalidValue;
  }
}

// true when the MFMA path handled the call
static bool attn_mfma(bool bwd, const uint16_t* q, const uint16_t* k, const uint16_t* v, const uint16_t* o,
                      const uint16_t* dout, const float* lse_in, float* lse_out, uint16_t* out0, uint16_t* dk,
                      uint16_t* dv, int Bsz, int H, int T, int D, int ldq, int ldo, float scale, hipStream_t st,
                      hipError_t* err) {
  if (T % 16 || D % 16 || T > 64 || !(D == 16 || D == 32 || D == 64)) return false;
  if (ldq % 4 || ldo % 4 || ((((uintptr_t)q) | ((uintptr_t)k) | ((uintptr_t)v) | ((uintptr_t)dout)) & 7)) return false;
  const int BH = Bsz * H, DT = D / 16;
  switch (T / 16) {
    case 1: *err = attn_mfma_d<1>(DT, bwd, q, k, v, o, dout, lse_in, lse_out, out0, dk, dv, BH, H, ldq, ldo, scale, st); break;
    case 2: *err = attn_mfma_d<2>(DT, bwd, q, k, v, o, dout, lse_in, lse_out, out0, dk, dv, BH, H, ldq, ldo, scale, st); break;
    case 3: *err = attn_mfma_d<3>(DT, bwd, q, k, v, o, dout, lse_in, lse_out, out0, dk, dv, BH, H, ldq, ldo, scale, st); break;
    default: *err = attn_mfma_d<4>(DT, bwd, q, k, v, o, dout, lse_in, lse_out, out0, dk, dv, BH, H, ldq, ldo, scale, st);
  }
  return true;
}

}  // namespace dct

extern "C" {

int dct_attention_fwd(const uint16_t* q, const uint16_t* k, const uint16_t* v, uint16_t* o, float* lse, int Bsz, int H,
                      int T, int D, int ldq, int ldo, float scale, void* stream) {
  if (D > dct::ATT_MAXD || T > 512 || T < 1) return (int)hipErrorInvalidValue;
  {
    hipError_t me = hipSuccess;
    if (dct::attn_mfma(false, q, k, v, nullptr, nullptr, nullptr, lse, o, nullptr, nullptr, Bsz, H, T, D, ldq, ldo,
                       scale, reinterpret_cast<hipStream_t>(stream), &me))
      return (int)me;
  }
  const size_t lds = (size_t)2 * T * D * sizeof(uint16_t);
  auto fn = dct::attn_fwd_kernel;
  hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(fn, dim3(Bsz * H), dim3(dct::ATT_NT), lds, reinterpret_cast<hipStream_t>(stream), q, k, v, o, lse,
                     H, T, D, ldq, ldo, scale);
  return (int)hipGetLastError();
}

int dct_attention_bwd(const uint16_t* q, const uint16_t* k, const uint16_t* v, const uint16_t* o,
                      const uint16_t* dout, const float* lse, uint16_t* dq, uint16_t* dk, uint16_t* dv, int Bsz, int H,
                      int T, int D, int ldq, int ldo, float scale, void* stream) {
  if (D > dct::ATT_MAXD || T > 512 || T < 1) return (int)hipErrorInvalidValue;
  {
    hipError_t me = hipSuccess;
    if (dct::attn_mfma(true, q, k, v, o, dout, lse, nullptr, dq, dk, dv, Bsz, H, T, D, ldq, ldo, scale,
                       reinterpret_cast<hipStream_t>(stream), &me))
      return (int)me;
  }
  const size_t lds = (size_t)4 * T * D * sizeof(uint16_t) + 4 + (size_t)2 * T * sizeof(float);
  if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
  auto fn = dct::attn_bwd_kernel;
  hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(fn, dim3(Bsz * H), dim3(dct::ATT_NT), lds, reinterpret_cast<hipStream_t>(stream), q, k, v, o,
                     dout, lse, dq, dk, dv, H, T, D, ldq, ldo, scale);
  return (int)hipGetLastError();
}

}  // extern "C"
