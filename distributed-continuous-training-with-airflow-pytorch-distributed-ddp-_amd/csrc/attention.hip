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

}  // namespace dct

extern "C" {

int dct_attention_fwd(const uint16_t* q, const uint16_t* k, const uint16_t* v, uint16_t* o, float* lse, int Bsz, int H,
                      int T, int D, int ldq, int ldo, float scale, void* stream) {
  if (D > dct::ATT_MAXD || T > 512 || T < 1) return (int)hipErrorInvalidValue;
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
