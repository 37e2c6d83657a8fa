// TabTransformer input / output ends as native kernels (BASELINE.json config 5).
//
// Feature-token embedding  h[b, f, :] = x[b, f] * E[f, :] + c[f, :]  and its parameter gradients
// (sums over the batch), and the classifier end  mean-pool over tokens -> LayerNorm -> Linear(D, C)
// -> mean cross-entropy  as one forward kernel (loss) plus one backward kernel that recomputes
// the tiny per-sample chain and emits dh, dE/dc-style parameter gradients and the head's.
// Under torch these were ~20 launches per step (broadcast mul/add, mean reduce, LN, skinny
// GEMMs, log-softmax/NLL forward and backward, expand, batch reductions) ~ 150 us at batch 512.
// Layout: one wave per sample for the head (lane = model dimension, D == 64); the embedding
// backward is a batch reduction split over (feature, batch-chunk) workgroups with fp32 atomics.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>

#include "dct_common.h"

namespace dct {
namespace ttio {

constexpr int D = 64;
constexpr int CMAX = 8;

__global__ __launch_bounds__(256) void embed_fwd_kernel(const float* __restrict__ x, const float* __restrict__ E,
                                                        const float* __restrict__ c, float* __restrict__ h, int B,
                                                        int F) {
  const int n4 = B * F * (D / 4);  // host checks it fits in int (32-bit index math: no 64-bit divides)
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n4; i += gridDim.x * 256) {
    const int tok = i >> 4;  // D / 4 == 16
    const int q = i & 15;
    const int f = tok % F;
    const float xv = x[tok];
    const float4 e = reinterpret_cast<const float4*>(E + (size_t)f * D)[q];
    const float4 cc = reinterpret_cast<const float4*>(c + (size_t)f * D)[q];
    reinterpret_cast<float4*>(h)[i] = make_float4(fmaf(xv, e.x, cc.x), fmaf(xv, e.y, cc.y), fmaf(xv, e.z, cc.z),
                                                  fmaf(xv, e.w, cc.w));
  }
}

// grid (F, chunks): workgroup sums samples b = chunk, chunk + chunks, ... of feature f;
// thread = (sample slot s = tid / 64, dimension d = tid % 64)
__global__ __launch_bounds__(256) void embed_bwd_kernel(const float* __restrict__ x, const float* __restrict__ dh,
                                                        float* dE, float* dc, int B, int F) {
  __shared__ float sw[4][D], sb[4][D];
  const int f = blockIdx.x, chunk = blockIdx.y, chunks = gridDim.y;
  const int s = threadIdx.x >> 6, d = threadIdx.x & 63;
  float aw = 0.f, ab = 0.f;
  for (int b = chunk * 4 + s; b < B; b += chunks * 4) {
    const size_t tok = (size_t)b * F + f;
    const float g = dh[tok * D + d];
    aw = fmaf(x[tok], g, aw);
    ab += g;
  }
  sw[s][d] = aw;
  sb[s][d] = ab;
  __syncthreads();
  if (threadIdx.x < D) {
    atomicAdd(dE + (size_t)f * D + d, sw[0][d] + sw[1][d] + sw[2][d] + sw[3][d]);
  } else if (threadIdx.x < 2 * D) {
    const int dd = threadIdx.x - D;
    atomicAdd(dc + (size_t)f * D + dd, sb[0][dd] + sb[1][dd] + sb[2][dd] + sb[3][dd]);
  }
}

struct HeadArgs {
  const float* h;  // [B][T][D] fp32 residual stream after the last block
  const int64_t* y;
  const float *ln_w, *ln_b, *W, *bias;  // LN (D), head W [C][D], bias [C]
  float* loss;                          // forward: mean CE (stored, no pre-zeroed output needed)
  float* partial;                       // forward: one loss partial per workgroup
  unsigned* ticket;                     // forward: finished-workgroup count, 0 between launches
  const float* dloss;                   // backward: upstream gradient of the loss (device scalar)
  float* dh; uint16_t* dh16;            // backward: d h (fp32 + bf16 copy)
  float *dln_w, *dln_b, *dW, *dbias;    // backward: accumulated
  int B, T, C;
  float eps;
};

__device__ __forceinline__ float wsum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// per-sample chain shared by both kernels: lane = dimension d
struct HeadFwd {
  float xhat, rstd, z, lnw;
  float logit[CMAX], w[CMAX];  // w[k] = head W[k][d]
};

__device__ __forceinline__ HeadFwd head_chain(const HeadArgs& a, int b, int d) {
  HeadFwd r;
  // parameter loads first and unconditionally (class slots past C re-read class C-1 and are masked), so
  // their latency hides under the token stream; loads guarded by k < C compiled to branches that each
  // drained the load queue (s_waitcnt vmcnt(0))
  r.lnw = a.ln_w[d];
  const float lnb = a.ln_b[d];
  float bk[CMAX];
#pragma unroll
  for (int k = 0; k < CMAX; ++k) {
    const int kc = k < a.C ? k : a.C - 1;
    r.w[k] = a.W[kc * D + d];
    bk[k] = a.bias[kc];
  }
  // mean over tokens with 16-byte loads: lane (tq = lane >> 4, dq = lane & 15) sums dims 4dq..4dq+3
  // of tokens tq, tq + 4, ...; then lane d fetches its dimension from lane d / 4 (tq = 0)
  const float* hb = a.h + (size_t)b * a.T * D;
  const int tq = d >> 4, dq = d & 15;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 8
  for (int t = tq; t < a.T; t += 4) {
    const float4 v = reinterpret_cast<const float4*>(hb + (size_t)t * D)[dq];
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  acc.x += __shfl_xor(acc.x, 16); acc.y += __shfl_xor(acc.y, 16); acc.z += __shfl_xor(acc.z, 16); acc.w += __shfl_xor(acc.w, 16);
  acc.x += __shfl_xor(acc.x, 32); acc.y += __shfl_xor(acc.y, 32); acc.z += __shfl_xor(acc.z, 32); acc.w += __shfl_xor(acc.w, 32);
  const float p0 = __shfl(acc.x, d >> 2), p1 = __shfl(acc.y, d >> 2), p2 = __shfl(acc.z, d >> 2), p3 = __shfl(acc.w, d >> 2);
  const int e = d & 3;
  float p = e == 0 ? p0 : e == 1 ? p1 : e == 2 ? p2 : p3;
  p *= 1.f / a.T;
  const float mean = wsum(p) * (1.f / D);
  const float dv = p - mean;
  r.rstd = rsqrtf(wsum(dv * dv) * (1.f / D) + a.eps);
  r.xhat = dv * r.rstd;
  r.z = r.xhat * r.lnw + lnb;
#pragma unroll
  for (int k = 0; k < CMAX; ++k) r.logit[k] = (k < a.C) ? wsum(r.z * r.w[k]) + bk[k] : -3.402823466e+38f;
  return r;
}

// NW samples per workgroup (one wave each).  The per-sample losses meet in LDS; each block stores ONE
// partial, and the last block to finish (ticket count) sums the partials in block order and stores
// the loss: deterministic, and the caller needs no zero-filled loss (a fill kernel per step before,
// 512 same-address float atomics, one per sample, before that).  The last block resets the ticket.
template <int NW>
__global__ __launch_bounds__(64 * NW) void head_fwd_kernel(HeadArgs a) {
  __shared__ float lsum[NW];
  const int w = threadIdx.x >> 6, d = threadIdx.x & 63;
  const int b = blockIdx.x * NW + w;
  if (d == 0) lsum[w] = 0.f;
  if (b < a.B) {
  const int yb = (int)a.y[b];
  const HeadFwd r = head_chain(a, b, d);
  if (d == 0) {
    float m = r.logit[0];
#pragma unroll
    for (int k = 1; k < CMAX; ++k) m = fmaxf(m, r.logit[k]);
    float se = 0.f;
#pragma unroll
    for (int k = 0; k < CMAX; ++k) se += (k < a.C) ? __expf(r.logit[k] - m) : 0.f;
    float ly = 0.f;
#pragma unroll
    for (int k = 0; k < CMAX; ++k) ly = (k == yb) ? r.logit[k] : ly;
    lsum[w] = (m + __logf(se) - ly) / a.B;
  }
  }
  __shared__ unsigned last;
  __syncthreads();
  if (threadIdx.x == 0) {
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < NW; ++i) v += lsum[i];
    // partial and ticket as memory-side atomics, ordered by waiting for the first to complete: no
    // agent-scope release / acquire fences (each writes back / invalidates the XCD's L2 - see the LN
    // replicas of tt_block.hip, whose gfx950 assumptions this shares), and the last block reads the
    // partials by atomics too (an L2 of another XCD may hold a stale line of them)
    atomicExch(a.partial + blockIdx.x, v);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  }
  __syncthreads();
  if (last && threadIdx.x < 64) {
    // wave 0 sums the partials: lane-strided loads all in flight at once, then the butterfly (a fixed
    // order, so the loss is bit-identical run to run); a one-thread serial sum cost ~18 us per step
    float s = 0.f;
    for (unsigned i = threadIdx.x; i < gridDim.x; i += 64) s += atomicAdd(a.partial + i, 0.f);
    s = wsum(s);
    if (threadIdx.x == 0) {
      a.loss[0] = s;
      __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// FWD: the training forward with the backward folded in (dct_tt_head_fused): the loss as head_fwd_kernel
// stores it, and every gradient as this kernel computes it for an upstream gradient of exactly 1 - the
// seed the autograd engine's loss.backward(ones) passes - so the training step needs no backward launch
template <int NW, bool FWD = false>
__global__ __launch_bounds__(64 * NW) void head_bwd_kernel(HeadArgs a) {
  __shared__ float red[NW][2 + CMAX][D];  // per wave: dln_w, dln_b, dW[C]
  __shared__ float rbias[NW][CMAX];
  __shared__ float lsum[NW];
  const int w = threadIdx.x >> 6, d = threadIdx.x & 63;
  const int b = blockIdx.x * NW + w;
  const bool live = b < a.B;
  float gw = 0.f, gb = 0.f, gW[CMAX], gbias[CMAX];
#pragma unroll
  for (int k = 0; k < CMAX; ++k) { gW[k] = 0.f; gbias[k] = 0.f; }
  if (FWD && d == 0) lsum[w] = 0.f;
  if (live) {
    const int yb = (int)a.y[b];
    const float dls = FWD ? 1.f : a.dloss[0];
    const HeadFwd r = head_chain(a, b, d);
    float m = r.logit[0];
#pragma unroll
    for (int k = 1; k < CMAX; ++k) m = fmaxf(m, r.logit[k]);
    float se = 0.f;
#pragma unroll
    for (int k = 0; k < CMAX; ++k) se += (k < a.C) ? __expf(r.logit[k] - m) : 0.f;
    if (FWD && d == 0) {  // the sample's loss, as head_fwd_kernel
      float ly = 0.f;
#pragma unroll
      for (int k = 0; k < CMAX; ++k) ly = (k == yb) ? r.logit[k] : ly;
      lsum[w] = (m + __logf(se) - ly) / a.B;
    }
    const float scale = dls / a.B, inv = 1.f / se;
    float dz = 0.f;
#pragma unroll
    for (int k = 0; k < CMAX; ++k) {
      const float dl = (k < a.C) ? (__expf(r.logit[k] - m) * inv - (k == yb ? 1.f : 0.f)) * scale : 0.f;
      gW[k] = dl * r.z;
      gbias[k] = dl;
      dz = fmaf(dl, r.w[k], dz);  // dl = 0 past C
    }
    gw = dz * r.xhat;
    gb = dz;
    const float g = dz * r.lnw;
    const float m1 = wsum(g) * (1.f / D), m2 = wsum(g * r.xhat) * (1.f / D);
    const float dp = r.rstd * (g - m1 - r.xhat * m2) * (1.f / a.T);
    // broadcast over tokens with 16-byte stores: lane (tq, dq) writes dims 4dq..4dq+3 of tokens tq, tq + 4, ...
    const int tq = d >> 4, dq = d & 15;
    float4 v4;
    v4.x = __shfl(dp, 4 * dq); v4.y = __shfl(dp, 4 * dq + 1); v4.z = __shfl(dp, 4 * dq + 2); v4.w = __shfl(dp, 4 * dq + 3);
    uint2 h4;
    h4.x = f32_to_bf16(v4.x) | ((uint32_t)f32_to_bf16(v4.y) << 16);
    h4.y = f32_to_bf16(v4.z) | ((uint32_t)f32_to_bf16(v4.w) << 16);
    float* dhb = a.dh + (size_t)b * a.T * D;
    uint16_t* dh16b = a.dh16 + (size_t)b * a.T * D;
#pragma unroll 8
    for (int t = tq; t < a.T; t += 4) {
      reinterpret_cast<float4*>(dhb + (size_t)t * D)[dq] = v4;
      reinterpret_cast<uint2*>(dh16b + (size_t)t * D)[dq] = h4;
    }
  }
  red[w][0][d] = gw;
  red[w][1][d] = gb;
#pragma unroll
  for (int k = 0; k < CMAX; ++k) red[w][2 + k][d] = gW[k];
  {  // bias gradient per class is the same in every lane of the wave
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < CMAX; ++k) v = (k == d) ? gbias[k] : v;
    if (d < CMAX) rbias[w][d] = v;
  }
  __syncthreads();
  // workgroup reduction over its NW samples, then one atomic per parameter element
  for (int i = threadIdx.x; i < (2 + a.C) * D; i += 64 * NW) {
    const int row = i / D, dd = i - row * D;
    float v = 0.f;
#pragma unroll
    for (int q = 0; q < NW; ++q) v += red[q][row][dd];
    float* dst = row == 0 ? a.dln_w + dd : row == 1 ? a.dln_b + dd : a.dW + (row - 2) * D + dd;
    atomicAdd(dst, v);
  }
  if (threadIdx.x < a.C) {
    float v = 0.f;
#pragma unroll
    for (int q = 0; q < NW; ++q) v += rbias[q][threadIdx.x];
    atomicAdd(a.dbias + threadIdx.x, v);
  }
  if constexpr (FWD) {  // the loss: block partials and the last block's ordered sum, as head_fwd_kernel
    __shared__ unsigned last;
    if (threadIdx.x == 0) {
      float v = 0.f;
#pragma unroll
      for (int i = 0; i < NW; ++i) v += lsum[i];
      atomicExch(a.partial + blockIdx.x, v);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      last = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    }
    __syncthreads();
    if (last && threadIdx.x < 64) {
      float s = 0.f;
      for (unsigned i = threadIdx.x; i < gridDim.x; i += 64) s += atomicAdd(a.partial + i, 0.f);
      s = wsum(s);
      if (threadIdx.x == 0) {
        a.loss[0] = s;
        __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

// samples per workgroup (one wave each): 4.  16-sample (1024-thread) blocks quarter the
// parameter-gradient atomics but measured no faster on the TabTransformer step (0.4195-0.4240 vs
// 0.4184-0.4221 ms, profiles/tt_head_spb_side_dw_ab_r2.log), nor 2 / 1 (profiles/tt_head_spb_ab_r4.log).
constexpr int HEAD_SPB = 4;
// the pooled head (T = 1: the last block handed over the token means) has ~nothing to load per sample;
// there the same-address parameter-gradient atomics of ceil(B / 4) workgroups dominate the backward:
// 16 samples per workgroup (a quarter of the adders per address): TT step 0.3412-0.3440 -> 0.3384-0.3392 ms
// (bench.py alternating on one box, profiles/tt_pooled_head_spb_ab_r5.log)
constexpr int HEAD_SPB_POOLED = 16;

}  // namespace ttio
}  // namespace dct

static inline int grid_cap(int64_t work, int per, int cap) {
  int64_t g = (work + per - 1) / per;
  return (int)(g < 1 ? 1 : g > cap ? cap : g);
}

extern "C" {

int dct_tt_embed_fwd(const float* x, const float* E, const float* c, float* h, int B, int F, int Dm, void* stream) {
  if (Dm != dct::ttio::D || B <= 0 || F <= 0 || ((((uintptr_t)E) | ((uintptr_t)c) | ((uintptr_t)h)) & 15) ||
      (int64_t)B * F * (Dm / 4) >= (int64_t)1 << 31)
    return (int)hipErrorInvalidValue;
  const int64_t n4 = (int64_t)B * F * (Dm / 4);
  hipLaunchKernelGGL(dct::ttio::embed_fwd_kernel, dim3(grid_cap(n4, 256, 4096)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), x, E, c, h, B, F);
  return (int)hipGetLastError();
}

int dct_tt_embed_bwd(const float* x, const float* dh, float* dE, float* dc, int B, int F, int Dm, void* stream) {
  if (Dm != dct::ttio::D || B <= 0 || F <= 0) return (int)hipErrorInvalidValue;
  const int chunks = (int)std::min<int64_t>(std::max<int64_t>(1, 1024 / F), (B + 3) / 4);
  hipLaunchKernelGGL(dct::ttio::embed_bwd_kernel, dim3(F, chunks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     x, dh, dE, dc, B, F);
  return (int)hipGetLastError();
}

// ptrs: h, y(int64), ln_w, ln_b, W, bias, loss, partial (>= ceil(B / 4) floats), ticket
// (uint32, zero before the first launch; every launch leaves it zero)  (forward)
int dct_tt_head_fwd(const uintptr_t* p, int n_ptrs, int B, int T, int Dm, int C, float eps, void* stream) {
  if (n_ptrs != 9 || Dm != dct::ttio::D || C < 1 || C > dct::ttio::CMAX || B <= 0 || T <= 0 || (p[0] & 15))
    return (int)hipErrorInvalidValue;
  dct::ttio::HeadArgs a{};
  a.h = (const float*)p[0]; a.y = (const int64_t*)p[1]; a.ln_w = (const float*)p[2]; a.ln_b = (const float*)p[3];
  a.W = (const float*)p[4]; a.bias = (const float*)p[5]; a.loss = (float*)p[6];
  a.partial = (float*)p[7]; a.ticket = (unsigned*)p[8];
  a.B = B; a.T = T; a.C = C; a.eps = eps;
  constexpr int nw = dct::ttio::HEAD_SPB, nwp = dct::ttio::HEAD_SPB_POOLED;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (T == 1)
    hipLaunchKernelGGL(dct::ttio::head_fwd_kernel<nwp>, dim3((B + nwp - 1) / nwp), dim3(64 * nwp), 0, st, a);
  else
    hipLaunchKernelGGL(dct::ttio::head_fwd_kernel<nw>, dim3((B + nw - 1) / nw), dim3(64 * nw), 0, st, a);
  return (int)hipGetLastError();
}

// ptrs: h, y(int64), ln_w, ln_b, W, bias, dloss, dh, dh16, dln_w, dln_b, dW, dbias  (backward)
int dct_tt_head_bwd(const uintptr_t* p, int n_ptrs, int B, int T, int Dm, int C, float eps, void* stream) {
  if (n_ptrs != 13 || Dm != dct::ttio::D || C < 1 || C > dct::ttio::CMAX || B <= 0 || T <= 0 ||
      ((p[0] | p[7] | p[8]) & 15))
    return (int)hipErrorInvalidValue;
  dct::ttio::HeadArgs a{};
  a.h = (const float*)p[0]; a.y = (const int64_t*)p[1]; a.ln_w = (const float*)p[2]; a.ln_b = (const float*)p[3];
  a.W = (const float*)p[4]; a.bias = (const float*)p[5]; a.dloss = (const float*)p[6];
  a.dh = (float*)p[7]; a.dh16 = (uint16_t*)p[8]; a.dln_w = (float*)p[9]; a.dln_b = (float*)p[10];
  a.dW = (float*)p[11]; a.dbias = (float*)p[12];
  a.B = B; a.T = T; a.C = C; a.eps = eps;
  constexpr int nw = dct::ttio::HEAD_SPB, nwp = dct::ttio::HEAD_SPB_POOLED;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (T == 1)
    hipLaunchKernelGGL(dct::ttio::head_bwd_kernel<nwp>, dim3((B + nwp - 1) / nwp), dim3(64 * nwp), 0, st, a);
  else
    hipLaunchKernelGGL(dct::ttio::head_bwd_kernel<nw>, dim3((B + nw - 1) / nw), dim3(64 * nw), 0, st, a);
  return (int)hipGetLastError();
}

// ptrs: h, y(int64), ln_w, ln_b, W, bias, loss, partial, ticket, dh, dh16, dln_w, dln_b, dW, dbias:
// the forward's loss and the backward's gradients for an upstream loss gradient of 1, one launch
int dct_tt_head_fused(const uintptr_t* p, int n_ptrs, int B, int T, int Dm, int C, float eps, void* stream) {
  if (n_ptrs != 15 || Dm != dct::ttio::D || C < 1 || C > dct::ttio::CMAX || B <= 0 || T <= 0 ||
      ((p[0] | p[9] | p[10]) & 15))
    return (int)hipErrorInvalidValue;
  dct::ttio::HeadArgs a{};
  a.h = (const float*)p[0]; a.y = (const int64_t*)p[1]; a.ln_w = (const float*)p[2]; a.ln_b = (const float*)p[3];
  a.W = (const float*)p[4]; a.bias = (const float*)p[5]; a.loss = (float*)p[6];
  a.partial = (float*)p[7]; a.ticket = (unsigned*)p[8];
  a.dh = (float*)p[9]; a.dh16 = (uint16_t*)p[10]; a.dln_w = (float*)p[11]; a.dln_b = (float*)p[12];
  a.dW = (float*)p[13]; a.dbias = (float*)p[14];
  a.B = B; a.T = T; a.C = C; a.eps = eps;
  constexpr int nw = dct::ttio::HEAD_SPB, nwp = dct::ttio::HEAD_SPB_POOLED;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (T == 1)
    hipLaunchKernelGGL((dct::ttio::head_bwd_kernel<nwp, true>), dim3((B + nwp - 1) / nwp), dim3(64 * nwp), 0, st, a);
  else
    hipLaunchKernelGGL((dct::ttio::head_bwd_kernel<nw, true>), dim3((B + nw - 1) / nw), dim3(64 * nw), 0, st, a);
  return (int)hipGetLastError();
}

}  // extern "C"
