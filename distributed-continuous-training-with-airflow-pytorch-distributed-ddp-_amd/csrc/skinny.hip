// Skinny layers: C <= 8 outputs (the classifier head of the tabular / TabTransformer models).
//
// A 128x128 MFMA tile would compute 2 useful columns out of 128, and the dW of such a layer
// (2 x 1024 with K = batch) has too few rows for any tile shape.  These layers are HBM
// streams, so they are written as bandwidth kernels: 16-byte loads, fp32 accumulation, the
// tiny weight panel read through the cache, wave reductions by shuffles.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "dct_common.h"

namespace dct {

constexpr int SK_CMAX = 8;

__device__ __forceinline__ void unpack8(const uint4& v, float (&f)[8]) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    f[2 * j] = bf16_to_f32(w[j] & 0xffff);
    f[2 * j + 1] = bf16_to_f32(w[j] >> 16);
  }
}

// Y[b][c] = X[b] . W[c] + bias[c]: one wave per row, each lane 8 k per 512-k chunk.  CT = C rounded up
// to 1/2/4/8; class rows past C re-read row C-1 (never stored): loads stay unconditional, since a
// guarded load compiles to a branch that drains every load in flight (s_waitcnt vmcnt(0)).
template <int CT>
__global__ __launch_bounds__(256) void skinny_fwd_kernel(const uint16_t* __restrict__ X,
                                                         const uint16_t* __restrict__ W,
                                                         const float* __restrict__ bias, uint16_t* __restrict__ Y,
                                                         int B, int K, int C) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  float acc[CT];
#pragma unroll
  for (int c = 0; c < CT; ++c) acc[c] = 0.f;
  for (int k = lane * 8; k < K; k += 512) {
    uint4 raw[CT + 1];
    raw[CT] = *reinterpret_cast<const uint4*>(X + (size_t)b * K + k);
#pragma unroll
    for (int c = 0; c < CT; ++c) raw[c] = *reinterpret_cast<const uint4*>(W + (size_t)(c < C ? c : C - 1) * K + k);
    float x[8];
    unpack8(raw[CT], x);
#pragma unroll
    for (int c = 0; c < CT; ++c) {
      float w[8];
      unpack8(raw[c], w);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[c] += x[e] * w[e];
    }
  }
#pragma unroll
  for (int c = 0; c < CT; ++c) {
    if (c < C) {
      float v = wave_sum(acc[c]);
      if (lane == 0) Y[(size_t)b * C + c] = f32_to_bf16(v + (bias ? bias[c] : 0.f));
    }
  }
}

// dX[b][k..k+8) = sum_c dZ[b][c] W[c][k..k+8)  (masked by the ReLU output aux > 0); CT as above
template <int CT>
__global__ __launch_bounds__(256) void skinny_dx_kernel(const uint16_t* __restrict__ dZ,
                                                        const uint16_t* __restrict__ W,
                                                        const uint16_t* __restrict__ aux, uint16_t* __restrict__ dX,
                                                        int B, int K, int C) {
  const int kv = K / 8;
  const int64_t total = (int64_t)B * kv;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int b = (int)(e / kv);
    const int k = (int)(e - (int64_t)b * kv) * 8;
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = 0.f;
    const size_t off = (size_t)b * K + k;
    const uint4 araw = aux ? *reinterpret_cast<const uint4*>(aux + off) : make_uint4(0, 0, 0, 0);
    uint4 wraw[CT];
    float dz[CT];
#pragma unroll
    for (int c = 0; c < CT; ++c) {
      const int cc = c < C ? c : C - 1;
      wraw[c] = *reinterpret_cast<const uint4*>(W + (size_t)cc * K + k);
      const float z = bf16_to_f32(dZ[(size_t)b * C + cc]);
      dz[c] = c < C ? z : 0.f;
    }
#pragma unroll
    for (int c = 0; c < CT; ++c) {
      float w[8];
      unpack8(wraw[c], w);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] += dz[c] * w[j];
    }
    if (aux) {
      float a[8];
      unpack8(araw, a);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = a[j] > 0.f ? o[j] : 0.f;
    }
    uint4 v;
    v.x = f32_to_bf16(o[0]) | ((uint32_t)f32_to_bf16(o[1]) << 16);
    v.y = f32_to_bf16(o[2]) | ((uint32_t)f32_to_bf16(o[3]) << 16);
    v.z = f32_to_bf16(o[4]) | ((uint32_t)f32_to_bf16(o[5]) << 16);
    v.w = f32_to_bf16(o[6]) | ((uint32_t)f32_to_bf16(o[7]) << 16);
    *reinterpret_cast<uint4*>(dX + off) = v;
  }
}

// dW[c][k] += sum_b dZ[b][c] X[b][k], db[c] += sum_b dZ[b][c].
// Block: 64 lanes x 8 k = 512 columns, 4 row lanes (waves); blockIdx.y splits the rows.  CT = the
// class count rounded up to 1/2/4/8, so registers and the cross-wave LDS reduction cover only real
// classes (CT = 2 -> 16 KB of LDS partials, several blocks per CU).  The X rows are the only HBM stream; the head's dZ is read as wave-uniform scalars.
template <int CT>
__global__ __launch_bounds__(256) void skinny_dw_kernel(const uint16_t* __restrict__ dZ,
                                                        const uint16_t* __restrict__ X, float* __restrict__ dW,
                                                        float* __restrict__ db, int B, int K, int C, int rows_per) {
  // partials in column order ([wave][c][col], col = lane * 8 + j): each lane writes its 8 columns as two
  // 16-byte stores and the fold reads lane-contiguous columns (the [j][lane] layout read 8 columns per
  // lane group from 8 rows of the tile: ~59% of its LDS cycles were bank conflicts, profiles/pmc_*)
  __shared__ float4 red4[4][CT][128];
  float (*red)[CT][512] = reinterpret_cast<float (*)[CT][512]>(red4);
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int k = (blockIdx.x * 64 + tx) * 8;
  const int r0 = blockIdx.y * rows_per;
  const int r1 = min(B, r0 + rows_per);
  float acc[CT][8];
  float dbs[CT];
#pragma unroll
  for (int c = 0; c < CT; ++c) {
    dbs[c] = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[c][j] = 0.f;
  }
  // Rows go in batches of U per wave: all U row loads (and their dZ scalars) are issued before any
  // FMA, so a wave pays one HBM latency per batch.  The loop this replaces guarded its dZ loads, which
  // compiled to a branch + s_waitcnt vmcnt(0) per load and drained every X load in flight: its time grew
  // with rows per block, 11.5 us at 64 rows and 39 us at 256 (profiles/skinny_dw_split_sweep_r1.txt).  Rows past
  // r1 re-read row r0 with dz = 0; lanes past K read column 0 and their sums are never stored.
  constexpr int U = CT <= 2 ? 8 : 4;
  const int kc = k < K ? k : 0;
  for (int b0 = r0 + ty; b0 < r1; b0 += 4 * U) {
    uint4 raw[U];
    float dz[U][CT];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int b = b0 + 4 * u;
      const bool ok = b < r1;
      const int bs = ok ? b : r0;
      raw[u] = *reinterpret_cast<const uint4*>(X + (size_t)bs * K + kc);
#pragma unroll
      for (int c = 0; c < CT; ++c) {  // unconditional load, masked after: a guarded load compiles to a
        const float z = bf16_to_f32(dZ[(size_t)bs * C + (c < C ? c : C - 1)]);  // branch + vmcnt(0) drain
        dz[u][c] = (ok && c < C) ? z : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float x[8];
      unpack8(raw[u], x);
#pragma unroll
      for (int c = 0; c < CT; ++c) {
        dbs[c] += dz[u][c];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[c][j] += dz[u][c] * x[j];
      }
    }
  }
#pragma unroll
  for (int c = 0; c < CT; ++c) {
    red4[ty][c][2 * tx] = make_float4(acc[c][0], acc[c][1], acc[c][2], acc[c][3]);
    red4[ty][c][2 * tx + 1] = make_float4(acc[c][4], acc[c][5], acc[c][6], acc[c][7]);
  }
  __syncthreads();
  // fold the 4 waves' partials in COLUMN order: thread t owns columns t and t + 256 of the block's
  // 512, so each atomic wave-instruction covers 256 contiguous bytes (the full-rate atomic shape;
  // a lane-per-8-columns pattern ran the head dW at 42 us)
  const int kbase = blockIdx.x * 512;
#pragma unroll
  for (int c = 0; c < CT; ++c) {
    if (c >= C) break;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int col = threadIdx.x + 256 * h;
      if (kbase + col < K) {
        const float v = red[0][c][col] + red[1][c][col] + red[2][c][col] + red[3][c][col];
        atomicAdd(dW + (size_t)c * K + kbase + col, v);
      }
    }
  }
  if (db && blockIdx.x == 0) {  // bias grads: every row lane saw every row of its stride
    __syncthreads();
    if (tx == 0) {
#pragma unroll
      for (int c = 0; c < CT; ++c) red[ty][c][0] = dbs[c];
    }
    __syncthreads();
    if (threadIdx.x < C) {
      const int c = threadIdx.x;
      atomicAdd(db + c, red[0][c][0] + red[1][c][0] + red[2][c][0] + red[3][c][0]);
    }
  }
}

// The whole classifier head of a training step in one kernel (the executor's skinny fwd -> loss
// -> skinny dW -> skinny dX chain, four launches and three extra passes over H, fused):
//   z[b]   = bf16(H[b] . W^T + bias)                      (rounded like the unfused bf16 logits)
//   loss  += CE(z[b], y[b]) or MSE(z[b], onehot(y[b]))     (summed, * loss_scale, one atomic/block)
//   dz[b]  = bf16(dL/dz * grad_scale)                      (rounded like the unfused bf16 dlogits)
//   dH[b]  = (dz[b] . W) * (H[b] > 0 if relu_mask)         (the layer below's pre-activation grad)
//   dW    += dz^T H,  db += colsum(dz)                     (block partials folded in LDS, fp32 atomics)
// One wave per RPW rows: the wave loads its W panel (CT x K bf16) and all RPW rows of H up front
// (loads unconditional; rows past B re-read row B-1 and are masked), then each row's logits are a
// butterfly sum per class, the loss math runs redundantly in every lane (no LDS round trip) and the
// row's dH chunk is stored while its H chunk is still in registers.  NJ = K / 512 chunks per lane.
// The head's H is read once instead of three times and dz never goes through memory.
template <int CT, int NJ, int RPW, int NWV>
__global__ __launch_bounds__(64 * NWV) void skinny_head_kernel(const uint16_t* __restrict__ H,
                                                          const uint16_t* __restrict__ W,
                                                          const float* __restrict__ bias,
                                                          const int* __restrict__ labels, uint16_t* __restrict__ dH,
                                                          float* __restrict__ dW, float* __restrict__ db,
                                                          float* __restrict__ loss_sum, int B, int K, int C,
                                                          float grad_scale, int loss_kind, float loss_scale,
                                                          int relu_mask) {
  __shared__ float4 red4[NWV][CT][NJ * 128];  // per-wave dW partials, [wave][c][k / 4]
  __shared__ float red_s[NWV][CT + 1];        // per-wave db partials and loss
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r0 = (blockIdx.x * NWV + wv) * RPW;
  uint4 wraw[CT][NJ];
#pragma unroll
  for (int c = 0; c < CT; ++c)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
      wraw[c][j] = *reinterpret_cast<const uint4*>(W + (size_t)(c < C ? c : C - 1) * K + j * 512 + lane * 8);
  uint4 hraw[RPW][NJ];
  int ys[RPW];
#pragma unroll
  for (int i = 0; i < RPW; ++i) {
    const int r = min(r0 + i, B - 1);
    ys[i] = labels[r];
#pragma unroll
    for (int j = 0; j < NJ; ++j) hraw[i][j] = *reinterpret_cast<const uint4*>(H + (size_t)r * K + j * 512 + lane * 8);
  }
  float bs[CT];
#pragma unroll
  for (int c = 0; c < CT; ++c) bs[c] = bias ? bias[c < C ? c : C - 1] : 0.f;
  float acc[CT][NJ][8];
  float dbs[CT];
#pragma unroll
  for (int c = 0; c < CT; ++c) {
    dbs[c] = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[c][j][e] = 0.f;
  }
  float lsum = 0.f;
#pragma unroll
  for (int i = 0; i < RPW; ++i) {
    const bool ok = r0 + i < B;
    float h[NJ][8];
#pragma unroll
    for (int j = 0; j < NJ; ++j) unpack8(hraw[i][j], h[j]);
    float z[CT];
#pragma unroll
    for (int c = 0; c < CT; ++c) {
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        float w[8];
        unpack8(wraw[c][j], w);
#pragma unroll
        for (int e = 0; e < 8; ++e) s += h[j][e] * w[e];
      }
      z[c] = bf16_to_f32(f32_to_bf16(wave_sum(s) + bs[c]));
    }
    // loss + dlogits of the row, as dct::loss_kernel computes them (same formulas, fp32)
    const int y = ys[i];
    float dz[CT];
    float rl;
    if (loss_kind == 0) {
      float mx = z[0], zy = z[0];
#pragma unroll
      for (int c = 1; c < CT; ++c) {
        if (c < C && z[c] > mx) mx = z[c];
        if (c == y) zy = z[c];
      }
      float ex[CT], s = 0.f;
#pragma unroll
      for (int c = 0; c < CT; ++c) {
        ex[c] = c < C ? __expf(z[c] - mx) : 0.f;
        s += ex[c];
      }
      rl = mx + __logf(s) - zy;
      const float rs = 1.f / s;
#pragma unroll
      for (int c = 0; c < CT; ++c) dz[c] = (ex[c] * rs - (c == y ? 1.f : 0.f)) * grad_scale;
    } else {
      rl = 0.f;
#pragma unroll
      for (int c = 0; c < CT; ++c) {
        const float d = c < C ? z[c] - (c == y ? 1.f : 0.f) : 0.f;
        rl += d * d;
        dz[c] = 2.f * d * grad_scale / (float)C;
      }
      rl /= (float)C;
    }
#pragma unroll
    for (int c = 0; c < CT; ++c) dz[c] = (ok && c < C) ? bf16_to_f32(f32_to_bf16(dz[c])) : 0.f;
    lsum += ok ? rl : 0.f;
    // dH chunk of the row, then the dW / db contributions
    if (dH && ok) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        float o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = 0.f;
#pragma unroll
        for (int c = 0; c < CT; ++c) {
          float w[8];
          unpack8(wraw[c][j], w);
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] += dz[c] * w[e];
        }
        if (relu_mask) {
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = h[j][e] > 0.f ? o[e] : 0.f;
        }
        uint4 v;
        v.x = f32_to_bf16(o[0]) | ((uint32_t)f32_to_bf16(o[1]) << 16);
        v.y = f32_to_bf16(o[2]) | ((uint32_t)f32_to_bf16(o[3]) << 16);
        v.z = f32_to_bf16(o[4]) | ((uint32_t)f32_to_bf16(o[5]) << 16);
        v.w = f32_to_bf16(o[6]) | ((uint32_t)f32_to_bf16(o[7]) << 16);
        *reinterpret_cast<uint4*>(dH + (size_t)(r0 + i) * K + j * 512 + lane * 8) = v;
      }
    }
#pragma unroll
    for (int c = 0; c < CT; ++c) {
      dbs[c] += dz[c];
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[c][j][e] += dz[c] * h[j][e];
    }
  }
  // fold the NWV waves' partials in column order, one atomic per (class, column) per block
#pragma unroll
  for (int c = 0; c < CT; ++c)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      red4[wv][c][j * 128 + 2 * lane] = make_float4(acc[c][j][0], acc[c][j][1], acc[c][j][2], acc[c][j][3]);
      red4[wv][c][j * 128 + 2 * lane + 1] = make_float4(acc[c][j][4], acc[c][j][5], acc[c][j][6], acc[c][j][7]);
    }
  if (lane == 0) {
#pragma unroll
    for (int c = 0; c < CT; ++c) red_s[wv][c] = dbs[c];
    red_s[wv][CT] = lsum;
  }
  __syncthreads();
  const float* red = reinterpret_cast<const float*>(red4);
  constexpr int PER_WAVE = CT * NJ * 512;
#pragma unroll
  for (int c = 0; c < CT; ++c) {
    if (c >= C) break;
#pragma unroll
    for (int q = 0; q < 8 * NJ / NWV; ++q) {
      const int col = threadIdx.x + 64 * NWV * q;
      const int o = c * NJ * 512 + col;
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < NWV; ++w) v += red[w * PER_WAVE + o];
      atomicAdd(dW + (size_t)c * K + col, v);
    }
  }
  if (threadIdx.x < C && db) {
    const int c = threadIdx.x;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NWV; ++w) v += red_s[w][c];
    atomicAdd(db + c, v);
  }
  if (threadIdx.x == 64 && loss_sum) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NWV; ++w) v += red_s[w][CT];
    atomicAdd(loss_sum, v * loss_scale);
  }
}

}  // namespace dct

extern "C" {

int dct_skinny_fwd(const uint16_t* X, const uint16_t* W, const float* bias, uint16_t* Y, int B, int K, int C,
                   void* stream) {
  if (C > dct::SK_CMAX || C < 1 || K % 8 || (((uintptr_t)X | (uintptr_t)W) & 15)) return (int)hipErrorInvalidValue;
  if (B <= 0) return 0;
  const dim3 grid((B + 3) / 4);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (C == 1) hipLaunchKernelGGL(dct::skinny_fwd_kernel<1>, grid, dim3(256), 0, st, X, W, bias, Y, B, K, C);
  else if (C == 2) hipLaunchKernelGGL(dct::skinny_fwd_kernel<2>, grid, dim3(256), 0, st, X, W, bias, Y, B, K, C);
  else if (C <= 4) hipLaunchKernelGGL(dct::skinny_fwd_kernel<4>, grid, dim3(256), 0, st, X, W, bias, Y, B, K, C);
  else hipLaunchKernelGGL(dct::skinny_fwd_kernel<8>, grid, dim3(256), 0, st, X, W, bias, Y, B, K, C);
  return (int)hipGetLastError();
}

int dct_skinny_dx(const uint16_t* dZ, const uint16_t* W, const uint16_t* aux, uint16_t* dX, int B, int K, int C,
                  void* stream) {
  if (C > dct::SK_CMAX || C < 1 || K % 8 || (((uintptr_t)W | (uintptr_t)dX | (uintptr_t)aux) & 15))
    return (int)hipErrorInvalidValue;
  if (B <= 0) return 0;
  const int64_t total = (int64_t)B * (K / 8);
  int grid = (int)((total + 255) / 256);
  grid = grid > 4096 ? 4096 : grid;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (C == 1) hipLaunchKernelGGL(dct::skinny_dx_kernel<1>, dim3(grid), dim3(256), 0, st, dZ, W, aux, dX, B, K, C);
  else if (C == 2) hipLaunchKernelGGL(dct::skinny_dx_kernel<2>, dim3(grid), dim3(256), 0, st, dZ, W, aux, dX, B, K, C);
  else if (C <= 4) hipLaunchKernelGGL(dct::skinny_dx_kernel<4>, dim3(grid), dim3(256), 0, st, dZ, W, aux, dX, B, K, C);
  else hipLaunchKernelGGL(dct::skinny_dx_kernel<8>, dim3(grid), dim3(256), 0, st, dZ, W, aux, dX, B, K, C);
  return (int)hipGetLastError();
}

// Shapes the fused head covers (register budget: W panel + RPW rows of H + the dW partials stay
// resident): K a multiple of 512 with C <= 2 and K <= 2048, C <= 4 and K <= 1024, or C <= 8 and K = 512.
int dct_skinny_head_supported(int K, int C) {
  if (C < 1 || K < 512 || K % 512) return 0;
  return (C <= 2 && K <= 2048) || (C <= 4 && K <= 1024) || (C <= 8 && K == 512);
}

int dct_skinny_head(const uint16_t* H, const uint16_t* W, const float* bias, const int* labels, uint16_t* dH,
                    float* dW, float* db, float* loss_sum, int B, int K, int C, float grad_scale, int loss_kind,
                    float loss_scale, int relu_mask, void* stream) {
  if (!dct_skinny_head_supported(K, C) || !H || !W || !labels || !dW ||
      (((uintptr_t)H | (uintptr_t)W | (uintptr_t)dH) & 15))
    return (int)hipErrorInvalidValue;
  if (B <= 0) return 0;
  // two-class heads up to K = 1024: 8 waves x 4 rows (32 rows per block, 2 waves per SIMD) once
  // that still gives >= 128 blocks; otherwise 4 waves x 4 rows
  const bool w8 = C <= 2 && K <= 1024;  // 8-wave blocks: LDS partials 8 x C x K fp32 <= 64 KB
  // 4 rows per wave (2 and 8 measured no faster: profiles/skinny_dw_split_sweep_*_r1.txt)
  const int nwv = (w8 && B >= 128 * 32) ? 8 : 4;
  const dim3 grid((B + nwv * 4 - 1) / (nwv * 4));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int NJ = K / 512;
#define SKH_LAUNCH(CT_, NJ_, W_)                                                                             \
  hipLaunchKernelGGL((dct::skinny_head_kernel<CT_, NJ_, 4, W_>), grid, dim3(64 * W_), 0, st, H, W, bias, labels, \
                     dH, dW, db, loss_sum, B, K, C, grad_scale, loss_kind, loss_scale, relu_mask)
#define SKH_WAVES(CT_, NJ_)                 \
  if (nwv == 8) SKH_LAUNCH(CT_, NJ_, 8);   \
  else SKH_LAUNCH(CT_, NJ_, 4)
  if (C == 1) {
    switch (NJ) { case 1: SKH_WAVES(1, 1); break; case 2: SKH_WAVES(1, 2); break;
                  case 3: SKH_LAUNCH(1, 3, 4); break; default: SKH_LAUNCH(1, 4, 4); break; }
  } else if (C == 2) {
    switch (NJ) { case 1: SKH_WAVES(2, 1); break; case 2: SKH_WAVES(2, 2); break;
                  case 3: SKH_LAUNCH(2, 3, 4); break; default: SKH_LAUNCH(2, 4, 4); break; }
  } else if (C <= 4) {
    if (NJ == 1) SKH_LAUNCH(4, 1, 4); else SKH_LAUNCH(4, 2, 4);
  } else {
    SKH_LAUNCH(8, 1, 4);
  }
#undef SKH_WAVES
#undef SKH_LAUNCH
  return (int)hipGetLastError();
}

int dct_skinny_dw(const uint16_t* dZ, const uint16_t* X, float* dW, float* db, int B, int K, int C, void* stream) {
  if (C > dct::SK_CMAX || C < 1 || K % 8 || (((uintptr_t)X) & 15)) return (int)hipErrorInvalidValue;
  if (B <= 0) return 0;
  const int kb = (K + 511) / 512;
  // ~256 blocks of >= 64 rows: the row stream spread over every CU, few atomics per column
  int splits = (256 + kb - 1) / kb;
  const int max_splits = (B + 63) / 64;
  splits = splits > max_splits ? max_splits : splits;
  splits = splits < 1 ? 1 : splits;
  const int rows_per = (B + splits - 1) / splits;
  const dim3 grid(kb, (B + rows_per - 1) / rows_per);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (C == 1) hipLaunchKernelGGL(dct::skinny_dw_kernel<1>, grid, dim3(256), 0, st, dZ, X, dW, db, B, K, C, rows_per);
  else if (C == 2) hipLaunchKernelGGL(dct::skinny_dw_kernel<2>, grid, dim3(256), 0, st, dZ, X, dW, db, B, K, C, rows_per);
  else if (C <= 4) hipLaunchKernelGGL(dct::skinny_dw_kernel<4>, grid, dim3(256), 0, st, dZ, X, dW, db, B, K, C, rows_per);
  else hipLaunchKernelGGL(dct::skinny_dw_kernel<8>, grid, dim3(256), 0, st, dZ, X, dW, db, B, K, C, rows_per);
  return (int)hipGetLastError();
}

}  // extern "C"
