// Tabular classifier head (B = 4096 rows, K = 1024, C = 2): where do the fused skinny_head
// kernel's ~10.5 us go?  Its 128 blocks each fold their dW partial (C x K fp32) into dW with
// C * K device-scope float atomics, i.e. 128 atomics on every one of the 2048 dW words.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I<pkg>/csrc tools/probes/head_reduce_probe.hip \
//         <pkg>/csrc/knobs.cpp -o build/head_reduce_probe && ./build/head_reduce_probe
//
// Variants timed (200 back-to-back launches, hipEvents):
//   prod      dct_skinny_head (csrc/skinny.hip) as the step executor launches it
//   stage1    the same kernel body, each block storing its partial to a [block][C x K] workspace
//   two-pass  stage1 + a column reduce over the blocks (deterministic, one plain add per word)
// and the two-pass dW / dH / loss are checked against prod's.
#include "skinny.hip"

#include <cmath>
#include <cstdio>
#include <vector>

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__); \
      exit(1);                                                              \
    }                                                                       \
  } while (0)

namespace probe {
using namespace dct;

// skinny_head_kernel<2, 2, 4, 8> with the dW fold stored per block instead of atomically added
template <int CT, int NJ, int RPW, int NWV>
__global__ __launch_bounds__(64 * NWV) void head_stage1(const uint16_t* __restrict__ H, const uint16_t* __restrict__ W,
                                                        const float* __restrict__ bias, const int* __restrict__ labels,
                                                        uint16_t* __restrict__ dH, float* __restrict__ part,
                                                        float* __restrict__ db, float* __restrict__ loss_sum, int B,
                                                        int K, int C, float grad_scale, float loss_scale) {
  __shared__ float4 red4[NWV][CT][NJ * 128];
  __shared__ float red_s[NWV][CT + 1];
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
  for (int c = 0; c < CT; ++c) bs[c] = bias[c < C ? c : C - 1];
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
    const int y = ys[i];
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
    const float rl = mx + __logf(s) - zy;
    const float rs = 1.f / s;
    float dz[CT];
#pragma unroll
    for (int c = 0; c < CT; ++c) dz[c] = (ex[c] * rs - (c == y ? 1.f : 0.f)) * grad_scale;
#pragma unroll
    for (int c = 0; c < CT; ++c) dz[c] = (ok && c < C) ? bf16_to_f32(f32_to_bf16(dz[c])) : 0.f;
    lsum += ok ? rl : 0.f;
    if (ok) {
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
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = h[j][e] > 0.f ? o[e] : 0.f;
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
  float* mine = part + (size_t)blockIdx.x * C * K;
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
      mine[c * K + col] = v;
    }
  }
  if (threadIdx.x < C) {
    const int c = threadIdx.x;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NWV; ++w) v += red_s[w][c];
    atomicAdd(db + c, v);
  }
  if (threadIdx.x == 64) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NWV; ++w) v += red_s[w][CT];
    atomicAdd(loss_sum, v * loss_scale);
  }
}

// dW[col] += sum_b part[b][col]: 64 columns per block, 8 waves over the blocks' rows, folded in LDS
__global__ __launch_bounds__(512) void head_stage2(const float* __restrict__ part, float* __restrict__ dW, int nblk,
                                                   int n) {
  __shared__ float red[8][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (col < n)
    for (int b = wv; b < nblk; b += 8) s += part[(size_t)b * n + col];
  red[wv][lane] = s;
  __syncthreads();
  if (wv == 0 && col < n) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) v += red[w][lane];
    dW[col] += v;
  }
}
}  // namespace probe

static uint16_t f2bf_h(float f) {
  uint32_t u = __builtin_bit_cast(uint32_t, f);
  u += 0x7fff + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}

int main() {
  const int B = 4096, K = 1024, C = 2, NWV = 8, RPW = 4;
  const int nblk = B / (NWV * RPW);
  std::vector<uint16_t> hH((size_t)B * K), hW((size_t)C * K);
  std::vector<int> hy(B);
  uint32_t st = 12345;
  auto rnd = [&]() { st = st * 1664525u + 1013904223u; return ((st >> 8) & 0xffff) / 65536.f - 0.5f; };
  for (auto& v : hH) { float x = rnd(); v = f2bf_h(x > 0 ? 2 * x : 0.f); }
  for (auto& v : hW) v = f2bf_h(0.06f * rnd());
  for (int i = 0; i < B; ++i) hy[i] = (st = st * 1664525u + 1013904223u) >> 31;
  uint16_t *H, *W, *dH1, *dH2;
  float *bias, *dW1, *dW2, *db1, *db2, *l1, *l2, *part;
  int* y;
  CK(hipMalloc(&H, (size_t)B * K * 2));
  CK(hipMalloc(&W, (size_t)C * K * 2));
  CK(hipMalloc(&dH1, (size_t)B * K * 2));
  CK(hipMalloc(&dH2, (size_t)B * K * 2));
  CK(hipMalloc(&bias, C * 4));
  CK(hipMalloc(&dW1, C * K * 4));
  CK(hipMalloc(&dW2, C * K * 4));
  CK(hipMalloc(&db1, C * 4));
  CK(hipMalloc(&db2, C * 4));
  CK(hipMalloc(&l1, 4));
  CK(hipMalloc(&l2, 4));
  CK(hipMalloc(&part, (size_t)nblk * C * K * 4));
  CK(hipMalloc(&y, B * 4));
  CK(hipMemcpy(H, hH.data(), hH.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(W, hW.data(), hW.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(y, hy.data(), B * 4, hipMemcpyHostToDevice));
  CK(hipMemset(bias, 0, C * 4));
  const float gs = 1.f / B;
  auto prod = [&]() {
    if (dct_skinny_head(H, W, bias, y, dH1, dW1, db1, l1, B, K, C, gs, 0, gs, 1, nullptr)) exit(2);
  };
  auto s1 = [&]() {
    hipLaunchKernelGGL((probe::head_stage1<2, 2, 4, 8>), dim3(nblk), dim3(512), 0, nullptr, H, W, bias, y, dH2, part,
                       db2, l2, B, K, C, gs, gs);
  };
  auto s2 = [&]() { hipLaunchKernelGGL(probe::head_stage2, dim3(C * K / 64), dim3(512), 0, nullptr, part, dW2, nblk, C * K); };
  auto two = [&]() { s1(); s2(); };
  auto timeit = [&](auto fn) {
    for (int i = 0; i < 10; ++i) fn();
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    for (int i = 0; i < 200; ++i) fn();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e3f / 200;
  };
  // one clean launch of each for the numerics check
  CK(hipMemset(dW1, 0, C * K * 4)); CK(hipMemset(dW2, 0, C * K * 4));
  CK(hipMemset(db1, 0, C * 4)); CK(hipMemset(db2, 0, C * 4));
  CK(hipMemset(l1, 0, 4)); CK(hipMemset(l2, 0, 4));
  prod();
  two();
  CK(hipDeviceSynchronize());
  std::vector<float> a(C * K), b(C * K);
  std::vector<uint16_t> ha((size_t)B * K), hb((size_t)B * K);
  CK(hipMemcpy(a.data(), dW1, C * K * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(b.data(), dW2, C * K * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(ha.data(), dH1, ha.size() * 2, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hb.data(), dH2, hb.size() * 2, hipMemcpyDeviceToHost));
  float la, lb;
  CK(hipMemcpy(&la, l1, 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&lb, l2, 4, hipMemcpyDeviceToHost));
  double md = 0, mx = 0;
  for (int i = 0; i < C * K; ++i) { md = fmax(md, fabs(a[i] - b[i])); mx = fmax(mx, fabs(a[i])); }
  size_t dh_diff = 0;
  for (size_t i = 0; i < ha.size(); ++i) dh_diff += ha[i] != hb[i];
  printf("check: max|dW prod - two-pass| = %.3g (max|dW| %.3g), dH words differing %zu, loss %.6f vs %.6f\n", md, mx,
         dh_diff, la, lb);
  printf("prod (atomics)   %7.2f us\n", timeit(prod));
  printf("stage1 only      %7.2f us\n", timeit(s1));
  printf("stage2 only      %7.2f us\n", timeit(s2));
  printf("two-pass         %7.2f us\n", timeit(two));
  return 0;
}
