// Flat-buffer Adam device code (the fused optimizer of every engine), shared by optim.hip (the
// standalone launches) and gemm_bf16.hip (Adam ranges riding in the wide-MLP executor's dW GEMM
// launches, mlp_executor.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dct_common.h"
#include "kernels.h"

namespace dct {

struct AdamArgs {
  float* p;
  const float* g;
  float* m;
  float* v;
  uint16_t* p_bf16;  // optional shadow copy
  int64_t n;
  float lr, b1, b2, eps, wd;
  float step_size;  // lr / (1 - b1^t)
  float rbc2;       // 1 / sqrt(1 - b2^t)
  float grad_scale;
  int decoupled;  // 1 = AdamW
  const int* step_counter;  // optional: t read on device (graph-replayable launches)
  // optional step epilogue of the graph-captured MLP step (folded in to save a launch per step):
  // loss_out[*cursor] = *loss_slot (the all-reduced batch loss), then *cursor += 1
  int* cursor;
  const float* loss_slot;
  float* loss_out;
  int loss_cap;
  // optional (adam_flat_kernel<true, S>): split-K partials, <= S (4 or 8) slices, standing in for g
  // over up to three whole float4-aligned ranges (the wide-MLP executor's dW GEMMs without a DDP
  // reducer): g[off + e] = sum_s part[r][s * n + e] in slice order, the values the reduce pass would store
  int nparts;
  int64_t part_off[3], part_n[3];
  const float* part[3];
  int part_splits[3];
};

__device__ __forceinline__ void adam_one(float& p, float g, float& m, float& v, const AdamArgs& a) {
  g *= a.grad_scale;
  if (a.decoupled) {
    p -= a.lr * a.wd * p;
  } else {
    g += a.wd * p;
  }
  m = a.b1 * m + (1.f - a.b1) * g;
  v = a.b2 * v + (1.f - a.b2) * g * g;
  const float denom = sqrtf(v) * a.rbc2 + a.eps;
  p -= a.step_size * m / denom;
}

// step_size / rbc2 from the device step counter t (graph-replayable launches)
__device__ __forceinline__ void adam_bias_correction(AdamArgs& a) {
  const float t = (float)__hip_atomic_load(a.step_counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  a.step_size = a.lr / (1.f - pow_t(log2f(a.b1), t));
  a.rbc2 = rsqrtf(1.f - pow_t(log2f(a.b2), t));
}

// elements [lo, hi) of the flat buffers (lo % 4 == 0; hi == n or hi % 4 == 0), worked by workgroups
// blk = 0 .. nblk - 1 of the launch (grid-stride over float4s, the n % 4 tail by the last range)
// One element per thread and iteration (no float4): the Adam ranges riding in the dW GEMM launches
// (gemm2_dw_adam_kernel).  There the float4 path's paired component math (v_pk_* ops) went wrong
// for the low component of 16 lanes now and then while the GEMM's MFMA waves shared the SIMD
// (16 of 1 M W1 elements updated with denom = eps in one step, profiles/adam_ride_debug_r5.log);
// scalar code has nothing to pair, and its per-element arithmetic is the float4 path's, bit for bit.
template <bool PARTS, int S = 4>
__device__ __forceinline__ void adam_scalar_range(AdamArgs a, int64_t lo, int64_t hi, int blk, int nblk) {
  bool pending = a.step_counter != nullptr;
  const int64_t end = hi < a.n ? hi : a.n;
  const int64_t stride = (int64_t)nblk * blockDim.x;
  for (int64_t e = lo + (int64_t)blk * blockDim.x + threadIdx.x; e < end; e += stride) {
    float p = a.p[e], m = a.m[e], v = a.v[e];
    float g;
    if constexpr (!PARTS) {
      g = a.g[e];
    } else {
      const bool in0 = a.nparts > 0 && e >= a.part_off[0] && e < a.part_off[0] + a.part_n[0];
      const bool in1 = a.nparts > 1 && e >= a.part_off[1] && e < a.part_off[1] + a.part_n[1];
      const bool in2 = a.nparts > 2 && e >= a.part_off[2] && e < a.part_off[2] + a.part_n[2];
      const bool in = in0 || in1 || in2;
      const float* ps = in2 ? a.part[2] : (in1 ? a.part[1] : a.part[0]);
      const int64_t nr = in2 ? a.part_n[2] : (in1 ? a.part_n[1] : a.part_n[0]);
      const int64_t er = e - (in2 ? a.part_off[2] : (in1 ? a.part_off[1] : a.part_off[0]));
      const int sp = in ? (in2 ? a.part_splits[2] : (in1 ? a.part_splits[1] : a.part_splits[0])) : 1;
      const float* q0 = in ? ps + er : a.g + e;
      float vs[S];
#pragma unroll
      for (int q = 0; q < S; ++q) vs[q] = *((in && q < sp) ? ps + q * nr + er : q0);
      g = vs[0];
#pragma unroll
      for (int q = 1; q < S; ++q) g += q < sp ? vs[q] : 0.f;
    }
    if (pending) {
      adam_bias_correction(a);
      pending = false;
    }
    adam_one(p, g, m, v, a);
    a.p[e] = p;
    a.m[e] = m;
    a.v[e] = v;
    if (a.p_bf16) a.p_bf16[e] = f32_to_bf16(p);
  }
}

template <bool PARTS, int S = 4>
__device__ __forceinline__ void adam_flat_range(AdamArgs a, int64_t lo, int64_t hi, int blk, int nblk) {
  if (a.cursor && blk == 0 && threadIdx.x == 0) {
    const int c = a.cursor[0];
    if (a.loss_out && c >= 0 && c < a.loss_cap) a.loss_out[c] = a.loss_slot[0];
    a.cursor[0] = c + 1;
  }
  // the device step count is read AFTER the first element's loads are issued (first pass of the loop),
  // so its memory round trip overlaps theirs: one latency before the first store instead of two
  // (a 17.7 k-parameter launch is all latency: ~4.6 -> see BASELINE.md)
  bool pending = a.step_counter != nullptr;
  const int64_t n4 = (hi < a.n ? hi : a.n) >> 2;
  const int64_t stride = (int64_t)nblk * blockDim.x;
  float4* p4 = reinterpret_cast<float4*>(a.p);
  const float4* g4 = reinterpret_cast<const float4*>(a.g);
  float4* m4 = reinterpret_cast<float4*>(a.m);
  float4* v4 = reinterpret_cast<float4*>(a.v);
  for (int64_t i = (lo >> 2) + (int64_t)blk * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 p = p4[i], m = m4[i], v = v4[i];
    float4 g;
    if constexpr (!PARTS) {
      g = g4[i];
    } else {
      // every load unconditional (selected addresses, masked values): a load behind a branch
      // drains the load queue (s_waitcnt vmcnt(0)); slices summed in order, as the reduce does
      const int64_t e = 4 * i;
      // (selects, not a runtime index into the by-value kernel arguments: that would copy them to scratch)
      const bool in0 = a.nparts > 0 && e >= a.part_off[0] && e < a.part_off[0] + a.part_n[0];
      const bool in1 = a.nparts > 1 && e >= a.part_off[1] && e < a.part_off[1] + a.part_n[1];
      const bool in2 = a.nparts > 2 && e >= a.part_off[2] && e < a.part_off[2] + a.part_n[2];
      const bool in = in0 || in1 || in2;
      const float4* ps = reinterpret_cast<const float4*>(in2 ? a.part[2] : (in1 ? a.part[1] : a.part[0]));
      const int64_t n4r = (in2 ? a.part_n[2] : (in1 ? a.part_n[1] : a.part_n[0])) >> 2;
      const int64_t e4 = (e - (in2 ? a.part_off[2] : (in1 ? a.part_off[1] : a.part_off[0]))) >> 2;
      const int sp = in ? (in2 ? a.part_splits[2] : (in1 ? a.part_splits[1] : a.part_splits[0])) : 1;
      const float4* q0 = in ? ps + e4 : g4 + i;
      float4 vs[S];
#pragma unroll
      for (int q = 0; q < S; ++q) vs[q] = *((in && q < sp) ? ps + q * n4r + e4 : q0);
      g = vs[0];
#pragma unroll
      for (int q = 1; q < S; ++q) {
        const bool t = q < sp;
        g.x += t ? vs[q].x : 0.f;
        g.y += t ? vs[q].y : 0.f;
        g.z += t ? vs[q].z : 0.f;
        g.w += t ? vs[q].w : 0.f;
      }
    }
    if (pending) {
      adam_bias_correction(a);
      pending = false;
    }
    adam_one(p.x, g.x, m.x, v.x, a);
    adam_one(p.y, g.y, m.y, v.y, a);
    adam_one(p.z, g.z, m.z, v.z, a);
    adam_one(p.w, g.w, m.w, v.w, a);
    p4[i] = p;
    m4[i] = m;
    v4[i] = v;
    if (a.p_bf16) {
      ushort4 h;
      h.x = f32_to_bf16(p.x);
      h.y = f32_to_bf16(p.y);
      h.z = f32_to_bf16(p.z);
      h.w = f32_to_bf16(p.w);
      reinterpret_cast<ushort4*>(a.p_bf16)[i] = h;
    }
  }
  // tail (n % 4), by the range that ends the buffer
  const int64_t tail0 = (a.n >> 2) << 2;
  const int64_t gt = (int64_t)blk * blockDim.x + threadIdx.x;
  if (hi >= a.n && gt < a.n - tail0) {
    if (pending) adam_bias_correction(a);
    const int64_t i = tail0 + gt;
    float p = a.p[i], m = a.m[i], v = a.v[i];
    adam_one(p, a.g[i], m, v, a);
    a.p[i] = p;
    a.m[i] = m;
    a.v[i] = v;
    if (a.p_bf16) a.p_bf16[i] = f32_to_bf16(p);
  }
}

template <bool PARTS, int S = 4>
__global__ __launch_bounds__(256) void adam_flat_kernel(AdamArgs a) {
  adam_flat_range<PARTS, S>(a, 0, a.n, blockIdx.x, gridDim.x);
}

template <int S>
__global__ __launch_bounds__(256) void adam_range_kernel(AdamArgs a, int64_t lo, int64_t hi) {
  adam_flat_range<true, S>(a, lo, hi, blockIdx.x, gridDim.x);
}

// AdamArgs of an AdamRange (kernels.h), validated; *max_sp = the deepest slice count (S of the kernel)
inline int adam_args_from_range(const AdamRange& r, AdamArgs& a, int* max_sp) {
  if (r.n <= 0 || r.lo < 0 || r.lo % 4 || r.hi > r.n || r.lo >= r.hi || (r.hi % 4 && r.hi != r.n) || !r.step_counter ||
      r.nparts < 0 || r.nparts > 3 || (((uintptr_t)r.p | (uintptr_t)r.g | (uintptr_t)r.m | (uintptr_t)r.v) & 15))
    return (int)hipErrorInvalidValue;
  a = AdamArgs{};
  a.p = r.p; a.g = r.g; a.m = r.m; a.v = r.v; a.p_bf16 = r.p_bf16; a.n = r.n;
  a.lr = r.lr; a.b1 = r.b1; a.b2 = r.b2; a.eps = r.eps; a.wd = r.wd;
  a.grad_scale = r.grad_scale;
  a.decoupled = r.decoupled;
  a.step_counter = r.step_counter;
  a.nparts = r.nparts;
  *max_sp = 1;
  for (int q = 0; q < r.nparts; ++q) {
    if ((r.part_off[q] | r.part_n[q]) & 3 || r.part_off[q] + r.part_n[q] > (r.n & ~3LL) || ((uintptr_t)r.part[q] & 15) ||
        r.part_splits[q] < 1 || r.part_splits[q] > 8)
      return (int)hipErrorInvalidValue;
    a.part_off[q] = r.part_off[q]; a.part_n[q] = r.part_n[q]; a.part[q] = r.part[q]; a.part_splits[q] = r.part_splits[q];
    *max_sp = r.part_splits[q] > *max_sp ? r.part_splits[q] : *max_sp;
  }
  return 0;
}

}  // namespace dct
