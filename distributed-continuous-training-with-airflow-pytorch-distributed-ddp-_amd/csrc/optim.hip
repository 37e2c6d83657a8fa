// Fused flat-buffer Adam for MI355X.
//
// Replaces torch.optim.Adam's per-parameter loop (reference train_lightning_ddp.py:88,
// torch 2.1 single-tensor implementation on CPU). All parameters of a model live in ONE
// flat fp32 buffer (the DDP gradient buckets are views of the matching flat grad buffer),
// so one launch updates every parameter: float4 loads, grid sized to the chip
// (<= 2048 workgroups, grid-stride), bias correction folded into two scalars.
// Optional outputs: a bf16 shadow copy of the updated weights for the MFMA GEMM path, and
// gradient pre-scaling (e.g. 1/world_size when the all-reduce summed).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "dct_common.h"

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

template <bool PARTS, int S = 4>
__global__ __launch_bounds__(256) void adam_flat_kernel(AdamArgs a) {
  if (a.cursor && blockIdx.x == 0 && threadIdx.x == 0) {
    const int c = a.cursor[0];
    if (a.loss_out && c >= 0 && c < a.loss_cap) a.loss_out[c] = a.loss_slot[0];
    a.cursor[0] = c + 1;
  }
  if (a.step_counter) {
    const float t = (float)__hip_atomic_load(a.step_counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    a.step_size = a.lr / (1.f - pow_t(log2f(a.b1), t));
    a.rbc2 = rsqrtf(1.f - pow_t(log2f(a.b2), t));
  }
  const int64_t n4 = a.n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  float4* p4 = reinterpret_cast<float4*>(a.p);
  const float4* g4 = reinterpret_cast<const float4*>(a.g);
  float4* m4 = reinterpret_cast<float4*>(a.m);
  float4* v4 = reinterpret_cast<float4*>(a.v);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
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
  // tail (n % 4)
  const int64_t tail0 = n4 << 2;
  const int64_t gt = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gt < a.n - tail0) {
    const int64_t i = tail0 + gt;
    float p = a.p[i], m = a.m[i], v = a.v[i];
    adam_one(p, a.g[i], m, v, a);
    a.p[i] = p;
    a.m[i] = m;
    a.v[i] = v;
    if (a.p_bf16) a.p_bf16[i] = f32_to_bf16(p);
  }
}

// out = in * scale (+ optional bf16 cast) - used to average summed gradients and to refresh
// bf16 weight shadows after a checkpoint load.
__global__ __launch_bounds__(256) void f32_to_bf16_kernel(const float* in, uint16_t* out, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = f32_to_bf16(in[i]);
}

}  // namespace dct

static inline int grid_for(int64_t work, int block) {
  int64_t g = (work + block - 1) / block;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

extern "C" {

int dct_adam_flat_step(float* p, const float* g, float* m, float* v, uint16_t* p_bf16, int64_t n, float lr,
                       float b1, float b2, float eps, float wd, int64_t t, float grad_scale, int decoupled,
                       const int* step_counter, int* cursor, const float* loss_slot, float* loss_out, int loss_cap,
                       void* stream) {
  if (n <= 0) return 0;
  if (cursor && !loss_slot) return (int)hipErrorInvalidValue;
  if (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) return (int)hipErrorInvalidValue;
  dct::AdamArgs a{};
  a.p = p; a.g = g; a.m = m; a.v = v; a.p_bf16 = p_bf16; a.n = n;
  a.lr = lr; a.b1 = b1; a.b2 = b2; a.eps = eps; a.wd = wd;
  const double bc1 = 1.0 - __builtin_pow((double)b1, (double)t);
  const double bc2 = 1.0 - __builtin_pow((double)b2, (double)t);
  a.step_size = (float)(lr / bc1);
  a.rbc2 = (float)(1.0 / __builtin_sqrt(bc2));
  a.grad_scale = grad_scale;
  a.decoupled = decoupled;
  a.step_counter = step_counter;
  a.cursor = cursor;
  a.loss_slot = loss_slot;
  a.loss_out = loss_out;
  a.loss_cap = loss_cap;
  hipLaunchKernelGGL(dct::adam_flat_kernel<false>, dim3(grid_for((n + 3) / 4, 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), a);
  return (int)hipGetLastError();
}

// dct_adam_flat_step with up to three gradient ranges read from split-K partials of up to 8 slices
// (see AdamArgs)
int dct_adam_flat_step_parts(float* p, const float* g, float* m, float* v, uint16_t* p_bf16, int64_t n, float lr,
                             float b1, float b2, float eps, float wd, float grad_scale, int decoupled,
                             const int* step_counter, int* cursor, const float* loss_slot, float* loss_out,
                             int loss_cap, int nparts, const int64_t* part_off, const int64_t* part_n,
                             const float* const* part, const int* part_splits, void* stream) {
  if (n <= 0) return 0;
  if (!step_counter || (cursor && !loss_slot) || nparts < 0 || nparts > 3) return (int)hipErrorInvalidValue;
  if (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) return (int)hipErrorInvalidValue;
  dct::AdamArgs a{};
  a.p = p; a.g = g; a.m = m; a.v = v; a.p_bf16 = p_bf16; a.n = n;
  a.lr = lr; a.b1 = b1; a.b2 = b2; a.eps = eps; a.wd = wd;
  a.grad_scale = grad_scale;
  a.decoupled = decoupled;
  a.step_counter = step_counter;
  a.cursor = cursor;
  a.loss_slot = loss_slot;
  a.loss_out = loss_out;
  a.loss_cap = loss_cap;
  a.nparts = nparts;
  int max_sp = 1;
  for (int r = 0; r < nparts; ++r) {
    if ((part_off[r] | part_n[r]) & 3 || part_off[r] + part_n[r] > (n & ~3LL) || ((uintptr_t)part[r] & 15) ||
        part_splits[r] < 1 || part_splits[r] > 8)
      return (int)hipErrorInvalidValue;
    a.part_off[r] = part_off[r]; a.part_n[r] = part_n[r]; a.part[r] = part[r]; a.part_splits[r] = part_splits[r];
    max_sp = std::max(max_sp, part_splits[r]);
  }
  const dim3 grid(grid_for((n + 3) / 4, 256));
  if (max_sp > 4)
    hipLaunchKernelGGL((dct::adam_flat_kernel<true, 8>), grid, dim3(256), 0, reinterpret_cast<hipStream_t>(stream), a);
  else
    hipLaunchKernelGGL((dct::adam_flat_kernel<true, 4>), grid, dim3(256), 0, reinterpret_cast<hipStream_t>(stream), a);
  return (int)hipGetLastError();
}

int dct_adam_flat(float* p, const float* g, float* m, float* v, uint16_t* p_bf16, int64_t n, float lr,
                  float b1, float b2, float eps, float wd, int64_t t, float grad_scale, int decoupled,
                  const int* step_counter, void* stream) {
  return dct_adam_flat_step(p, g, m, v, p_bf16, n, lr, b1, b2, eps, wd, t, grad_scale, decoupled, step_counter,
                            nullptr, nullptr, nullptr, 0, stream);
}

int dct_f32_to_bf16(const float* in, uint16_t* out, int64_t n, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(dct::f32_to_bf16_kernel, dim3(grid_for(n, 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), in, out, n);
  return (int)hipGetLastError();
}

}  // extern "C"
