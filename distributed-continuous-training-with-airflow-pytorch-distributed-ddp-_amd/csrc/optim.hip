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

#include "adam_impl.h"
#include "dct_common.h"
#include "kernels.h"

namespace dct {

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

int dct_adam_range(const dct::AdamRange* r, int* cursor, const float* loss_slot, float* loss_out, int loss_cap,
                   void* stream) {
  dct::AdamArgs a{};
  int max_sp = 1;
  const int e = dct::adam_args_from_range(*r, a, &max_sp);
  if (e) return e;
  if (cursor && !loss_slot) return (int)hipErrorInvalidValue;
  a.cursor = cursor;
  a.loss_slot = loss_slot;
  a.loss_out = loss_out;
  a.loss_cap = loss_cap;
  const dim3 grid(grid_for((r->hi - r->lo + 3) / 4, 256));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (max_sp > 4) hipLaunchKernelGGL((dct::adam_range_kernel<8>), grid, dim3(256), 0, st, a, r->lo, r->hi);
  else hipLaunchKernelGGL((dct::adam_range_kernel<4>), grid, dim3(256), 0, st, a, r->lo, r->hi);
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
