// Shared helpers for the dct HIP kernels (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#define DCT_WAVE 64

namespace dct {

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  return v;
}

// bf16 <-> f32 on raw 16-bit storage (round-to-nearest-even; NaN kept NaN via the cast path)
__device__ __forceinline__ float bf16_to_f32(uint16_t h) {
  return __uint_as_float(((uint32_t)h) << 16);
}
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  return __bfloat16_as_ushort(__float2bfloat16(f));
}

// b^t for Adam's bias corrections as ONE v_exp_f32: 2^(t log2 b) with log2 b hoisted out of the
// step loop.  (__powf lowers to the full-precision libm sequence - a few hundred instructions
// per call, which was ~40 % of a 2.3 us single-wave optimizer step.)
__device__ __forceinline__ float pow_t(float log2b, float t) { return __builtin_amdgcn_exp2f(t * log2b); }

}  // namespace dct
