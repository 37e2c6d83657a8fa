// Shared helpers for the dct HIP kernels (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include "knobs.h"
#include <hip/hip_bf16.h>
#include <stdint.h>



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

// p[i] for a wave-uniform i, through the scalar cache: a peer buffer address loaded this way stays in
// SGPRs, so the buffer descriptor built from it is scalar.  Loaded with a vector load instead, the
// descriptor lands in VGPRs and every buffer op on it becomes a readfirstlane / compare / exec-mask
// waterfall loop (~13 extra instructions per store) holding 4 VGPRs per peer.
template <class T>
__device__ __forceinline__ T* sload_ptr(T* const* p, int i) {
  return (T*)((const __attribute__((address_space(4))) unsigned long long*)p)[i];
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

// erf(x) by Abramowitz-Stegun 7.1.26 (|err| < 6e-7 in fp32) on one v_rcp_f32 + one v_exp_f32,
// given e = exp(-x^2).  The ocml erff is ~44 VALU ops with range branches; GEMM epilogues that
// apply GELU to every output element were bound by it.
__device__ __forceinline__ float erf_exp(float x, float e) {
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, fabsf(x), 1.f));
  const float p = fmaf(fmaf(fmaf(fmaf(1.061405429f, t, -1.453152027f), t, 1.421413741f), t, -0.284496736f), t,
                       0.254829592f) * t;
  return copysignf(1.f - p * e, x);
}
// exact-form (erf) GELU and its derivative; both share exp(-z^2/2) between erf and the pdf
__device__ __forceinline__ float gelu_f(float z) {
  const float x = z * 0.70710678118654752f;
  const float e = __builtin_amdgcn_exp2f(-x * x * 1.4426950408889634f);
  return 0.5f * z * (1.f + erf_exp(x, e));
}
__device__ __forceinline__ float gelu_grad_f(float z) {
  const float x = z * 0.70710678118654752f;
  const float e = __builtin_amdgcn_exp2f(-x * x * 1.4426950408889634f);
  return 0.5f * (1.f + erf_exp(x, e)) + z * 0.3989422804014327f * e;
}

}  // namespace dct
