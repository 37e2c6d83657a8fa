// Wave-level building blocks of the register-resident 3x128 trainers (mlp_block3.hip): DPP /
// permlane reductions, the folded Adam update, 4x4x1 fp32 MFMA, scalar-cache loads and the
// swizzled LDS staging of a 128x128 fp32 block.  gfx950 only.
#pragma once
#include "mlp_fused_impl.h"

namespace dct {
namespace bku {

constexpr int QP_X1 = 0xB1;     // quad_perm [1,0,3,2]: lane ^ 1
constexpr int QP_X2 = 0x4E;     // quad_perm [2,3,0,1]: lane ^ 2
constexpr int ROR4 = 0x124;     // row_ror:4 (lane i of a 16-lane row reads lane (i - 4) % 16: tools/probes/dpp_dir_probe)
constexpr int ROR8 = 0x128;     // row_ror:8 == lane ^ 8 inside a 16-lane row
constexpr int HMIRROR = 0x141;  // row_half_mirror: lane i <-> 7 - i inside each 8 lanes (lane ^ 7)
constexpr int QB0 = 0x00, QB1 = 0x55, QB2 = 0xAA, QB3 = 0xFF;  // quad broadcast of lane 0..3

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  // every control used here reads a valid lane of the same row: bound_ctrl lets the compiler fold
  // the move into the consuming VALU op (v_add_f32_dpp) instead of copying the operand first
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ float quad_bcast(float v, int c) {
  return c == 0 ? dpp<QB0>(v) : (c == 1 ? dpp<QB1>(v) : (c == 2 ? dpp<QB2>(v) : dpp<QB3>(v)));
}

// Adam with the step size folded into the denominator: p -= m / (sqrt(v) * A + E), A = rbc2 / ss,
// E = eps / ss (ss = lr / (1 - b1^t), rbc2 = 1 / sqrt(1 - b2^t)) - torch's update up to rounding;
// m moves like torch's lerp_(g, 1 - b1).  WD = false drops the L2 term (wd == 0: one op less).
template <bool WD>
__device__ __forceinline__ void adam_lean(float& p, float g, float& m, float& v, float c1, float b2, float c2,
                                          float wd, float A, float E) {
  if constexpr (WD) g = fmaf(wd, p, g);
  m = fmaf(c1, g - m, m);
  v = fmaf(c2 * g, g, v * b2);
  p = fmaf(-m, __builtin_amdgcn_rcpf(fmaf(__builtin_amdgcn_sqrtf(v), A, E)), p);
}

// The same update on SCALED moments mh = m / (1 - b1), vh = v / (1 - b2) (converted on load and
// store): mh' = b1 mh + g, vh' = b2 vh + g^2 - one op less each; A and E absorb the scales:
// A = sqrt(1 - b2) rbc2 / (ss (1 - b1)), E = eps / (ss (1 - b1)).  7 VALU ops (2 transcendental).
template <bool WD>
__device__ __forceinline__ void adam_scaled(float& p, float g, float& mh, float& vh, float b1, float b2, float wd,
                                            float A, float E) {
  if constexpr (WD) g = fmaf(wd, p, g);
  mh = fmaf(b1, mh, g);
  vh = fmaf(b2, vh, g * g);
  p = fmaf(-mh, __builtin_amdgcn_rcpf(fmaf(__builtin_amdgcn_sqrtf(vh), A, E)), p);
}

__device__ __forceinline__ float swap32_sum(float lo, float hi) {
  // lanes 0-31 get lo(own) + lo(partner), lanes 32-63 hi(partner) + hi(own)
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(lo), __float_as_uint(hi), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float swap16_sum(float lo, float hi) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(lo), __float_as_uint(hi), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// Wave reduce-scatter of N = 8 or 16 per-lane values: afterwards lane l holds the wave sum of
// value l >> 3 (N = 8) or l >> 2 (N = 16), i.e. DPP row r holds values [N/4 r, N/4 (r+1)).
// Levels: lane bit 5 (v_permlane32_swap), 4 (v_permlane16_swap), 3 (row_ror 8 = lane ^ 8),
// [N = 16: bit 2 via row_half_mirror, partner lane ^ 7, which agrees on bits 5..3], then an
// all-reduce over the remaining low bits; every partner agrees on the bits already decided, so
// each kept value sums disjoint lane sets and the last one covers all 64 lanes.
template <int N>
__device__ __forceinline__ float rs_small(float (&P)[N], int lane) {
  static_assert(N == 8 || N == 16, "");
#pragma unroll
  for (int i = 0; i < N / 2; ++i) P[i] = swap32_sum(P[i], P[i + N / 2]);
#pragma unroll
  for (int i = 0; i < N / 4; ++i) P[i] = swap16_sum(P[i], P[i + N / 4]);
  const bool b3 = (lane >> 3) & 1;
  float r;
  if constexpr (N == 8) {
    const float keep = b3 ? P[1] : P[0], send = b3 ? P[0] : P[1];
    r = keep + dpp<ROR8>(send);
    r += dpp<QP_X1>(r);
    r += dpp<QP_X2>(r);
    r += dpp<HMIRROR>(r);  // quads are uniform now: the mirror pairs quad 0 with quad 1
  } else {
    const bool b2 = (lane >> 2) & 1;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const float keep = b3 ? P[i + 2] : P[i], send = b3 ? P[i] : P[i + 2];
      P[i] = keep + dpp<ROR8>(send);
    }
    const float keep = b2 ? P[1] : P[0], send = b2 ? P[0] : P[1];
    r = keep + dpp<HMIRROR>(send);
    r += dpp<QP_X1>(r);
    r += dpp<QP_X2>(r);
  }
  return r;
}

// wave all-reduce over lane bits 2..5 (the 16 lanes sharing l % 4)
__device__ __forceinline__ float sum_bits2to5(float v) {
  v += dpp<ROR4>(v);  // rotations by 4 and 8 inside the row: lanes i, i+4, i+8, i+12 (mod 16)
  v += dpp<ROR8>(v);
  v = swap16_sum(v, v);
  return swap32_sum(v, v);
}
// quad all-reduce (lane bits 0..1)
__device__ __forceinline__ float quad_sum(float v) {
  v += dpp<QP_X1>(v);
  return v + dpp<QP_X2>(v);
}

// Selects among register values.  The operands pass an empty asm first: otherwise InstCombine
// folds the select chain into a dynamically indexed load, which pins the array in scratch.
__device__ __forceinline__ float opq(float x) {
  asm volatile("" : "+v"(x));
  return x;
}
template <int N>
__device__ __forceinline__ float selc(const float (&v)[N], int i) {
  float r = opq(v[0]);
#pragma unroll
  for (int k = 1; k < N; ++k) r = i == k ? opq(v[k]) : r;
  return r;
}

// v_mfma_f32_4x4x1_16b_f32: 16 independent 4x4 outer products per wave, exact fp32 (an fmaf chain),
// on the matrix pipe.  Block b = lane / 4: A[b][m] comes from lane 4b + m, B[b][n] from lane 4b + n,
// and lane 4b + n holds C[b][m = 0..3][n] in its 4 registers (tools/probes/mfma4x4_probe.hip).
typedef float f32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4_t mfma4(float a, float b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float rl(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

// uniform int read through the scalar cache (a constant-address-space load is an s_load)
__device__ __forceinline__ int sload(const int* p) { return *(const __attribute__((address_space(4))) int*)p; }

// [128][128] fp32 block staged in LDS with the 16-B slot of row r XOR-swizzled by r % 16: the
// per-lane row-segment reads/writes (16 lanes = 16 rows of one column slot) hit 16 distinct slots.
// Native vector type: a float4 (struct) copy becomes a memcpy that SROA leaves in scratch.
typedef float v4f __attribute__((ext_vector_type(4)));
template <int H, int NT>
struct Stage {
  static constexpr int LD = H * H / 4 / NT;  // 16-B pieces per thread
  static __device__ __forceinline__ int slot(int r, int c) { return r * H + 4 * (c ^ (r & 15)); }
  // coalesced piece g = i * NT + t of the flat block <-> slot (row g / (H/4), column g % (H/4))
  static __device__ __forceinline__ void put(float* lds, const v4f (&s)[LD], int t) {
#pragma unroll
    for (int i = 0; i < LD; ++i) {
      const int g = i * NT + t;
      *reinterpret_cast<v4f*>(lds + slot(g / (H / 4), g % (H / 4))) = s[i];
    }
  }
  static __device__ __forceinline__ void store(float* dst, const float* lds, int t) {
#pragma unroll
    for (int i = 0; i < LD; ++i) {
      const int g = i * NT + t;
      *reinterpret_cast<v4f*>(dst + 4 * g) = *reinterpret_cast<const v4f*>(lds + slot(g / (H / 4), g % (H / 4)));
    }
  }
  // a lane's own KS-wide k-slice (16-B column slots cs .. cs + KS/4) of rows l and l + 64
  template <int KS>
  static __device__ __forceinline__ void get(const float* lds, float (&d)[2][KS], int l, int cs) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < KS / 4; ++q) {
        const v4f t4 = *reinterpret_cast<const v4f*>(lds + slot(l + 64 * j, cs + q));
        d[j][4 * q] = t4.x; d[j][4 * q + 1] = t4.y; d[j][4 * q + 2] = t4.z; d[j][4 * q + 3] = t4.w;
      }
  }
  template <int KS>
  static __device__ __forceinline__ void own(float* lds, const float (&s)[2][KS], int l, int cs) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < KS / 4; ++q)
        *reinterpret_cast<v4f*>(lds + slot(l + 64 * j, cs + q)) =
            (v4f){s[j][4 * q], s[j][4 * q + 1], s[j][4 * q + 2], s[j][4 * q + 3]};
  }
};

}  // namespace bku
}  // namespace dct
