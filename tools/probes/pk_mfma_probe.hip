// Packed fp32 VALU beside MFMA on gfx950: which v_pk_* pattern loses its LOW half while another wave
// of the same SIMD runs MFMAs?  (profiles/adam_ride_debug_r5.log, tools/probes/adam_ride_probe.hip:
// the float4 Adam riding in the dW GEMM launch updated the low component of 16 consecutive lanes with
// denom = eps - only beside the GEMM's MFMA workgroups, never alone, never without v_pk_*.)
// Each launch: even workgroups run back-to-back v_mfma_f32_16x16x32_bf16 chains, odd workgroups run
// one inline-asm packed-fp32 pattern in a loop and check both halves against v_fma_f32 on the same
// operands (bit compare); mismatches are counted per (pattern, half, 16-lane group).
//   pattern 0: v_pk_fma_f32, operands produced long before (no forwarding)
//   pattern 1: v_pk_fma_f32 whose low source was written by the instruction right before it (v_add_f32)
//   pattern 2: v_pk_fma_f32 whose low source is a v_sqrt_f32 result (s_nop 1: the trans-use wait state)
//   pattern 3: v_pk_fma_f32 with op_sel:[0,1,0] op_sel_hi:[1,1,0] (low half reads the HIGH register of
//              src1: the compiler's form of the riding Adam's denominator, sqrt * rbc2 + eps)
//   pattern 4: v_pk_mul_f32, operands produced long before
//   pattern 5: scalar control: two v_fma_f32
//   pattern 6: pattern 3 with an SGPR-pair src2 (op_sel_hi 0: its low register for both halves), the
//              compiler's exact form: v_pk_fma_f32 v[16:17], v[18:19], v[48:49], s[74:75] op_sel:[0,1,0] op_sel_hi:[1,1,0]
//   pattern 7: pattern 6 without op_sel on src1
// MFMA role (second argument): 1 = register-operand MFMA chains, 2 = MFMA fed from LDS + a global load per step,
// 3 = LDS-DMA streaming (global_load_lds_dwordx4) beside MFMA chains, 4 = LDS-DMA streaming alone
// Build: hipcc --offload-arch=gfx950 -O3 tools/probes/pk_mfma_probe.hip -o tools/probes/pk_mfma_probe
// Run:   pk_mfma_probe <pattern> <mfma role: 0 off / 1 / 2> <launches>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef float v2f __attribute__((ext_vector_type(2)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));

constexpr int ITERS = 4096;

// explicit registers v40..v47 (clobbered): a -> v[40:41], b -> v[42:43], c -> v[44:45], result v[46:47]
#define PK_IN "v_mov_b32 v40, %2\n\tv_mov_b32 v41, %3\n\tv_mov_b32 v42, %4\n\tv_mov_b32 v43, %5\n\t" \
              "v_mov_b32 v44, %6\n\tv_mov_b32 v45, %7\n\t"
#define PK_OUT "\n\tv_mov_b32 %0, v46\n\tv_mov_b32 %1, v47"
#define PK_ARGS : "=v"(lo), "=v"(hi) : "v"(a.x), "v"(a.y), "v"(b.x), "v"(b.y), "v"(c.x), "v"(c.y), "v"(s) \
                : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47"
template <int PAT>
__device__ __forceinline__ void one(v2f a, v2f b, v2f c, float s, v2f cs, v2f& r) {
  float lo, hi;
  if constexpr (PAT == 0) {  // operands written long before (no forwarding)
    asm volatile(PK_IN "s_nop 7\n\ts_nop 7\n\tv_pk_fma_f32 v[46:47], v[40:41], v[42:43], v[44:45]" PK_OUT PK_ARGS);
  } else if constexpr (PAT == 1) {  // low source written by the instruction right before
    asm volatile(PK_IN "s_nop 7\n\tv_add_f32 v40, v40, 0\n\tv_pk_fma_f32 v[46:47], v[40:41], v[42:43], v[44:45]" PK_OUT
                 PK_ARGS);
  } else if constexpr (PAT == 2) {  // low source = a v_sqrt_f32 result, one wait state (trans use)
    asm volatile(PK_IN "v_mul_f32 v40, %8, %8\n\tv_sqrt_f32 v40, v40\n\ts_nop 1\n\t"
                 "v_pk_fma_f32 v[46:47], v[40:41], v[42:43], v[44:45]" PK_OUT PK_ARGS);
  } else if constexpr (PAT == 3) {  // lo = a.lo * b.hi + c.lo, hi = a.hi * b.hi + c.lo
    asm volatile(PK_IN "s_nop 7\n\ts_nop 7\n\tv_pk_fma_f32 v[46:47], v[40:41], v[42:43], v[44:45] op_sel:[0,1,0] "
                 "op_sel_hi:[1,1,0]" PK_OUT PK_ARGS);
  } else if constexpr (PAT == 4) {
    asm volatile(PK_IN "s_nop 7\n\ts_nop 7\n\tv_pk_mul_f32 v[46:47], v[40:41], v[42:43]" PK_OUT PK_ARGS);
  } else if constexpr (PAT == 6) {  // the riding Adam's denominator: SGPR src2, op_sel on src1's low half
    asm volatile(PK_IN "s_nop 7\n\ts_nop 7\n\tv_pk_fma_f32 v[46:47], v[40:41], v[42:43], %8 op_sel:[0,1,0] "
                 "op_sel_hi:[1,1,0]" PK_OUT
                 : "=v"(lo), "=v"(hi) : "v"(a.x), "v"(a.y), "v"(b.x), "v"(b.y), "v"(c.x), "v"(c.y), "s"(cs)
                 : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");
  } else if constexpr (PAT == 7) {  // same, no op_sel on src1 (low half reads src1's LOW register)
    asm volatile(PK_IN "s_nop 7\n\ts_nop 7\n\tv_pk_fma_f32 v[46:47], v[40:41], v[42:43], %8 op_sel_hi:[1,1,0]" PK_OUT
                 : "=v"(lo), "=v"(hi) : "v"(a.x), "v"(a.y), "v"(b.x), "v"(b.y), "v"(c.x), "v"(c.y), "s"(cs)
                 : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");
  } else {  // scalar control
    asm volatile(PK_IN "s_nop 7\n\tv_fma_f32 v46, v40, v42, v44\n\tv_fma_f32 v47, v41, v43, v45" PK_OUT PK_ARGS);
  }
  r = (v2f){lo, hi};
}

template <int PAT>
__device__ __forceinline__ void expect(v2f a, v2f b, v2f c, float s, v2f cs, float& lo, float& hi) {
  if constexpr (PAT == 2) a.x = __builtin_amdgcn_sqrtf(s * s);  // the raw v_sqrt_f32 the pattern uses
  if constexpr (PAT == 3) {
    lo = __builtin_fmaf(a.x, b.y, c.x);
    hi = __builtin_fmaf(a.y, b.y, c.x);
  } else if constexpr (PAT == 6) {
    lo = __builtin_fmaf(a.x, b.y, cs.x);
    hi = __builtin_fmaf(a.y, b.y, cs.x);
  } else if constexpr (PAT == 7) {
    lo = __builtin_fmaf(a.x, b.x, cs.x);
    hi = __builtin_fmaf(a.y, b.y, cs.x);
  } else if constexpr (PAT == 4) {
    lo = a.x * b.x;
    hi = a.y * b.y;
  } else {
    lo = __builtin_fmaf(a.x, b.x, c.x);
    hi = __builtin_fmaf(a.y, b.y, c.y);
  }
}

template <int PAT>
__global__ __launch_bounds__(256) void probe(const float* in, unsigned* bad, float* sink, int mfma_on, float cs0,
                                             float cs1, float* sample) {
  __shared__ __attribute__((aligned(16))) __bf16 tile[2][256 * 8];
  const int lane = threadIdx.x & 63;
  if ((blockIdx.x & 1) == 0) {
    if (!mfma_on) return;
    if (mfma_on >= 3) {
      // LDS-DMA streaming (global_load_lds_dwordx4, M0 set in asm like the GEMM tiles), role 3 with
      // MFMA chains beside it, role 4 without any MFMA
      v4f acc[4];
      for (int j = 0; j < 4; ++j) acc[j] = (v4f){0.f, 0.f, 0.f, 0.f};
      bf8 x, y;
      for (int i = 0; i < 8; ++i) {
        x[i] = (__bf16)in[(lane + i) & 255];
        y[i] = (__bf16)in[(lane * 3 + i) & 255];
      }
      const int wave = threadIdx.x >> 6;
      for (int it = 0; it < ITERS / 2; ++it) {
        const float* g = in + ((it * 64 + lane) & 255);
        const uint32_t dst =
            __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(&tile[0][0]) + (uint32_t)(((it & 1) * 4 + wave) * 1024));
        uint32_t keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(g), "s"(dst) : "memory");
        if (mfma_on == 3) {
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, y, acc[j], 0, 0, 0);
        }
        if ((it & 7) == 7) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      float t = 0.f;
      for (int j = 0; j < 4; ++j) t += acc[j][0] + acc[j][3];
      if (t == 12345.f) sink[blockIdx.x] = t;
      return;
    }
    if (mfma_on == 2) {
      // MFMA fed from LDS every step (ds_read_b128 returns land in VGPRs beside the MFMAs), plus a global
      // load per step: the GEMM tiles' register traffic
      for (int i = threadIdx.x; i < 2 * 256 * 8; i += 256) (&tile[0][0])[i] = (__bf16)in[i & 255];
      __syncthreads();
      v4f acc[8];
      for (int j = 0; j < 8; ++j) acc[j] = (v4f){0.f, 0.f, 0.f, 0.f};
      float gs = 0.f;
      for (int it = 0; it < ITERS / 2; ++it) {
        const bf8 x = *reinterpret_cast<const bf8*>(&tile[0][((threadIdx.x + it) & 255) * 8]);
        const bf8 y = *reinterpret_cast<const bf8*>(&tile[1][((threadIdx.x * 3 + it) & 255) * 8]);
        gs += in[(threadIdx.x + it) & 255];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, y, acc[j], 0, 0, 0);
      }
      float t = gs;
      for (int j = 0; j < 8; ++j) t += acc[j][0] + acc[j][3];
      if (t == 12345.f) sink[blockIdx.x] = t;
      return;
    }
    // MFMA role: 8 independent accumulators, back-to-back 16x16x32 bf16 MFMAs
    bf8 x, y;
    for (int i = 0; i < 8; ++i) {
      x[i] = (__bf16)in[(lane + i) & 255];
      y[i] = (__bf16)in[(lane * 3 + i) & 255];
    }
    v4f acc[8];
    for (int j = 0; j < 8; ++j) acc[j] = (v4f){0.f, 0.f, 0.f, 0.f};
    for (int it = 0; it < ITERS / 2; ++it) {
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, y, acc[j], 0, 0, 0);
    }
    float t = 0.f;
    for (int j = 0; j < 8; ++j) t += acc[j][0] + acc[j][3];
    if (t == 12345.f) sink[blockIdx.x] = t;
    return;
  }
  // packed-VALU role
  const float base = in[lane] + 1.0f;
  unsigned nbad_lo = 0, nbad_hi = 0;
  for (int it = 0; it < ITERS; ++it) {
    const float f = (float)it * 1e-3f;
    v2f a = (v2f){base + f, base * 0.5f - f};
    v2f b = (v2f){1.25f + f * 0.5f, 0.75f - f * 0.25f};
    v2f c = (v2f){f * 3.0f, -f * 2.0f};
    const float s = base + 0.25f;  // sqrt(s * s) == s exactly for these magnitudes
    asm volatile("" : "+v"(a), "+v"(b), "+v"(c));
    const v2f cs = (v2f){cs0, cs1};  // kernel arguments: an SGPR pair
    v2f r;
    one<PAT>(a, b, c, s, cs, r);
    float lo, hi;
    expect<PAT>(a, b, c, s, cs, lo, hi);
    const bool blo = __float_as_uint(r.x) != __float_as_uint(lo);
    nbad_lo += blo;
    nbad_hi += __float_as_uint(r.y) != __float_as_uint(hi);
    if (blo && sample[0] == 0.f) {  // one example: got, expected, and the three low / high operands
      sample[0] = 1.f; sample[1] = r.x; sample[2] = lo; sample[3] = a.x; sample[4] = b.x; sample[5] = b.y;
      sample[6] = c.x; sample[7] = cs.x;
    }
  }
  // per 16-lane group of the wave, low / high half
  if (nbad_lo) atomicAdd(&bad[(lane >> 4) * 2 + 0], nbad_lo);
  if (nbad_hi) atomicAdd(&bad[(lane >> 4) * 2 + 1], nbad_hi);
}

int main(int argc, char** argv) {
  const int pat = argc > 1 ? std::atoi(argv[1]) : 0;
  const int mfma_on = argc > 2 ? std::atoi(argv[2]) : 1;
  const int launches = argc > 3 ? std::atoi(argv[3]) : 20;
  float* in;
  unsigned* bad;
  float* sink;
  hipMalloc(&in, 256 * 4);
  hipMalloc(&bad, 8 * 4);
  hipMalloc(&sink, 4096 * 4);
  float h[256];
  for (int i = 0; i < 256; ++i) h[i] = 0.5f + 0.001f * i;
  hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  hipMemset(bad, 0, 8 * 4);
  void (*k)(const float*, unsigned*, float*, int, float, float, float*) =
      pat == 0 ? probe<0> : pat == 1 ? probe<1> : pat == 2 ? probe<2> : pat == 3 ? probe<3> : pat == 4 ? probe<4>
      : pat == 6 ? probe<6> : pat == 7 ? probe<7> : probe<5>;
  float* sample;
  hipMalloc(&sample, 8 * 4);
  hipMemset(sample, 0, 8 * 4);
  for (int i = 0; i < launches; ++i)
    hipLaunchKernelGGL(k, dim3(2048), dim3(256), 0, 0, in, bad, sink, mfma_on, 1e-8f, 3.0f, sample);
  if (hipDeviceSynchronize() != hipSuccess) {
    std::printf("launch failed\n");
    return 2;
  }
  unsigned b[8];
  hipMemcpy(b, bad, sizeof(b), hipMemcpyDeviceToHost);
  const unsigned long long total = 1ull * launches * 1024 * 256 * ITERS;
  std::printf("pattern %d mfma %d: mismatches lo/hi per 16-lane group: [%u/%u] [%u/%u] [%u/%u] [%u/%u] of %llu results\n",
              pat, mfma_on, b[0], b[1], b[2], b[3], b[4], b[5], b[6], b[7], total);
  float sm[8];
  hipMemcpy(sm, sample, sizeof(sm), hipMemcpyDeviceToHost);
  if (sm[0] != 0.f)
    std::printf("  example: got %.9g expected %.9g (a.lo %.9g b.lo %.9g b.hi %.9g c.lo %.9g s-pair.lo %.9g)\n", sm[1], sm[2],
                sm[3], sm[4], sm[5], sm[6], sm[7]);
  return 0;
}
