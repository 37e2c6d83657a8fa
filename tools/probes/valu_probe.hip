// VALU issue probe on gfx950 for the register-resident trainers: cycles per wave-instruction of
// independent v_fma_f32 / v_pk_fma_f32 / v_rcp_f32 / v_add_f32 DPP streams with 1 wave, 1 wave
// per SIMD (4 waves) and 2 waves per SIMD (8 waves, the 3x128 kernel's shape), and dependent
// chains.  Answers: is a 2-wave SIMD's VALU throughput 1 per 2 cycles (latency-bound kernel) or
// 1 per 4 (issue-bound), and does packed f32 pay at this occupancy?
// Build: hipcc --offload-arch=gfx950 -O3 tools/probes/valu_probe.hip -o tools/probes/valu_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int REP = 16;

template <int KIND, int NCH>
__global__ void probe(const float* in, float* out, unsigned long long* cyc, int iters) {
  // cyc[w] = s_memtime cycles, cyc[16 + w] = s_memrealtime ticks (100 MHz) of the timed loop
  const int l = threadIdx.x & 63;
  float a = in[l], b = in[(l + 3) & 63];
  float x[NCH];
  f2 y[NCH];
#pragma unroll
  for (int i = 0; i < NCH; ++i) { x[i] = in[(l + i) & 63]; y[i] = (f2){x[i], x[i] + 1.f}; }
  const f2 a2 = {a, b}, b2 = {b, a};
  __syncthreads();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int rep = 0; rep < REP; ++rep)  // REP copies per loop trip: the loop's SALU + branch amortised
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      if constexpr (KIND == 0) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x[i]) : "v"(a), "v"(b));
      if constexpr (KIND == 1) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(y[i]) : "v"(a2), "v"(b2));
      if constexpr (KIND == 2) asm volatile("v_rcp_f32 %0, %0" : "+v"(x[i]));
      if constexpr (KIND == 3) asm volatile("v_add_f32_dpp %0, %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(x[i]) : "v"(a));
      if constexpr (KIND == 4) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x[i]) : "v"(a));
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NCH; ++i) s += x[i] + y[i].x + y[i].y;
  out[threadIdx.x] = s;
  if (l == 0) {
    cyc[threadIdx.x >> 6] = t1 - t0;
    cyc[16 + (threadIdx.x >> 6)] = r1 - r0;
  }
}

// clock warm-up: every CU busy for ~50 ms before the timed probes
__global__ void spin(float* out, int iters) {
  float x = threadIdx.x * 1e-3f;
  for (int i = 0; i < iters; ++i) x = fmaf(x, 0.999f, 1e-4f);
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

static void ck(hipError_t e, const char* w) {
  if (e != hipSuccess) { printf("%s: %s\n", w, hipGetErrorString(e)); exit(1); }
}

template <int KIND, int NCH>
static void run(const char* name, const float* in, float* out, unsigned long long* cyc) {
  const int iters = 256;
  for (int waves : {1, 4, 8, 16}) {
    unsigned long long h[32] = {};
    hipLaunchKernelGGL((probe<KIND, NCH>), dim3(1), dim3(64 * waves), 0, 0, in, out, cyc, iters);  // warm
    hipLaunchKernelGGL((probe<KIND, NCH>), dim3(1), dim3(64 * waves), 0, 0, in, out, cyc, iters);
    ck(hipDeviceSynchronize(), "sync");
    ck(hipMemcpy(h, cyc, 32 * 8, hipMemcpyDeviceToHost), "cpy");
    double lo = 1e30, hi = 0, ns = 0;
    for (int w = 0; w < waves; ++w) {
      const double c = (double)h[w] / (iters * NCH * REP);
      lo = c < lo ? c : lo; hi = c > hi ? c : hi;
      ns = (double)h[16 + w] * 10.0 / (iters * NCH * REP);
    }
    printf("%-28s %d chain(s), %d wave(s): %.2f .. %.2f cycles per instruction per wave (%.2f ns; clock %.2f GHz)\n",
           name, NCH, waves, lo, hi, ns, lo / ns);
  }
}

int main() {
  float *in, *out;
  unsigned long long* cyc;
  ck(hipMalloc(&in, 64 * 4), "malloc"); ck(hipMalloc(&out, 1 << 20), "malloc"); ck(hipMalloc(&cyc, 32 * 8), "malloc");
  hipLaunchKernelGGL(spin, dim3(1024), dim3(256), 0, 0, out, 200000);
  ck(hipDeviceSynchronize(), "spin");
  float h[64];
  for (int i = 0; i < 64; ++i) h[i] = 1.0f + 1e-3f * i;
  ck(hipMemcpy(in, h, 256, hipMemcpyHostToDevice), "cpy");
  run<0, 1>("v_fma_f32 dependent", in, out, cyc);
  run<0, 8>("v_fma_f32 independent", in, out, cyc);
  run<1, 1>("v_pk_fma_f32 dependent", in, out, cyc);
  run<1, 8>("v_pk_fma_f32 independent", in, out, cyc);
  run<4, 8>("v_mul_f32 independent", in, out, cyc);
  run<2, 8>("v_rcp_f32 independent", in, out, cyc);
  run<3, 1>("v_add_f32_dpp dependent", in, out, cyc);
  run<3, 8>("v_add_f32_dpp independent", in, out, cyc);
  run<0, 2>("v_fma_f32 2 chains", in, out, cyc);
  run<0, 4>("v_fma_f32 4 chains", in, out, cyc);
  printf("done\n");
  return 0;
}
