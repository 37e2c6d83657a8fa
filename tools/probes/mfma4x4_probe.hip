// Probe of v_mfma_f32_4x4x1_16b_f32 on gfx950 (the batch-4 outer-product MFMA the 3x128 trainer
// could use for its 128x128 layer): operand / accumulator lane maps and issue cost.
//   layout: C[lane][reg] for A = 1 + lane, B = 1  -> which A lane feeds (lane, reg)
//           C[lane][reg] for A = 1, B = 1 + lane  -> which B lane feeds (lane, reg)
//   timing: s_memtime over 4096 MFMAs, 1 and 4 independent accumulators, 1 wave and 4 waves
// Build: hipcc --offload-arch=gfx950 -O3 tools/probes/mfma4x4_probe.hip -o tools/probes/mfma4x4_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void layout_kernel(const float* A, const float* B, float* C) {
  const int l = threadIdx.x;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_f32_4x4x1f32(A[l], B[l], acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) C[l * 4 + r] = acc[r];
}

template <int NACC>
__global__ void timing_kernel(const float* A, float* out, unsigned long long* cyc, int iters) {
  const int l = threadIdx.x & 63;
  float a = A[l], b = A[(l + 7) & 63];
  f32x4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, acc[i], 0, 0, 0);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[threadIdx.x] = s;
  if (l == 0) cyc[threadIdx.x >> 6] = t1 - t0;
}

static void ck(hipError_t e, const char* w) {
  if (e != hipSuccess) { printf("%s: %s\n", w, hipGetErrorString(e)); exit(1); }
}

int main() {
  float hA[64], hB[64], hC[256];
  float *A, *B, *C, *O;
  unsigned long long* cyc;
  ck(hipMalloc(&A, 256 * 4), "malloc"); ck(hipMalloc(&B, 256 * 4), "malloc"); ck(hipMalloc(&C, 256 * 4), "malloc");
  ck(hipMalloc(&O, 1024 * 4), "malloc"); ck(hipMalloc(&cyc, 16 * 8), "malloc");
  for (int pass = 0; pass < 2; ++pass) {
    for (int l = 0; l < 64; ++l) { hA[l] = pass == 0 ? 1.f + l : 1.f; hB[l] = pass == 0 ? 1.f : 1.f + l; }
    ck(hipMemcpy(A, hA, 256, hipMemcpyHostToDevice), "cpy"); ck(hipMemcpy(B, hB, 256, hipMemcpyHostToDevice), "cpy");
    hipLaunchKernelGGL(layout_kernel, dim3(1), dim3(64), 0, 0, A, B, C);
    ck(hipDeviceSynchronize(), "sync");
    ck(hipMemcpy(hC, C, 1024, hipMemcpyDeviceToHost), "cpy");
    printf("%s lane of C[lane][reg] (value - 1):\n", pass == 0 ? "A" : "B");
    for (int l = 0; l < 64; ++l) {
      printf("  lane %2d:", l);
      for (int r = 0; r < 4; ++r) printf(" %3d", (int)hC[l * 4 + r] - 1);
      printf("\n");
    }
  }
  const int iters = 4096;
  unsigned long long hc[16];
  for (int waves = 1; waves <= 8; waves *= 2) {
    hipLaunchKernelGGL((timing_kernel<1>), dim3(1), dim3(64 * waves), 0, 0, A, O, cyc, iters);
    ck(hipDeviceSynchronize(), "sync");
    ck(hipMemcpy(hc, cyc, 8 * waves, hipMemcpyDeviceToHost), "cpy");
    printf("1 accumulator, %d waves: %.1f cycles per MFMA per wave\n", waves, (double)hc[0] / iters);
    hipLaunchKernelGGL((timing_kernel<4>), dim3(1), dim3(64 * waves), 0, 0, A, O, cyc, iters);
    ck(hipDeviceSynchronize(), "sync");
    ck(hipMemcpy(hc, cyc, 8 * waves, hipMemcpyDeviceToHost), "cpy");
    printf("4 accumulators, %d waves: %.1f cycles per MFMA per wave\n", waves, (double)hc[0] / (4.0 * iters));
  }
  printf("done\n");
  return 0;
}
