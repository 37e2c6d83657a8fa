// Which lane does DPP row_ror:4 read on gfx950?  Prints the source lane seen by lanes 0..15.
// Build: hipcc --offload-arch=gfx950 -O2 tools/probes/dpp_dir_probe.hip -o tools/probes/dpp_dir_probe
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(int* out) {
  const int l = threadIdx.x;
  out[l] = __builtin_amdgcn_mov_dpp(l, 0x124, 0xF, 0xF, true);          // row_ror:4
  out[64 + l] = __builtin_amdgcn_mov_dpp(l, 0x12C, 0xF, 0xF, true);     // row_ror:12
}

int main() {
  int* d;
  int h[128];
  if (hipMalloc(&d, 128 * sizeof(int)) != hipSuccess) return 1;
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  printf("row_ror:4  lanes 0..15 read:");
  for (int i = 0; i < 16; ++i) printf(" %d", h[i]);
  printf("\nrow_ror:12 lanes 0..15 read:");
  for (int i = 0; i < 16; ++i) printf(" %d", h[64 + i]);
  printf("\n");
  hipFree(d);
  return 0;
}
