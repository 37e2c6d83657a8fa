// Small device-side step bookkeeping kernels of the graph-captured training step
// (mlp_executor.cpp): everything that changes from one step to the next lives in device
// memory (batch cursor, Adam step counter, loss stats), so ONE captured hipGraph replays
// every step of an epoch with no host involvement.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dct_common.h"

namespace dct {

// Batch gather: row r (< B) of the batch is dataset row idx[(*cursor) * stride + r] (wrapping inside
// [0, n_items) for a partial last batch). 16-byte vector copies; labels gathered alongside.
__global__ __launch_bounds__(256) void gather_batch_kernel(const uint4* __restrict__ X, int row_vec,
                                                           const int* __restrict__ Y, const int* __restrict__ idx,
                                                           const int* __restrict__ cursor, int stride, int B,
                                                           int n_items, uint4* __restrict__ xdst,
                                                           int* __restrict__ ydst) {
  const int c = *cursor;
  const int total = B * row_vec;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const int r = e / row_vec;
    const int v = e - r * row_vec;
    int q = c * stride + r;
    q = q < n_items ? q : (n_items > 0 ? q % n_items : 0);
    const int row = idx[q];
    xdst[e] = X[(size_t)row * row_vec + v];
    if (v == 0) ydst[r] = Y[row];
  }
}

// step prologue: Adam step counter += 1 (read by adam_flat), loss/correct sums = 0
__global__ void step_begin_kernel(int* step_counter, float* stats) {
  if (threadIdx.x == 0) {
    step_counter[0] += 1;
    stats[0] = 0.f;
    stats[1] = 0.f;
  }
}

// after the loss kernel: the batch-mean loss goes into the gradient buffer's extra slot so
// the DDP all-reduce averages it across ranks together with the gradients (sync_dist)
__global__ void loss_to_slot_kernel(const float* stats, float* slot, float inv_rows) {
  if (threadIdx.x == 0) slot[0] = stats[0] * inv_rows;
}

// step epilogue: loss_out[*cursor] = reduced loss, cursor += 1
__global__ void step_end_kernel(int* cursor, const float* slot, float* loss_out, int loss_cap) {
  if (threadIdx.x == 0) {
    const int c = cursor[0];
    if (loss_out && c >= 0 && c < loss_cap) loss_out[c] = slot[0];
    cursor[0] = c + 1;
  }
}

}  // namespace dct

extern "C" {

int dct_gather_batch(const void* X, int row_bytes, const int* Y, const int* idx, const int* cursor, int stride,
                     int B, int n_items, void* xdst, int* ydst, void* stream) {
  if (B <= 0) return 0;
  if (row_bytes % 16 || (((uintptr_t)X) | ((uintptr_t)xdst)) & 15) return (int)hipErrorInvalidValue;
  const int rv = row_bytes / 16;
  int grid = (B * rv + 255) / 256;
  grid = grid > 1024 ? 1024 : (grid < 1 ? 1 : grid);
  hipLaunchKernelGGL(dct::gather_batch_kernel, dim3(grid), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     (const uint4*)X, rv, Y, idx, cursor, stride, B, n_items, (uint4*)xdst, ydst);
  return (int)hipGetLastError();
}

int dct_step_begin(int* step_counter, float* stats, void* stream) {
  hipLaunchKernelGGL(dct::step_begin_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream),
                     step_counter, stats);
  return (int)hipGetLastError();
}

int dct_loss_to_slot(const float* stats, float* slot, float inv_rows, void* stream) {
  hipLaunchKernelGGL(dct::loss_to_slot_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), stats,
                     slot, inv_rows);
  return (int)hipGetLastError();
}

int dct_step_end(int* cursor, const float* slot, float* loss_out, int loss_cap, void* stream) {
  hipLaunchKernelGGL(dct::step_end_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), cursor, slot,
                     loss_out, loss_cap);
  return (int)hipGetLastError();
}

}  // extern "C"
