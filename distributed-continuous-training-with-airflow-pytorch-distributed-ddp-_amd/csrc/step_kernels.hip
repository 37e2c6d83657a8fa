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
// up to 4 ranges of the flat gradient buffer to zero (element offset / count; 16-B aligned starts)
struct ZeroRanges {
  int n;
  int64_t off[4], cnt[4];
};

__device__ __forceinline__ void zero_range(float* base, int64_t n) {
  const int64_t n4 = n >> 2;
  const int64_t gs = (int64_t)gridDim.x * blockDim.x;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  float4* z4 = reinterpret_cast<float4*>(base);
  for (int64_t i = t; i < n4; i += gs) z4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (t < n - (n4 << 2)) base[(n4 << 2) + t] = 0.f;
}

__global__ __launch_bounds__(256) void gather_batch_kernel(const uint4* __restrict__ X, int row_vec,
                                                           const int* __restrict__ Y, const int* __restrict__ idx,
                                                           const int* __restrict__ cursor, int stride, int B,
                                                           int n_items, uint4* __restrict__ xdst,
                                                           int* __restrict__ ydst, int* __restrict__ step_counter,
                                                           float* __restrict__ zero, ZeroRanges zr) {
  const int c = cursor ? *cursor : 0;
  // the training step's prologue rides along: Adam step counter += 1 (read by adam_flat at the
  // end of the step) and the accumulated ranges of the flat gradient buffer (+ loss slot) zeroed by
  // the whole grid.  A kernel, not hipMemsetAsync: a captured memset node was not reliably ordered
  // after the previous replay's Adam kernel (back-to-back hipGraphLaunch, ROCm 7).
  if (step_counter && blockIdx.x == 0 && threadIdx.x == 0) step_counter[0] += 1;
  if (zero) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (q < zr.n) zero_range(zero + zr.off[q], zr.cnt[q]);
  }
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

// Prologue of the graph-replayed AUTOGRAD step (trainer/engines.py AutogradEngine device loop):
// batch rows idx[(*cursor) * B + r] (int64 dataset rows) -> fp32 feature rows + int64 labels in
// the captured step's static inputs, Adam step counter += 1, flat gradient buffer zeroed - one
// launch instead of two index_selects + a counter add + a zero kernel (and no host-side batch
// slicing between replays).  The cursor is advanced by the Adam epilogue at the end of the step.
__global__ __launch_bounds__(256) void ag_prologue_kernel(const uint4* __restrict__ X, int row_vec,
                                                          const int64_t* __restrict__ Y,
                                                          const int64_t* __restrict__ idx,
                                                          const int* __restrict__ cursor, int B, int64_t n_items,
                                                          uint4* __restrict__ xdst, int64_t* __restrict__ ydst,
                                                          int* __restrict__ step_counter, float* __restrict__ zero,
                                                          int64_t zero_n) {
  const int64_t c = *cursor;
  if (step_counter && blockIdx.x == 0 && threadIdx.x == 0) step_counter[0] += 1;
  if (zero) {
    const int64_t n4 = zero_n >> 2;
    const int64_t gs = (int64_t)gridDim.x * blockDim.x;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    float4* z4 = reinterpret_cast<float4*>(zero);
    for (int64_t i = t; i < n4; i += gs) z4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (t < zero_n - (n4 << 2)) zero[(n4 << 2) + t] = 0.f;
  }
  const int total = B * row_vec;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const int r = e / row_vec;
    const int v = e - r * row_vec;
    int64_t q = c * B + r;
    q = q < n_items ? q : (n_items > 0 ? q % n_items : 0);
    const int64_t row = idx[q];
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

// Device-side barrier over the xGMI peer mappings of the in-kernel exchange (runtime.cpp
// PeerExchange::barrier).  Lane q < W (q != rank) writes this barrier's tag into slot `rank` of
// peer q's barrier region (system-scope store across xGMI), then every lane polls slot q of its
// own uncached region until peer q's tag (or a later one) arrived.  One wave, no host round trip and no RCCL
// launch: it replaces the RCCL barrier where the bench brackets the timed steps (a 4-byte
// all-reduce + host wait) with one peer-write latency.  Bounded spin: a timeout writes
// 0x80000000 | tag into the exchange status word (xg_verify then reports the exchange failed).
__global__ __launch_bounds__(64) void xg_barrier_kernel(char* recv, char* const* __restrict__ peers, int64_t off,
                                                        unsigned* status, int W, int rank, unsigned tag,
                                                        long long timeout_ticks) {
  const int q = threadIdx.x;
  if (q < W && q != rank) {
    unsigned* dst = reinterpret_cast<unsigned*>(peers[q] + off) + rank * 4;
    __hip_atomic_store(dst, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  const unsigned* src = reinterpret_cast<const unsigned*>(recv + off) + (q < W ? q : 0) * 4;
  bool ok = q >= W || q == rank;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (!__all(ok)) {
    // any tag at or past this barrier's: tags only grow (reset() zeroes the region), and a fast
    // peer may already have left this barrier and written the NEXT one's tag into our slot
    // before we polled - an exact compare would then spin to the timeout (wrap-safe compare)
    if (!ok) ok = (int)(__hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - tag) >= 0;
    if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > timeout_ticks) {
      if (q == 0) __hip_atomic_store(status, 0x80000000u | tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// Reducer instrumentation (runtime.cpp BucketReducer, enable_timing): one-thread kernels, so the
// stamps ride inside captured step graphs too (an event timing pair does not survive capture).
// s[0] first bucket's all-reduce start (comm stream), s[1] end of backward (compute stream),
// s[2] / s[3] accumulated span / exposed ticks of s_memrealtime (100 MHz), s[4] comm-stream
// closes, s[5] compute-stream checks, s[6] ordering violations, s[7] steps.
__global__ void reducer_stamp_kernel(unsigned long long* dst) {
  if (threadIdx.x == 0) *dst = __builtin_amdgcn_s_memrealtime();
}
__global__ void reducer_close_kernel(unsigned long long* s) {
  if (threadIdx.x == 0) {
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    const unsigned long long t0 = s[0], tb = s[1];
    s[2] += t > t0 ? t - t0 : 0ull;   // all-reduce span: first bucket start -> last bucket done
    s[3] += t > tb ? t - tb : 0ull;   // exposed: backward end -> last bucket done
    __hip_atomic_store(&s[4], s[4] + 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s[7] += 1ull;
  }
}
// debug mode: runs on the compute stream right after it joined the comm stream - if that wait
// were missing the comm stream's close for this step might not have run yet
__global__ void reducer_check_kernel(unsigned long long* s) {
  if (threadIdx.x == 0) {
    const unsigned long long c = s[5] + 1ull;
    s[5] = c;
    if (__hip_atomic_load(&s[4], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != c) s[6] = 1ull;
  }
}

// Cross-stream edges of the bucket reducer's eager steps (runtime.cpp BucketReducer::edge): the
// producer stream bumps a device counter, the consumer stream runs a one-wave kernel that waits
// for it.  hipEventRecord + hipStreamWaitEvent cost 6-13 us of queue time per edge on MI355X
// (a marker packet that held the compute queue ~6.5 us per bucket fork, ~12 us at the join: kernel
// trace of the forced-DDP tabular step); a one-wave kernel on each side costs about a dispatch.
// The wait is bounded (2 s): on expiry it sets *status (coherent host memory) and lets the stream
// go on - never a hung queue; BucketReducer::prepare() throws on the next step (check_edges), so the
// expired edge is a loud failure, not a silent one.
__global__ __launch_bounds__(64) void flag_signal_kernel(int* flag) {
  if (threadIdx.x == 0) __hip_atomic_fetch_add(flag, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}
__global__ __launch_bounds__(64) void flag_wait_kernel(int* flag, int* consumed, int* status) {
  if (threadIdx.x != 0) return;
  const int c = __hip_atomic_load(consumed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) <= c) {
    if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {  // 2 s at 100 MHz
      __hip_atomic_store(status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  __hip_atomic_store(consumed, c + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Stand-in collective (test-only, DCT_REDUCER_STANDIN_US, runtime.cpp BucketReducer): each one-wave
// workgroup stays resident for `ticks` of s_memrealtime (100 MHz) from its own start, sleeping
// between polls - the CU / queue footprint of an all-reduce of that duration without its traffic,
// so comm / compute overlap can be measured on a one-GPU box.
__global__ __launch_bounds__(64) void busy_spin_kernel(long long ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while ((long long)(__builtin_amdgcn_s_memrealtime() - t0) < ticks) __builtin_amdgcn_s_sleep(8);
}

// Step-phase timing (utils/tracing.py DevicePhaseTimer): b[0..n) stamps of the phase marks of
// the current step (reducer_stamp_kernel writes them), b[n..2n-1) accumulated ticks per phase,
// b[2n-1] step count.  One thread; captured into step graphs like any kernel.
__global__ void phase_accum_kernel(unsigned long long* b, int n) {
  if (threadIdx.x == 0) {
    for (int i = 0; i + 1 < n; ++i) {
      const unsigned long long a = b[i], c = b[i + 1];
      b[n + i] += c > a ? c - a : 0ull;
    }
    b[2 * n - 1] += 1ull;
  }
}

}  // namespace dct

extern "C" {

int dct_phase_accum(unsigned long long* b, int n, void* stream) {
  hipLaunchKernelGGL(dct::phase_accum_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), b, n);
  return (int)hipGetLastError();
}

int dct_flag_signal(int* flag, void* stream) {
  hipLaunchKernelGGL(dct::flag_signal_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), flag);
  return (int)hipGetLastError();
}
int dct_flag_wait(int* flag, int* consumed, int* status, void* stream) {
  hipLaunchKernelGGL(dct::flag_wait_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), flag, consumed,
                     status);
  return (int)hipGetLastError();
}

int dct_busy_spin(long long ticks, int wgs, void* stream) {
  if (ticks <= 0) return 0;
  if (wgs < 1 || wgs > 1024) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(dct::busy_spin_kernel, dim3(wgs), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), ticks);
  return (int)hipGetLastError();
}

int dct_reducer_stamp(unsigned long long* dst, void* stream) {
  hipLaunchKernelGGL(dct::reducer_stamp_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), dst);
  return (int)hipGetLastError();
}
int dct_reducer_close(unsigned long long* s, void* stream) {
  hipLaunchKernelGGL(dct::reducer_close_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), s);
  return (int)hipGetLastError();
}
int dct_reducer_check(unsigned long long* s, void* stream) {
  hipLaunchKernelGGL(dct::reducer_check_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), s);
  return (int)hipGetLastError();
}

// zero: buffer base; nr ranges [off[q], off[q] + cnt[q]) of it (off[q] % 4 == 0), nr <= 4
int dct_gather_batch_step_ranges(const void* X, int row_bytes, const int* Y, const int* idx, const int* cursor,
                                 int stride, int B, int n_items, void* xdst, int* ydst, int* step_counter, float* zero,
                                 int nr, const int64_t* off, const int64_t* cnt, void* stream) {
  if (B <= 0) return 0;
  if (row_bytes % 16 || (((uintptr_t)X) | ((uintptr_t)xdst)) & 15) return (int)hipErrorInvalidValue;
  if (zero && (((uintptr_t)zero) & 15)) return (int)hipErrorInvalidValue;
  if (nr < 0 || nr > 4) return (int)hipErrorInvalidValue;
  dct::ZeroRanges zr{};
  zr.n = zero ? nr : 0;
  int64_t zmax = 0;
  for (int q = 0; q < zr.n; ++q) {
    if (off[q] % 4 || cnt[q] < 0) return (int)hipErrorInvalidValue;
    zr.off[q] = off[q];
    zr.cnt[q] = cnt[q];
    zmax = cnt[q] > zmax ? cnt[q] : zmax;
  }
  const int rv = row_bytes / 16;
  int64_t work = (int64_t)B * rv;
  if ((zmax + 3) / 4 > work) work = (zmax + 3) / 4;
  int grid = (int)((work + 255) / 256);
  grid = grid > 2048 ? 2048 : (grid < 1 ? 1 : grid);
  hipLaunchKernelGGL(dct::gather_batch_kernel, dim3(grid), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     (const uint4*)X, rv, Y, idx, cursor, stride, B, n_items, (uint4*)xdst, ydst, step_counter, zero,
                     zr);
  return (int)hipGetLastError();
}

int dct_gather_batch_step(const void* X, int row_bytes, const int* Y, const int* idx, const int* cursor, int stride,
                          int B, int n_items, void* xdst, int* ydst, int* step_counter, float* zero,
                          int64_t zero_n, void* stream) {
  const int64_t off = 0;
  return dct_gather_batch_step_ranges(X, row_bytes, Y, idx, cursor, stride, B, n_items, xdst, ydst, step_counter,
                                      zero, zero ? 1 : 0, &off, &zero_n, stream);
}

// Zero n fp32 values with a kernel (graph-captured steps: a kernel node instead of a memset node,
// see gather_batch_kernel).
int dct_zero_f32(float* p, int64_t n, void* stream) {
  if (n <= 0) return 0;
  if (((uintptr_t)p) & 15) return (int)hipErrorInvalidValue;
  int grid = (int)(((n + 3) / 4 + 255) / 256);
  grid = grid > 2048 ? 2048 : (grid < 1 ? 1 : grid);
  dct::ZeroRanges zr{};
  zr.n = 1;
  zr.off[0] = 0;
  zr.cnt[0] = n;
  hipLaunchKernelGGL(dct::gather_batch_kernel, dim3(grid), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     nullptr, 0, nullptr, nullptr, nullptr, 0, 0, 0, nullptr, nullptr, nullptr, p, zr);
  return (int)hipGetLastError();
}

int dct_gather_batch(const void* X, int row_bytes, const int* Y, const int* idx, const int* cursor, int stride,
                     int B, int n_items, void* xdst, int* ydst, void* stream) {
  return dct_gather_batch_step(X, row_bytes, Y, idx, cursor, stride, B, n_items, xdst, ydst, nullptr, nullptr, 0,
                               stream);
}

int dct_ag_step_prologue(const void* X, int row_bytes, const int64_t* Y, const int64_t* idx, const int* cursor, int B,
                         int64_t n_items, void* xdst, int64_t* ydst, int* step_counter, float* zero, int64_t zero_n,
                         void* stream) {
  if (B <= 0 || !cursor) return (int)hipErrorInvalidValue;
  if (row_bytes % 16 || (((uintptr_t)X) | ((uintptr_t)xdst)) & 15) return (int)hipErrorInvalidValue;
  if (zero && (((uintptr_t)zero) & 15)) return (int)hipErrorInvalidValue;
  const int rv = row_bytes / 16;
  int64_t work = (int64_t)B * rv;
  if (zero && (zero_n + 3) / 4 > work) work = (zero_n + 3) / 4;
  int grid = (int)((work + 255) / 256);
  grid = grid > 2048 ? 2048 : (grid < 1 ? 1 : grid);
  hipLaunchKernelGGL(dct::ag_prologue_kernel, dim3(grid), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     (const uint4*)X, rv, Y, idx, cursor, B, n_items, (uint4*)xdst, ydst, step_counter, zero, zero_n);
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

int dct_xg_barrier(void* recv, void* const* peers, int64_t off, unsigned* status, int world, int rank, unsigned tag,
                   long long timeout_ticks, void* stream) {
  if (world < 2 || world > 64 || rank < 0 || rank >= world || !recv || !peers || !status) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(dct::xg_barrier_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream),
                     reinterpret_cast<char*>(recv), reinterpret_cast<char* const*>(peers), off, status, world, rank, tag,
                     timeout_ticks);
  return (int)hipGetLastError();
}

}  // extern "C"
