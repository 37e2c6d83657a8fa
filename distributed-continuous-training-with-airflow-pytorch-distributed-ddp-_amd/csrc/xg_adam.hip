// Peer-to-peer gradient all-reduce fused with the flat Adam update, for the DDP step path of the
// models the single-wave trainer does not cover (trainer/engines.py FusedEngine._ddp_step: the
// register-resident 3x128 weather trainer in grad mode, mlp_block5.hip).
//
// Reference semantics: DDP's Reducer averages the ranks' gradients (one bucket all-reduce, plus
// the 4-byte sync_dist loss all-reduce) before an identical Adam step on every rank
// (jobs/train_lightning_ddp.py:87-88,136).  The RCCL path does that as
// all-reduce(ncclAvg) + adam_flat: two launches, and the collective's protocol latency is several
// times the whole 4 us fused step.  Here one kernel does both over the xGMI peer mappings of a
// PeerExchange (runtime.cpp; IPC-mapped receive buffers, one node, fully connected):
//
//   thread i owns the element pair {2i, 2i+1} of gbuf (gradients, and the local loss at [P]);
//   it pushes one 16-B granule {g0, tag, g1, tag} into slot [par][rank][i] of every peer's buffer
//   (system-scope write-through store: each 8-B half carries the tag, so a torn 16-B write is never
//   taken for a complete one), polls slot [par][q][i] of its own buffer for every peer q until both
//   tags match, sums the W contributions in rank order (bit-identical result on every rank), scales
//   by 1/W and applies Adam to its elements.  tag = t (the 1-based step the grad kernel advanced the
//   device step counter to), par = t & 1: a rank can reach step t+2's push only after every rank
//   finished step t+1's poll, which stream order puts after its step-t poll - two slots suffice.
//
// Every peer link carries 8 B per element (value + tag), all links at once; no ring, no second
// sync.  Bounded spins: a timeout writes 0x80000000 | tag into the exchange status word, and a
// launch that finds the status already set does nothing (the engine checks it collectively and
// raises or falls back, as for the in-kernel exchange of the single-wave trainer).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dct_common.h"

namespace dct {

typedef unsigned int xa_v4u __attribute__((ext_vector_type(4)));
constexpr int XA_SYS = 17;  // buffer aux bits: sc0 | sc1 = system scope (write-through, no stale L2 hit)
constexpr int XA_MAXW = 8;

struct XgAdamArgs {
  float* g;                   // [n] local gradients (+ loss at [P]); overwritten by the rank average
  float *p, *m, *v;           // [P] parameters and Adam moments
  int n, P;                   // n = P + 1 (loss slot) or P
  const int* step_counter;    // t, already advanced by the grad kernel
  float lr, b1, b2, eps, wd;  // L2 weight decay (torch.optim.Adam weight_decay)
  char* recv;                 // this rank's receive buffer [2][W][npair] x 16 B
  char* const* peers;         // W device pointers (peers[rank] = recv)
  unsigned* status;
  int world, rank;
  long long timeout_ticks;    // s_memrealtime (100 MHz)
};

__device__ __forceinline__ void xa_adam(float& p, float g, float& m, float& v, const XgAdamArgs& a, float step_size,
                                        float rbc2) {
  g += a.wd * p;
  m = a.b1 * m + (1.f - a.b1) * g;
  v = a.b2 * v + (1.f - a.b2) * g * g;
  const float denom = sqrtf(v) * rbc2 + a.eps;
  p -= step_size * m / denom;
}

template <int XW>
__global__ __launch_bounds__(256) void xg_allreduce_adam_kernel(XgAdamArgs a) {
  const int npair = (a.n + 1) >> 1;
  const int i = blockIdx.x * 256 + threadIdx.x;
  // every independent load first (status, step counter, gradients, Adam state): one memory
  // latency instead of a chain of five; out-of-range lanes read a clamped, valid element
  const unsigned st = __hip_atomic_load(a.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const uint32_t t = (uint32_t)__hip_atomic_load(a.step_counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int i_c = i < npair ? i : npair - 1;  // every lane polls a valid slot; only i < npair writes
  const int e0 = 2 * i_c, e1 = 2 * i_c + 1;
  const float g0 = a.g[e0];
  const float g1 = a.g[e1 < a.n ? e1 : e0];
  const int q0 = e0 < a.P ? e0 : a.P - 1, q1 = e1 < a.P ? e1 : a.P - 1;
  float p0 = a.p[q0], m0 = a.m[q0], w0 = a.v[q0];
  float p1 = a.p[q1], m1 = a.m[q1], w1 = a.v[q1];
  if (st != 0u) return;  // an earlier exchange timed out: leave everything as it is
  const int W = a.world, rank = a.rank;
  const uint32_t tag = t;
  const int par = (int)(t & 1u) * W;
  const int nbytes = 2 * W * npair * 16;
  if (i < npair) {
    xa_v4u d;
    d.x = __float_as_uint(g0);
    d.y = tag;
    d.z = __float_as_uint(g1);
    d.w = tag;
    const int off = ((par + rank) * npair + i) * 16;
#pragma unroll
    for (int q = 0; q < XW; ++q) {
      if (q < W && q != rank) {
        const __amdgpu_buffer_rsrc_t pr = __builtin_amdgcn_make_buffer_rsrc(sload_ptr(a.peers, q), 0, nbytes, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(d, pr, off, 0, XA_SYS);
      }
    }
  }
  float v0[XW], v1[XW];
#pragma unroll
  for (int q = 0; q < XW; ++q) v0[q] = v1[q] = 0.f;
  if (W > 1) {
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(a.recv, 0, nbytes, 0x00020000);
    const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
    for (int spin = 0;; ++spin) {
      bool ok = true;
#pragma unroll
      for (int q = 0; q < XW; ++q) {
        if (q < W && q != rank) {  // wave-uniform
          const xa_v4u d = __builtin_amdgcn_raw_buffer_load_b128(rr, ((par + q) * npair + i_c) * 16, 0, XA_SYS);
          v0[q] = __uint_as_float(d.x);
          v1[q] = __uint_as_float(d.z);
          ok &= (d.y == tag) & (d.w == tag);
        }
      }
      if (__all(ok)) break;
      if ((spin & 15) == 15 && (long long)(__builtin_amdgcn_s_memrealtime() - t_start) > a.timeout_ticks) {
        if (threadIdx.x == 0)
          __hip_atomic_store(a.status, 0x80000000u | tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  if (i >= npair) return;
  float s0 = 0.f, s1 = 0.f;
#pragma unroll
  for (int q = 0; q < XW; ++q) {
    if (q < W) {
      s0 += q == rank ? g0 : v0[q];
      s1 += q == rank ? g1 : v1[q];
    }
  }
  const float inv = 1.f / (float)W;
  const float r0 = s0 * inv, r1 = s1 * inv;
  a.g[e0] = r0;
  if (e1 < a.n) a.g[e1] = r1;
  const float tf = (float)t;
  const float step_size = a.lr / (1.f - pow_t(log2f(a.b1), tf));
  const float rbc2 = rsqrtf(1.f - pow_t(log2f(a.b2), tf));
  if (e0 < a.P) {
    xa_adam(p0, r0, m0, w0, a, step_size, rbc2);
    a.p[e0] = p0;
    a.m[e0] = m0;
    a.v[e0] = w0;
  }
  if (e1 < a.P) {
    xa_adam(p1, r1, m1, w1, a, step_size, rbc2);
    a.p[e1] = p1;
    a.m[e1] = m1;
    a.v[e1] = w1;
  }
}

}  // namespace dct

extern "C" {

// receive-buffer bytes of the exchange for n floats and W ranks (both parities)
int64_t dct_xg_adam_buffer_bytes(int64_t n, int world) { return 2 * (int64_t)world * ((n + 1) / 2) * 16; }

int dct_xg_allreduce_adam(float* g, float* p, float* m, float* v, int64_t n, int64_t P, const int* step_counter,
                          float lr, float b1, float b2, float eps, float wd, void* recv, void* const* peers,
                          unsigned* status, int world, int rank, long long timeout_ticks, void* stream) {
  if (world < 1 || world > dct::XA_MAXW || rank < 0 || rank >= world || !g || !p || !m || !v || !step_counter ||
      !recv || !peers || !status || n < 1 || P < 1 || P > n || dct_xg_adam_buffer_bytes(n, world) > INT32_MAX)
    return (int)hipErrorInvalidValue;
  dct::XgAdamArgs a;
  a.g = g;
  a.p = p;
  a.m = m;
  a.v = v;
  a.n = (int)n;
  a.P = (int)P;
  a.step_counter = step_counter;
  a.lr = lr;
  a.b1 = b1;
  a.b2 = b2;
  a.eps = eps;
  a.wd = wd;
  a.recv = reinterpret_cast<char*>(recv);
  a.peers = reinterpret_cast<char* const*>(peers);
  a.status = status;
  a.world = world;
  a.rank = rank;
  a.timeout_ticks = timeout_ticks;
  const int npair = (int)((n + 1) / 2);
  const dim3 grid((npair + 255) / 256);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (world <= 2)
    hipLaunchKernelGGL(dct::xg_allreduce_adam_kernel<2>, grid, dim3(256), 0, st, a);
  else if (world <= 4)
    hipLaunchKernelGGL(dct::xg_allreduce_adam_kernel<4>, grid, dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL(dct::xg_allreduce_adam_kernel<8>, grid, dim3(256), 0, st, a);
  return (int)hipGetLastError();
}

}  // extern "C"
