// Single-wave, register-resident MLP trainer for narrow MLPs (every hidden width <= 64).
//
// The reference model (WeatherClassifier 5-64-2, jobs/train_lightning_ddp.py:57-62) has 514
// parameters and a batch of 4: one wave64 holds the whole training state in registers.
// Lane j owns hidden unit j: its input-weight row W0[j][:], bias b0[j], its output-weight
// column Wout[:, j] (and for 3 layers the middle row W1[j][:]), the Adam moments of all of
// them, and its activations.  Per optimizer step:
//   * the batch (x rows + labels, prefetched one step ahead into registers) is broadcast to
//     every lane with v_readlane into SGPRs - no LDS, no barrier;
//   * layer 0 is B x D0 FMAs per lane with SGPR operands; ReLU + inverted dropout
//     (counter hash of (seed, step, row, unit));
//   * hidden->hidden (3-layer nets): activations go through a 16 KB LDS tile read back as
//     broadcast ds_read_b128; the backward uses a transposed copy of W1 kept in LDS;
//   * the output layer is a cross-lane sum: DPP (quad_perm, row_ror) inside 16-lane rows,
//     then v_readlane of the four row sums -> logits are wave-uniform;
//   * CE/MSE and dlogits are computed redundantly by every lane (uniform values), so the
//     backward needs no communication: dWout, dh, dW0 are lane-local FMAs;
//   * Adam on the lane's own parameters (v_sqrt_f32 / v_rcp_f32).
// A single wave needs no s_barrier: LDS instructions of one wave execute in order.
//
// Data parallelism inside the kernel (XG): with W ranks (one process per GPU), every step
// each rank pushes its lane-local gradients as 8-byte {tag = global step + 1, fp32 value}
// granules, system-scope (write-through), straight into every peer's receive buffer - the
// peers' buffers are mapped into this process over xGMI with IPC handles.  The receiver
// polls its own (uncached) buffer until every granule of every peer carries the step's tag
// (the data IS the flag: no release fence, no separate flag round trip), then sums the W
// contributions in rank order, so all ranks hold bit-identical averaged gradients and apply
// identical Adam updates.  Two parity slabs make reuse safe: a rank can only write step s+2
// into a slab after receiving everyone's step s+1, i.e. after every peer finished reading
// step s.  Spins are bounded (xg_timeout); a timeout records the step in xg_status and ends
// the launch on every rank instead of hanging the GPU.
// Kernel and launch-template definitions of the narrow-MLP trainers (mlp_wave*.hip).
// Split over several translation units so the heavy template instantiations (row-parallel
// kernel x exchange width, single-wave kernel variants) compile in parallel:
//   mlp_wave.hip           extern "C" entry points (dispatch only)
//   mlp_wave_rows_x{0,2,4,8}.hip  row-parallel kernel per exchange width
//   mlp_wave_single.hip    single-wave kernel (no exchange), mlp_wave_single_xg.hip (with)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>

#include "dct_common.h"
#include "mlp_fused.h"

namespace dct {

struct WaveShape {
  int L;         // 2 or 3 linear layers
  int d0, h1, h2, C;
  int woff[3], boff[3];
  int P;
};

__device__ __forceinline__ uint32_t wave_hash(uint32_t key) {
  key ^= key >> 16;
  key *= 0x7feb352du;
  key ^= key >> 15;
  key *= 0x846ca68bu;
  key ^= key >> 16;
  return key;
}

template <int CTRL>
__device__ __forceinline__ float wdpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), CTRL, 0xF, 0xF, false));
}

__device__ __forceinline__ float rl(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

// sum over all 64 lanes of N values at once; results are wave-uniform
template <int N>
__device__ __forceinline__ void wave_sum_n(float (&v)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] += wdpp<0xB1>(v[i]);
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] += wdpp<0x4E>(v[i]);
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] += wdpp<0x124>(v[i]);
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] += wdpp<0x128>(v[i]);
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = (rl(v[i], 0) + rl(v[i], 16)) + (rl(v[i], 32) + rl(v[i], 48));
}

// wave_sum_n for the row-parallel kernel: each stage is ONE v_add_f32_dpp (mov_dpp with no live
// "old" operand folds into the add; update_dpp(v, v) above costs a copy + mov + add), and the
// cross-row part runs in DPP too (row_bcast:15 / row_bcast:31 accumulate rows into lane 63), so a
// value needs one v_readlane instead of four readlanes and three adds.
template <int CTRL>
__device__ __forceinline__ float dpp_add(float v) {
  return v + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
template <int N>
__device__ __forceinline__ void wave_sum_bcast(float (&v)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = dpp_add<0xB1>(v[i]);   // quad_perm [1,0,3,2]
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = dpp_add<0x4E>(v[i]);   // quad_perm [2,3,0,1]
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = dpp_add<0x124>(v[i]);  // row_ror:4
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = dpp_add<0x128>(v[i]);  // row_ror:8 -> every lane: its row's sum
  // row_bcast:15 (rows 1, 3 += rows 0, 2), then row_bcast:31 (rows 2, 3 += row 1). Written as
  // v_add_f32_dpp with the destination tied to the source: rows outside row_mask keep their value,
  // which no builtin expresses (update_dpp needs a zero "old" plus a separate add). The s_nops give
  // the two wait states a DPP read needs after a VALU write of its source.
  if constexpr (N == 2) {
    asm volatile(
        "s_nop 1\n\t"
        "v_add_f32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
        "v_add_f32_dpp %1, %1, %1 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
        "s_nop 0\n\t"
        "v_add_f32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n\t"
        "v_add_f32_dpp %1, %1, %1 row_bcast:31 row_mask:0xc bank_mask:0xf"
        : "+v"(v[0]), "+v"(v[1]));
  } else {
#pragma unroll
    for (int i = 0; i < N; ++i)
      asm volatile(
          "s_nop 1\n\t"
          "v_add_f32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
          "s_nop 1\n\t"
          "v_add_f32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf"
          : "+v"(v[i]));
  }
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = rl(v[i], 63);
}

__device__ __forceinline__ void adam1(float& p, float g, float& m, float& v, float b1, float b2, float wd,
                                      float step_size, float rbc2, float eps) {
  g += wd * p;
  m = b1 * m + (1.f - b1) * g;
  v = b2 * v + (1.f - b2) * g * g;
  p -= step_size * m * __builtin_amdgcn_rcpf(__builtin_amdgcn_sqrtf(v) * rbc2 + eps);
}

typedef unsigned int xg_v4u __attribute__((ext_vector_type(4)));
constexpr int XG_SYS = 17;  // buffer aux bits: sc0 | sc1 = system scope (write-through, no stale L2 hit)

// One step's gradient exchange; g (KX values per lane, KX even) is replaced by the rank average.
// Granule layout per (parity, source): [KX/2][64 lanes] x 16 B = two {value, tag} granules, so
// every store / load instruction moves one contiguous KB.  Pushes are 16-B system-scope stores;
// each 8-B half is tag-checked on its own, so a split 16-B write can never be mistaken for a
// complete one.  The poll sweeps ALL sources per pass (one round trip per pass, not per peer).
template <int KX, int XW>
__device__ __forceinline__ bool xg_allreduce(float (&g)[KX], const MlpArgs& a,
                                             const __amdgpu_buffer_rsrc_t (&prs)[XW], __amdgpu_buffer_rsrc_t rrs,
                                             uint32_t gstep, int j) {
  static_assert(KX % 2 == 0, "granule pairs");
  constexpr int K2 = KX / 2;
  const int W = a.xg_world, rank = a.xg_rank;
  const uint32_t tag = gstep + 1u;
  const int par = (int)(gstep & 1u) * W;
#pragma unroll
  for (int q = 0; q < XW; ++q) {
    if (q < W && q != rank) {
      const int base = ((par + rank) * K2 * 64 + j) * 16;
#pragma unroll
      for (int k2 = 0; k2 < K2; ++k2) {
        xg_v4u d;
        d.x = __float_as_uint(g[2 * k2]);
        d.y = tag;
        d.z = __float_as_uint(g[2 * k2 + 1]);
        d.w = tag;
        __builtin_amdgcn_raw_buffer_store_b128(d, prs[q], base + k2 * 64 * 16, 0, XG_SYS);
      }
    }
  }
  float v[XW][KX];
  unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
  int spin = 0;
  auto timed_out = [&]() -> bool {
    if ((++spin & 15) == 0 && (long long)(__builtin_amdgcn_s_memrealtime() - t_start) > a.xg_timeout) {
      if (j == 0) __hip_atomic_store(a.xg_status, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return true;
    }
    __builtin_amdgcn_s_sleep(1);
    return false;
  };
  // load every granule pair of source q into v[q]; true when all carry this step's tag
  auto load_src = [&](int q, float (&vq)[KX]) -> bool {
    const int qq = q < W ? q : 0;
    const int base = ((par + qq) * K2 * 64 + j) * 16;
    bool okq = true;
#pragma unroll
    for (int k2 = 0; k2 < K2; ++k2) {
      const xg_v4u d = __builtin_amdgcn_raw_buffer_load_b128(rrs, base + k2 * 64 * 16, 0, XG_SYS);
      vq[2 * k2] = __uint_as_float(d.x);
      vq[2 * k2 + 1] = __uint_as_float(d.z);
      okq &= (d.y == tag) & (d.w == tag);
    }
    return okq;
  };
  if (a.xg_poll == 2) {  // sequential: one source at a time
#pragma unroll
    for (int q = 0; q < XW; ++q) {
      if (q < W && q != rank) {
        while (!__all(load_src(q, v[q])))
          if (timed_out()) return false;
      }
    }
  } else {
    if (a.xg_poll == 1) {  // cheap probe: the last granule pair of every source, then one sweep
      for (;;) {
        bool ok = true;
#pragma unroll
        for (int q = 0; q < XW; ++q) {
          const int qq = q < W ? q : 0;
          const int off = (((par + qq) * K2 + (K2 - 1)) * 64 + j) * 16;
          const xg_v4u d = __builtin_amdgcn_raw_buffer_load_b128(rrs, off, 0, XG_SYS);
          ok &= ((d.y == tag) & (d.w == tag)) | (q >= W) | (q == rank);
        }
        if (__all(ok)) break;
        if (timed_out()) return false;
      }
    }
    for (;;) {  // full sweep of all sources per pass
      bool ok = true;
#pragma unroll
      for (int q = 0; q < XW; ++q) ok &= load_src(q, v[q]) | (q >= W) | (q == rank);
      if (__all(ok)) break;
      if (timed_out()) return false;
    }
  }
  float acc[KX];
#pragma unroll
  for (int k = 0; k < KX; ++k) acc[k] = 0.f;
#pragma unroll
  for (int q = 0; q < XW; ++q) {
    if (q < W) {
#pragma unroll
      for (int k = 0; k < KX; ++k) acc[k] += (q == rank) ? g[k] : v[q][k];
    }
  }
  const float invw = 1.0f / (float)W;
#pragma unroll
  for (int k = 0; k < KX; ++k) g[k] = acc[k] * invw;
  return true;
}

// Per-wave exchange of the row-parallel kernel: wave w of every rank owns one region of the
// receive buffer, [2 parity][W src][NW waves][XV/2 pairs][64 lanes] x 16 B {value, tag, value, tag},
// and pushes / polls only that region - the waves of a CU exchange their owned parameter slots in
// parallel instead of one wave moving everything.  Same tag protocol as xg_allreduce (the data is
// the flag; parity slabs make reuse safe; sums in rank order; bounded spins).
template <int XV, int XW>
__device__ __forceinline__ bool xg_exchange_wave(float (&g)[XV], const MlpArgs& a,
                                                 const __amdgpu_buffer_rsrc_t (&prs)[XW], __amdgpu_buffer_rsrc_t rrs,
                                                 uint32_t gstep, int j, int w, int nw) {
  static_assert(XV % 2 == 0, "granule pairs");
  constexpr int P2 = XV / 2;
  const int W = a.xg_world, rank = a.xg_rank;
  const uint32_t tag = gstep + 1u;
  const int par = (int)(gstep & 1u);
  auto off = [&](int src, int p) { return ((((par * W + src) * nw + w) * P2 + p) * 64 + j) * 16; };
#pragma unroll
  for (int q = 0; q < XW; ++q) {
    if (q < W && q != rank) {
#pragma unroll
      for (int p = 0; p < P2; ++p) {
        xg_v4u d;
        d.x = __float_as_uint(g[2 * p]);
        d.y = tag;
        d.z = __float_as_uint(g[2 * p + 1]);
        d.w = tag;
        __builtin_amdgcn_raw_buffer_store_b128(d, prs[q], off(rank, p), 0, XG_SYS);
      }
    }
  }
  float v[XW][XV];
  const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
  int spin = 0;
  auto timed_out = [&]() -> bool {
    if ((++spin & 15) == 0 && (long long)(__builtin_amdgcn_s_memrealtime() - t_start) > a.xg_timeout) {
      if (j == 0) __hip_atomic_store(a.xg_status, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return true;
    }
    return false;
  };
  if ((a.xg_poll & 0xff) == 3) {
    // Pipelined polls (xg_poll = 3, stagger = xg_poll >> 8 sleeps of 64 cycles): two sweeps in
    // flight, issued half a round trip apart, so a granule that lands just after one sweep read
    // its slot is seen by the other half a round trip later instead of a whole one.
    xg_v4u dA[XW][P2], dB[XW][P2];
    auto issue = [&](xg_v4u (&d)[XW][P2]) {
#pragma unroll
      for (int q = 0; q < XW; ++q) {
        const int qq = (q < W && q != rank) ? q : (rank == 0 ? 1 : 0);
#pragma unroll
        for (int p = 0; p < P2; ++p) d[q][p] = __builtin_amdgcn_raw_buffer_load_b128(rrs, off(qq, p), 0, XG_SYS);
      }
    };
    auto ready = [&](const xg_v4u (&d)[XW][P2]) -> bool {
      bool ok = true;
#pragma unroll
      for (int q = 0; q < XW; ++q)
#pragma unroll
        for (int p = 0; p < P2; ++p) ok &= ((d[q][p].y == tag) & (d[q][p].w == tag)) | (q >= W) | (q == rank);
      return __all(ok);
    };
    auto take = [&](const xg_v4u (&d)[XW][P2]) {
#pragma unroll
      for (int q = 0; q < XW; ++q)
#pragma unroll
        for (int p = 0; p < P2; ++p) {
          v[q][2 * p] = __uint_as_float(d[q][p].x);
          v[q][2 * p + 1] = __uint_as_float(d[q][p].z);
        }
    };
    issue(dA);
    for (int k = a.xg_poll >> 8; k > 0; --k) __builtin_amdgcn_s_sleep(1);
    for (;;) {
      issue(dB);
      if (ready(dA)) { take(dA); break; }
      if (timed_out()) return false;
      __builtin_amdgcn_s_sleep(1);  // also keeps the re-issued loads from being merged with the last ones
      issue(dA);
      if (ready(dB)) { take(dB); break; }
      if (timed_out()) return false;
      __builtin_amdgcn_s_sleep(1);
    }
  } else {
  for (;;) {  // sweep every source per pass (one round trip per pass)
    bool ok = true;
#pragma unroll
    for (int q = 0; q < XW; ++q) {
      const int qq = (q < W && q != rank) ? q : (rank == 0 ? 1 : 0);
#pragma unroll
      for (int p = 0; p < P2; ++p) {
        const xg_v4u d = __builtin_amdgcn_raw_buffer_load_b128(rrs, off(qq, p), 0, XG_SYS);
        v[q][2 * p] = __uint_as_float(d.x);
        v[q][2 * p + 1] = __uint_as_float(d.z);
        ok &= ((d.y == tag) & (d.w == tag)) | (q >= W) | (q == rank);
      }
    }
    if (__all(ok)) break;
    if (timed_out()) return false;
    __builtin_amdgcn_s_sleep(1);
  }
  }
  float acc[XV];
#pragma unroll
  for (int i = 0; i < XV; ++i) acc[i] = 0.f;
#pragma unroll
  for (int q = 0; q < XW; ++q) {
    if (q < W) {
#pragma unroll
      for (int i = 0; i < XV; ++i) acc[i] += (q == rank) ? g[i] : v[q][i];
    }
  }
  const float invw = 1.0f / (float)W;
#pragma unroll
  for (int i = 0; i < XV; ++i) g[i] = acc[i] * invw;
  return true;
}

// receive-buffer granules per (parity, source rank) of the row-parallel kernel's per-wave regions:
// NW x XV x 64 with XV = even(ceil(KG / NW) + 1), at most 2048 over its instantiations
constexpr int XG_ROWS_GRANULES = 2048;

// EX: the shape equals the template bounds (d0 == D0, C == CM) -> every guard folds away.
// XW > 0: in-kernel gradient all-reduce across up to XW ranks (train mode, 2 layers).
template <int L, int BMAX, int D0, int CM, bool EX, int XW>
__global__ __launch_bounds__(64) void mlp_wave_kernel(WaveShape sh, MlpArgs a) {
  constexpr int HM = 64;
  constexpr int NPF = (BMAX * D0 + BMAX + 63) / 64;  // prefetch dwords per lane
  __shared__ __attribute__((aligned(16))) float hs[L == 3 ? BMAX * HM : 4];     // layer-0 activations
  __shared__ __attribute__((aligned(16))) float ds[L == 3 ? BMAX * HM : 4];     // dh of the middle layer
  __shared__ __attribute__((aligned(16))) float w1t[L == 3 ? HM * (HM + 4) : 4];  // W1^T (rows padded)
  const int j = threadIdx.x;  // lane = hidden unit
  const int d0 = EX ? D0 : sh.d0, H1 = sh.h1, H2 = (L == 3 ? sh.h2 : sh.h1), C = EX ? CM : sh.C;
  const bool adam = (a.mode == 0);
  const bool fuse_upd = (!adam) && (a.pending != nullptr);  // apply pending Adam, then grad
  const bool need_mv = adam || fuse_upd;
  const bool own1 = j < H1;
  const bool own2 = j < H2;  // unit of the last hidden layer

  // ---------------------------------------------------------------- parameters -> registers
  float w0[D0], mw0[D0], vw0[D0];
  float b0 = 0.f, mb0 = 0.f, vb0 = 0.f;
  float wo[CM], mwo[CM], vwo[CM];
  float bo = 0.f, mbo = 0.f, vbo = 0.f;  // lane c < C owns bout[c]
  float w1[L == 3 ? HM : 1], mw1[L == 3 ? HM : 1], vw1[L == 3 ? HM : 1];
  float b1 = 0.f, mb1 = 0.f, vb1 = 0.f;
  const int lo = L - 1;  // index of the output layer
#pragma unroll
  for (int k = 0; k < D0; ++k) {
    const bool ok = own1 && k < d0;
    const int f = sh.woff[0] + j * d0 + k;
    w0[k] = ok ? a.p[f] : 0.f;
    mw0[k] = (ok && need_mv) ? a.m[f] : 0.f;
    vw0[k] = (ok && need_mv) ? a.v[f] : 0.f;
  }
  if (own1) {
    b0 = a.p[sh.boff[0] + j];
    if (need_mv) { mb0 = a.m[sh.boff[0] + j]; vb0 = a.v[sh.boff[0] + j]; }
  }
  if (L == 3) {
#pragma unroll
    for (int i = 0; i < (L == 3 ? HM : 1); ++i) {
      const bool ok = own2 && i < H1;
      const int f = sh.woff[1] + j * H1 + i;
      w1[i] = ok ? a.p[f] : 0.f;
      mw1[i] = (ok && need_mv) ? a.m[f] : 0.f;
      vw1[i] = (ok && need_mv) ? a.v[f] : 0.f;
    }
    if (own2) {
      b1 = a.p[sh.boff[1] + j];
      if (need_mv) { mb1 = a.m[sh.boff[1] + j]; vb1 = a.v[sh.boff[1] + j]; }
    }
  }
#pragma unroll
  for (int c = 0; c < CM; ++c) {
    const bool ok = own2 && c < C;
    const int f = sh.woff[lo] + c * H2 + j;
    wo[c] = ok ? a.p[f] : 0.f;
    mwo[c] = (ok && need_mv) ? a.m[f] : 0.f;
    vwo[c] = (ok && need_mv) ? a.v[f] : 0.f;
  }
  if (j < C) {
    bo = a.p[sh.boff[lo] + j];
    if (need_mv) { mbo = a.m[sh.boff[lo] + j]; vbo = a.v[sh.boff[lo] + j]; }
  }
  int t0 = a.t0;
  uint32_t step_base = a.step_base;
  if (a.step_counter) {
    t0 = __hip_atomic_load(a.step_counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    step_base = (uint32_t)t0;
  }
  if (fuse_upd && __hip_atomic_load(a.pending, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
    // previous step's all-reduced gradients are in grad_out: apply its Adam update first
    const float tt = (float)t0;
    const float step_size = a.lr * __builtin_amdgcn_rcpf(1.f - pow_t(log2f(a.b1), tt));
    const float rbc2 = __builtin_amdgcn_rsqf(1.f - pow_t(log2f(a.b2), tt));
    if (own1) {
#pragma unroll
      for (int k = 0; k < D0; ++k)
        if (k < d0) adam1(w0[k], a.grad_out[sh.woff[0] + j * d0 + k], mw0[k], vw0[k], a.b1, a.b2, a.wd, step_size, rbc2, a.eps);
      adam1(b0, a.grad_out[sh.boff[0] + j], mb0, vb0, a.b1, a.b2, a.wd, step_size, rbc2, a.eps);
    }
    if (L == 3 && own2) {
#pragma unroll
      for (int i = 0; i < (L == 3 ? HM : 1); ++i)
        if (i < H1) adam1(w1[i], a.grad_out[sh.woff[1] + j * H1 + i], mw1[i], vw1[i], a.b1, a.b2, a.wd, step_size, rbc2, a.eps);
      adam1(b1, a.grad_out[sh.boff[1] + j], mb1, vb1, a.b1, a.b2, a.wd, step_size, rbc2, a.eps);
    }
    if (own2) {
#pragma unroll
      for (int c = 0; c < CM; ++c)
        if (c < C) adam1(wo[c], a.grad_out[sh.woff[lo] + c * H2 + j], mwo[c], vwo[c], a.b1, a.b2, a.wd, step_size, rbc2, a.eps);
    }
    if (j < C) adam1(bo, a.grad_out[sh.boff[lo] + j], mbo, vbo, a.b1, a.b2, a.wd, step_size, rbc2, a.eps);
  }
  if (L == 3) {  // W1^T (row i = column i of W1) for the middle layer's backward
#pragma unroll
    for (int i = 0; i < (L == 3 ? HM : 1); ++i) w1t[i * (HM + 4) + j] = w1[i];
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  }

  int cur0 = 0;
  if (a.cursor) {
    cur0 = __hip_atomic_load(a.cursor, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (j == 0 && cur0 > 0 && a.loss_out) a.loss_out[cur0 - 1] = a.grad_out[sh.P];
  }
  const int B = a.B;

  // ---------------------------------------------------------------- batch prefetch
  // slot r of lane j holds element e = j + 64 r: x[b][k] (e < BMAX*D0) or label b (next BMAX).
  // Depth-2 pipeline: idx of batch s+2 and the x/label dwords of batch s+1 are issued at the
  // top of step s; neither is consumed in step s, so no wait lands inside the step.
  auto slot_of = [&](int r, int& b, int& k, bool& isx) {
    const int e = j + 64 * r;
    isx = e < BMAX * D0;
    if (isx) { b = e / D0; k = e - b * D0; } else { b = e - BMAX * D0; k = 0; }
  };
  auto load_idx = [&](int sbatch, int (&ridx)[NPF]) {
#pragma unroll
    for (int r = 0; r < NPF; ++r) {
      int b, k; bool isx;
      slot_of(r, b, k, isx);
      int qi = sbatch * B + (b < BMAX ? b : 0);
      qi = (qi < a.n_items && qi >= 0) ? qi : 0;
      ridx[r] = a.idx[qi];
    }
  };
  auto load_vals = [&](int sbatch, const int (&ridx)[NPF], uint32_t (&raw)[NPF]) {
    const int bsz = min(B, a.n_items - sbatch * B);
#pragma unroll
    for (int r = 0; r < NPF; ++r) {
      int b, k; bool isx;
      slot_of(r, b, k, isx);
      const bool ok = (b < bsz) && (b < BMAX) && (!isx || k < d0);
      const uint32_t* src = isx ? reinterpret_cast<const uint32_t*>(a.X) + (size_t)ridx[r] * a.ldx + (k < d0 ? k : 0)
                                : reinterpret_cast<const uint32_t*>(a.Y) + ridx[r];
      const uint32_t v = *src;
      raw[r] = ok ? v : 0u;
    }
  };
  uint32_t cur[NPF], nxt[NPF];
  int ridx_a[NPF], ridx_b[NPF];
  bool staged = false;
  if (a.stage) {
    const int tag = (int)__hip_atomic_load(&a.stage[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int r = 0; r < NPF; ++r) cur[r] = a.stage[64 + r * 64 + j];
    staged = (tag == cur0 + 1);  // tag stores batch index + 1 (0 = empty)
  }
  if (!staged) {
    load_idx(cur0, ridx_a);
    load_vals(cur0, ridx_a, cur);
  }
  load_idx(cur0 + 1, ridx_a);  // idx of batch cur0 + 1

  const float keep_scale = (a.dropout > 0.f) ? 1.0f / (1.0f - a.dropout) : 1.0f;
  const float l2b1 = log2f(a.b1), l2b2 = log2f(a.b2);  // hoisted: bias corrections are exp2 per step
  const uint32_t drop_thr = (uint32_t)(a.dropout * 4294967296.0);
  const bool prof = (a.prof != nullptr) && j == 0;
  if (prof) a.prof[30] = __builtin_amdgcn_s_memrealtime();
  // diagnostic phase stamps (shader clock, wave-uniform branch; never set in production)
  const bool profu = a.prof != nullptr;
  unsigned long long pt[6] = {0, 0, 0, 0, 0, 0}, tprev = 0;
#ifndef WAVE_PROF_BUILD
#define WSTAMP(k)
#else
#define WSTAMP(k)                                                                          \
  if (profu) {                                                                             \
    unsigned long long t_;                                                                 \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");            \
    if ((k) >= 0) pt[(k) < 0 ? 0 : (k)] += t_ - tprev;                                     \
    tprev = t_;                                                                            \
  }
#endif
  constexpr bool XG = XW > 0;
  constexpr int XWN = XW > 0 ? XW : 1;
  __amdgpu_buffer_rsrc_t prs[XWN];
  __amdgpu_buffer_rsrc_t rrs = __builtin_amdgcn_make_buffer_rsrc(a.xg_recv, 0, 0, 0x00020000);
  if (XG) {
    const int nbytes = 2 * a.xg_world * (D0 + CM + 2 + ((D0 + CM) & 1)) * 64 * 8;
    rrs = __builtin_amdgcn_make_buffer_rsrc(a.xg_recv, 0, nbytes, 0x00020000);
#pragma unroll
    for (int q = 0; q < XWN; ++q) {
      void* pq = (q < a.xg_world) ? (void*)sload_ptr(a.xg_peers, q) : (void*)a.xg_recv;
      prs[q] = __builtin_amdgcn_make_buffer_rsrc(pq, 0, nbytes, 0x00020000);
    }
  }
  int done = a.steps;

  for (int s = 0; s < a.steps; ++s) {
    const int sb = s + cur0;
    const int bs = min(B, a.n_items - sb * B);
    const uint32_t gstep = step_base + (uint32_t)s;
    WSTAMP(-1)
    // issue: values of batch sb+1 (idx already in registers) and idx of batch sb+2
    load_vals(sb + 1, ridx_a, nxt);
    load_idx(sb + 2, ridx_b);

    // broadcast the current batch: x[b][k] and labels -> SGPR-uniform values
    float x[BMAX][D0];
    int y[BMAX];
#pragma unroll
    for (int b = 0; b < BMAX; ++b) {
#pragma unroll
      for (int k = 0; k < D0; ++k) {
        const int e = b * D0 + k;
        x[b][k] = __int_as_float(__builtin_amdgcn_readlane((int)cur[e / 64], e % 64));
      }
      const int e = BMAX * D0 + b;
      y[b] = __builtin_amdgcn_readlane((int)cur[e / 64], e % 64);
    }

    // ---- layer 0: h[b] = dropout(relu(W0[j] . x[b] + b0))
    const uint32_t hkey = (a.seed * 0x9E3779B1u) ^ (gstep * 0x85EBCA77u);
    float h[BMAX];
#pragma unroll
    for (int b = 0; b < BMAX; ++b) {
      float z = b0;
#pragma unroll
      for (int k = 0; k < D0; ++k) z += w0[k] * x[b][k];
      z = fmaxf(z, 0.f);
      if (drop_thr) {
        const uint32_t r = wave_hash(hkey ^ ((uint32_t)(b * 64 + j) * 0xC2B2AE3Du));
        z = (r < drop_thr) ? 0.f : z * keep_scale;
      }
      h[b] = own1 ? z : 0.f;
    }
    WSTAMP(0)
    // ---- middle layer (3-layer nets): h2[b] = dropout(relu(W1[j] . h[b] + b1))
    float h2[BMAX];
    if (L == 3) {
#pragma unroll
      for (int b = 0; b < BMAX; ++b) hs[b * HM + j] = h[b];
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS writes done (in-order DS)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
      for (int b = 0; b < BMAX; ++b) {
        float z = b1;
#pragma unroll
        for (int i4 = 0; i4 < HM / 4; ++i4) {
          const float4 hv = *reinterpret_cast<const float4*>(&hs[b * HM + i4 * 4]);
          z += w1[i4 * 4 + 0] * hv.x + w1[i4 * 4 + 1] * hv.y + w1[i4 * 4 + 2] * hv.z + w1[i4 * 4 + 3] * hv.w;
        }
        z = fmaxf(z, 0.f);
        if (drop_thr) {
          const uint32_t r = wave_hash(hkey ^ ((uint32_t)(4096 + b * 64 + j) * 0xC2B2AE3Du));
          z = (r < drop_thr) ? 0.f : z * keep_scale;
        }
        h2[b] = own2 ? z : 0.f;
      }
    } else {
#pragma unroll
      for (int b = 0; b < BMAX; ++b) h2[b] = h[b];
    }
    // ---- output layer: logits[b][c] = sum_j Wout[c][j] h2_j[b] + bout[c]  (cross-lane)
    float zc[BMAX * CM];
#pragma unroll
    for (int b = 0; b < BMAX; ++b)
#pragma unroll
      for (int c = 0; c < CM; ++c) zc[b * CM + c] = wo[c] * h2[b];
    wave_sum_n(zc);
    float boc[CM];
#pragma unroll
    for (int c = 0; c < CM; ++c) boc[c] = rl(bo, c);
    WSTAMP(1)
    // ---- loss + dlogits (wave-uniform, computed redundantly in every lane)
    float dz[BMAX * CM];
    float lsum = 0.f;
    const float inv = __builtin_amdgcn_rcpf((float)(bs > 0 ? bs : 1));  // bs <= 8: exact
    // the loss-kind branch is hoisted out of the row loop: a branch per row made every row a
    // basic block of its own and serialised their exp/log latency chains (~1.2k cycles / step)
    if (a.loss_kind == 0) {
#pragma unroll
      for (int b = 0; b < BMAX; ++b) {
        const bool live = b < bs;
        float zz[CM];
#pragma unroll
        for (int c = 0; c < CM; ++c) zz[c] = zc[b * CM + c] + boc[c];
        float mx = -3.402823466e+38f;
#pragma unroll
        for (int c = 0; c < CM; ++c)
          if (c < C) mx = fmaxf(mx, zz[c]);
        float e[CM], se = 0.f, zy = 0.f;
#pragma unroll
        for (int c = 0; c < CM; ++c) {
          e[c] = (c < C) ? __builtin_amdgcn_exp2f((zz[c] - mx) * 1.4426950408889634f) : 0.f;
          se += e[c];
          zy = (c == y[b]) ? zz[c] : zy;
        }
        const float lb = mx + __builtin_amdgcn_logf(se) * 0.69314718055994531f - zy;  // se in [1, C]
        const float rs = __builtin_amdgcn_rcpf(se);
#pragma unroll
        for (int c = 0; c < CM; ++c) dz[b * CM + c] = live ? (e[c] * rs - (c == y[b] ? 1.f : 0.f)) * inv : 0.f;
        lsum += live ? lb : 0.f;
      }
    } else {
      const float sc = 2.f / (float)C;
#pragma unroll
      for (int b = 0; b < BMAX; ++b) {
        const bool live = b < bs;
        float lb = 0.f;
#pragma unroll
        for (int c = 0; c < CM; ++c) {
          const float zz = zc[b * CM + c] + boc[c];
          const float d = (c < C) ? zz - (c == y[b] ? 1.f : 0.f) : 0.f;
          lb += d * d;
          dz[b * CM + c] = live ? d * sc * inv : 0.f;
        }
        lsum += live ? lb / (float)C : 0.f;
      }
    }
    if (j == 0) {
      const float bl = bs > 0 ? lsum * inv : 0.f;
      if (a.loss_out && !a.cursor && !XG) a.loss_out[s] = bl;
      if (!adam) a.grad_out[sh.P] = bl;
    }

    WSTAMP(2)
    // ---- backward (lane-local)
    float gwo[CM], gbo = 0.f;
#pragma unroll
    for (int c = 0; c < CM; ++c) {
      float g = 0.f;
#pragma unroll
      for (int b = 0; b < BMAX; ++b) g += dz[b * CM + c] * h2[b];
      gwo[c] = g;
    }
#pragma unroll
    for (int c = 0; c < CM; ++c) {
      float g = 0.f;
#pragma unroll
      for (int b = 0; b < BMAX; ++b) g += dz[b * CM + c];
      if (c == j) gbo = g;
    }
    float dh2[BMAX];  // dL/dpre-activation of the last hidden layer
#pragma unroll
    for (int b = 0; b < BMAX; ++b) {
      float g = 0.f;
#pragma unroll
      for (int c = 0; c < CM; ++c) g += dz[b * CM + c] * wo[c];
      dh2[b] = (h2[b] > 0.f) ? g * keep_scale : 0.f;
    }
    float dh[BMAX];
    float gw1[L == 3 ? HM : 1], gb1 = 0.f;
    if (L == 3) {
      // dW1[j][i] = sum_b dh2_j[b] h_i[b]  (h_i from the LDS tile), db1 = sum_b dh2
#pragma unroll
      for (int i = 0; i < (L == 3 ? HM : 1); ++i) gw1[i] = 0.f;
#pragma unroll
      for (int b = 0; b < BMAX; ++b) {
#pragma unroll
        for (int i4 = 0; i4 < HM / 4; ++i4) {
          const float4 hv = *reinterpret_cast<const float4*>(&hs[b * HM + i4 * 4]);
          gw1[i4 * 4 + 0] += dh2[b] * hv.x;
          gw1[i4 * 4 + 1] += dh2[b] * hv.y;
          gw1[i4 * 4 + 2] += dh2[b] * hv.z;
          gw1[i4 * 4 + 3] += dh2[b] * hv.w;
        }
        gb1 += dh2[b];
      }
      // dh_i[b] = sum_j W1[j][i] dh2_j[b]  via W1^T rows in LDS and dh2 broadcast
#pragma unroll
      for (int b = 0; b < BMAX; ++b) ds[b * HM + j] = dh2[b];
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
      for (int b = 0; b < BMAX; ++b) {
        float g = 0.f;
#pragma unroll
        for (int i4 = 0; i4 < HM / 4; ++i4) {
          const float4 wt = *reinterpret_cast<const float4*>(&w1t[j * (HM + 4) + i4 * 4]);
          const float4 dv = *reinterpret_cast<const float4*>(&ds[b * HM + i4 * 4]);
          g += wt.x * dv.x + wt.y * dv.y + wt.z * dv.z + wt.w * dv.w;
        }
        dh[b] = (h[b] > 0.f) ? g * keep_scale : 0.f;
      }
    } else {
#pragma unroll
      for (int b = 0; b < BMAX; ++b) dh[b] = dh2[b];
    }
    float gw0[D0], gb0 = 0.f;
#pragma unroll
    for (int k = 0; k < D0; ++k) {
      float g = 0.f;
#pragma unroll
      for (int b = 0; b < BMAX; ++b) g += dh[b] * x[b][k];
      gw0[k] = g;
    }
#pragma unroll
    for (int b = 0; b < BMAX; ++b) gb0 += dh[b];

    WSTAMP(3)
    if (XG) {  // average the gradients (and the batch loss) across ranks in-kernel
      static_assert(!XG || L == 2, "in-kernel all-reduce is implemented for 2-layer nets");
      constexpr int KX = D0 + CM + 2 + ((D0 + CM) & 1);  // even: 16-B granule pairs
      float gv[KX];
#pragma unroll
      for (int k = 0; k < KX; ++k) gv[k] = 0.f;
#pragma unroll
      for (int k = 0; k < D0; ++k) gv[k] = gw0[k];
      gv[D0] = gb0;
#pragma unroll
      for (int c = 0; c < CM; ++c) gv[D0 + 1 + c] = gwo[c];
      const float bl = bs > 0 ? lsum * inv : 0.f;
      gv[D0 + 1 + CM] = (j < C) ? gbo : (j == 63 ? bl : 0.f);  // bias grads + the batch loss
      const unsigned long long tx = prof ? __builtin_amdgcn_s_memrealtime() : 0ull;
      if (!xg_allreduce<KX, XWN>(gv, a, prs, rrs, gstep, j)) {
        done = s;
        break;
      }
      if (prof) a.prof[29] += __builtin_amdgcn_s_memrealtime() - tx;
#pragma unroll
      for (int k = 0; k < D0; ++k) gw0[k] = gv[k];
      gb0 = gv[D0];
#pragma unroll
      for (int c = 0; c < CM; ++c) gwo[c] = gv[D0 + 1 + c];
      gbo = gv[D0 + 1 + CM];
      const float lavg = rl(gv[D0 + 1 + CM], 63);
      if (j == 0 && a.loss_out && !a.cursor) a.loss_out[s] = lavg;
    }
    WSTAMP(4)
    if (adam) {
      const int t = t0 + s + 1;
      const float step_size = a.lr * __builtin_amdgcn_rcpf(1.f - pow_t(l2b1, (float)t));
      const float rbc2 = __builtin_amdgcn_rsqf(1.f - pow_t(l2b2, (float)t));
      if (own1) {
#pragma unroll
        for (int k = 0; k < D0; ++k)
          if (k < d0) adam1(w0[k], gw0[k], mw0[k], vw0[k], a.b1, a.b2, a.wd, step_size, rbc2, a.eps);
        adam1(b0, gb0, mb0, vb0, a.b1, a.b2, a.wd, step_size, rbc2, a.eps);
      }
      if (L == 3 && own2) {
#pragma unroll
        for (int i = 0; i < (L == 3 ? HM : 1); ++i)
          if (i < H1) adam1(w1[i], gw1[i], mw1[i], vw1[i], a.b1, a.b2, a.wd, step_size, rbc2, a.eps);
        adam1(b1, gb1, mb1, vb1, a.b1, a.b2, a.wd, step_size, rbc2, a.eps);
      }
      if (own2) {
#pragma unroll
        for (int c = 0; c < CM; ++c)
          if (c < C) adam1(wo[c], gwo[c], mwo[c], vwo[c], a.b1, a.b2, a.wd, step_size, rbc2, a.eps);
      }
      if (j < C) adam1(bo, gbo, mbo, vbo, a.b1, a.b2, a.wd, step_size, rbc2, a.eps);
      if (L == 3) {  // refresh W1^T for the next step's backward
#pragma unroll
        for (int i = 0; i < (L == 3 ? HM : 1); ++i) w1t[i * (HM + 4) + j] = w1[i];
      }
    } else {
      if (own1) {
#pragma unroll
        for (int k = 0; k < D0; ++k)
          if (k < d0) a.grad_out[sh.woff[0] + j * d0 + k] = gw0[k];
        a.grad_out[sh.boff[0] + j] = gb0;
      }
      if (L == 3 && own2) {
#pragma unroll
        for (int i = 0; i < (L == 3 ? HM : 1); ++i)
          if (i < H1) a.grad_out[sh.woff[1] + j * H1 + i] = gw1[i];
        a.grad_out[sh.boff[1] + j] = gb1;
      }
      if (own2) {
#pragma unroll
        for (int c = 0; c < CM; ++c)
          if (c < C) a.grad_out[sh.woff[lo] + c * H2 + j] = gwo[c];
      }
      if (j < C) a.grad_out[sh.boff[lo] + j] = gbo;
    }
    WSTAMP(5)
#pragma unroll
    for (int r = 0; r < NPF; ++r) {
      cur[r] = nxt[r];
      ridx_a[r] = ridx_b[r];
    }
  }
#undef WSTAMP
  if (prof) {
    a.prof[31] = __builtin_amdgcn_s_memrealtime();
#pragma unroll
    for (int k = 0; k < 6; ++k) a.prof[k] = pt[k];
  }
  if (a.stage) {  // hand the already-fetched next batch to the next launch
    const int nb = cur0 + done;
    const bool ok = nb * B < a.n_items;
    if (ok) {
#pragma unroll
      for (int r = 0; r < NPF; ++r) a.stage[64 + r * 64 + j] = cur[r];
    }
    __builtin_amdgcn_s_waitcnt(0);  // every lane's stage stores complete before the tag
    if (j == 0) __hip_atomic_store(&a.stage[0], ok ? (uint32_t)(nb + 1) : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (a.cursor && j == 0) __hip_atomic_store(a.cursor, cur0 + done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (a.step_counter && j == 0)
    __hip_atomic_store(a.step_counter, t0 + done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (fuse_upd && j == 0) __hip_atomic_store(a.pending, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (!need_mv) return;
  // ---- write back params + moments
#pragma unroll
  for (int k = 0; k < D0; ++k) {
    if (own1 && k < d0) {
      const int f = sh.woff[0] + j * d0 + k;
      a.p[f] = w0[k]; a.m[f] = mw0[k]; a.v[f] = vw0[k];
    }
  }
  if (own1) {
    const int f = sh.boff[0] + j;
    a.p[f] = b0; a.m[f] = mb0; a.v[f] = vb0;
  }
  if (L == 3 && own2) {
#pragma unroll
    for (int i = 0; i < (L == 3 ? HM : 1); ++i) {
      if (i < H1) {
        const int f = sh.woff[1] + j * H1 + i;
        a.p[f] = w1[i]; a.m[f] = mw1[i]; a.v[f] = vw1[i];
      }
    }
    const int f = sh.boff[1] + j;
    a.p[f] = b1; a.m[f] = mb1; a.v[f] = vb1;
  }
#pragma unroll
  for (int c = 0; c < CM; ++c) {
    if (own2 && c < C) {
      const int f = sh.woff[lo] + c * H2 + j;
      a.p[f] = wo[c]; a.m[f] = mwo[c]; a.v[f] = vwo[c];
    }
  }
  if (j < C) {
    const int f = sh.boff[lo] + j;
    a.p[f] = bo; a.m[f] = mbo; a.v[f] = vbo;
  }
}


// ============================================================================ row-parallel
// Row-parallel variant of the 2-layer train step (mode 0): ONE WAVE PER BATCH ROW.
//
// The single-wave kernel above is issue-bound: one wave64 issues every VALU instruction over
// 4 cycles on ONE SIMD16 of the CU, and a step is ~650 instructions (~3k cycles, 1.35 us).
// Here wave w (NW = 4 or 8 waves spread over the CU's 4 SIMDs; rows >= B idle) runs the
// forward, loss and backward of batch row w only, then the per-row gradients meet in LDS.
// Parameter slot k (lane j owns W0[j][:], b0[j], Wout[:, j], bout[j < C] as slots 0..KG-1)
// belongs to wave k % NW: the owner runs Adam on it (its moments live only in the owner) and
// publishes the new value through LDS; after the step's last barrier every wave reads the
// parameters it does not own.  Adam's ~12 VALU ops and 2 quarter-rate transcendentals per
// slot are spread over the SIMDs.
//   * XW == 0: after barrier 1 the owner sums slot k over the rows (order 0..NW-1).
//   * XW > 0: every wave runs the in-kernel xGMI exchange of ITS owned slots (and wave 0 of the
//     batch loss) in its own region of the receive buffer (xg_exchange_wave), so the waves push
//     and poll in parallel; Adam on the rank average is tentative until barrier 2 has shown
//     that no wave's exchange timed out (then all waves undo the step and leave together).
// Row sums run in a fixed order, so the result is bit-identical across waves and ranks.
template <int NW, int KG, bool XG>
struct RowsLds {
  float gslot[2][NW][KG][64];  // [step parity][row][slot][lane] per-row gradients
  float lslot[2][NW];          // per-row losses
  float pslot[KG][64];         // parameters published by their owner
  int xab[NW];                 // per-wave exchange timeout flags (XW > 0)
};

// The whole per-wave program with the wave id W as a compile-time constant, so slot ownership
// (k % NW == W) folds away instead of becoming a branch per slot.
template <int NW, int W, int D0, int CM, bool EX, int XW, bool REP>
__device__ __forceinline__ void mlp_rows_wave(const WaveShape& sh, const MlpArgs& a,
                                              RowsLds<NW, D0 + CM + 2, (XW > 0)>& L) {
  constexpr int KG = D0 + 1 + CM + 1;  // per-lane parameter slots: W0 row, b0, Wout column, bout
  constexpr int KB = D0;               // slot of b0
  constexpr int KO = D0 + 1;           // first slot of the Wout column
  constexpr int KC = D0 + 1 + CM;      // slot of bout (lanes < C)
  constexpr bool XG = XW > 0;
  auto& gslot = L.gslot;
  auto& lslot = L.lslot;
  auto& pslot = L.pslot;
  auto& xab = L.xab;
  const int j = threadIdx.x & 63;
  constexpr int w = W;  // wave = batch row
  const int d0 = EX ? D0 : sh.d0, H1 = sh.h1, C = EX ? CM : sh.C;
  const bool own1 = j < H1;

  // lane j's slot k: live in this lane?  flat index in p/m/v
  auto slot_live = [&](int k) -> bool {
    if (k < KB) return own1 && k < d0;
    if (k == KB) return own1;
    if (k < KC) return own1 && (k - KO) < C;
    return j < C;
  };
  auto slot_flat = [&](int k) -> int {
    if (k < KB) return sh.woff[0] + j * d0 + (k < d0 ? k : 0);
    if (k == KB) return sh.boff[0] + j;
    if (k < KC) return sh.woff[1] + (k - KO) * H1 + j;
    return sh.boff[1] + j;
  };
  // REP: every wave runs Adam on every slot (one barrier per step instead of two).  Measured on
  // the weather step it loses to the owner split: 0.893 vs 0.732 us/step (MI355X, round 2).
  // slot k -> wave (k + 1) % NW: the wave that owns an extra slot is not wave 0, which also sums
  // the batch loss
  auto owned = [](int k) constexpr -> bool { return REP || ((k + 1) % NW) == W; };

  // ---------------------------------------------------------------- parameters -> registers
  float pr[KG], mr[KG], vr[KG];
#pragma unroll
  for (int k = 0; k < KG; ++k) {
    const bool ok = slot_live(k);
    const int f = ok ? slot_flat(k) : 0;
    pr[k] = ok ? a.p[f] : 0.f;
    mr[k] = (ok && owned(k)) ? a.m[f] : 0.f;
    vr[k] = (ok && owned(k)) ? a.v[f] : 0.f;
  }
  int t0 = a.t0;
  uint32_t step_base = a.step_base;
  if (a.step_counter) {
    t0 = __hip_atomic_load(a.step_counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    step_base = (uint32_t)t0;
  }
  const int B = a.B;

  // ---------------------------------------------------------------- row prefetch
  // Lane k < D0 fetches x[row][k], lane D0 the label.  The random row gathers miss L2, and a
  // step (~0.5 us) is shorter than that latency, so loads run PF steps ahead: the row index of
  // step s+2PF and the values of step s+PF are issued at step s, into ring registers indexed by
  // s % PF.  The step loop is unrolled PF times so the ring never rotates through register moves
  // (a move of a register with a load in flight would wait for that load).
  // Lane j loads the index of row (j & 7): the loaded value is not wave-uniform, so the compiler
  // keeps it in a VGPR instead of a v_readfirstlane right behind the load (which would wait on
  // it); the row's index is picked with v_readlane when the value load is issued.
  constexpr int PF = 4;
  auto load_idx = [&](int sbatch) -> int {
    int qi = sbatch * B + (j & 7);
    qi = (qi < a.n_items && qi >= 0) ? qi : 0;
    return a.idx[qi];
  };
  auto load_val = [&](int ridx_v) -> uint32_t {
    const int ridx = __builtin_amdgcn_readlane(ridx_v, w);
    const int k = (j < d0) ? j : 0;
    const uint32_t* src = (j < D0) ? reinterpret_cast<const uint32_t*>(a.X) + (size_t)ridx * a.ldx + k
                                   : reinterpret_cast<const uint32_t*>(a.Y) + ridx;
    return *src;
  };
  uint32_t vr_ring[PF];
  int ir_ring[PF];
#pragma unroll
  for (int i = 0; i < PF; ++i) ir_ring[i] = load_idx(i);
#pragma unroll
  for (int i = 0; i < PF; ++i) {
    vr_ring[i] = load_val(ir_ring[i]);
    ir_ring[i] = load_idx(i + PF);
  }

  const float keep_scale = (a.dropout > 0.f) ? 1.0f / (1.0f - a.dropout) : 1.0f;
  const float l2b1 = log2f(a.b1), l2b2 = log2f(a.b2);
  const uint32_t drop_thr = (uint32_t)(a.dropout * 4294967296.0);
  constexpr int XWN = XW > 0 ? XW : 1;
  __amdgpu_buffer_rsrc_t prs[XWN];
  __amdgpu_buffer_rsrc_t rrs = __builtin_amdgcn_make_buffer_rsrc(a.xg_recv, 0, 0, 0x00020000);
  // exchange values per lane of this wave: its owned slots (k = w, w + NW, ...) then the batch loss
  constexpr int NOWN = (KG + NW - 1) / NW;
  constexpr int XV = (NOWN + 1 + 1) / 2 * 2;
  static_assert(NW * XV * 64 <= XG_ROWS_GRANULES, "exchange region exceeds the allocated slab");
  if (XG) {
    const int nbytes = 2 * a.xg_world * NW * XV * 64 * 8;
    rrs = __builtin_amdgcn_make_buffer_rsrc(a.xg_recv, 0, nbytes, 0x00020000);
#pragma unroll
    for (int q = 0; q < XWN; ++q) {
      void* pq = (q < a.xg_world) ? (void*)sload_ptr(a.xg_peers, q) : (void*)a.xg_recv;
      prs[q] = __builtin_amdgcn_make_buffer_rsrc(pq, 0, nbytes, 0x00020000);
    }
  }
  int done = a.steps;
  unsigned long long xg_ticks_acc = 0;

  // diagnostic phase stamps (profiling build, tools/prof_rows.py): shader-clock deltas of wave W
  // accumulated per phase; never compiled into production launches
#ifdef WAVE_PROF_BUILD
  unsigned long long rpt[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, rprev = 0;
#define RSTAMP(k)                                                                            \
  if (a.prof) {                                                                              \
    unsigned long long t_;                                                                   \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");              \
    if ((k) >= 0) rpt[(k) < 0 ? 0 : (k)] += t_ - rprev;                                      \
    rprev = t_;                                                                              \
  }
#else
#define RSTAMP(k)
#endif
  // one optimizer step; returns false when the launch must stop (exchange timeout)
  auto step = [&](const int s, uint32_t& vslot, int& islot) -> bool {
    RSTAMP(-1)
    const int bs = min(B, a.n_items - s * B);
    const bool live = w < bs;
    const uint32_t gstep = step_base + (uint32_t)s;
    const int par = s & 1;
    // this step's row leaves the ring register (readlanes) BEFORE that register is reloaded with
    // step s + PF's values: with the reload first, the old and the new value are live together,
    // the ring needs a fifth register, and the unrolled loop's back-edge rotates it with moves
    // that wait for every load in flight
    const uint32_t cur = vslot;
    float x[D0];
#pragma unroll
    for (int k = 0; k < D0; ++k) {
      const float xv = __int_as_float(__builtin_amdgcn_readlane((int)cur, k));
      x[k] = (live && k < d0) ? xv : 0.f;  // dead rows: zeros, never a stale NaN
    }
    const int y = live ? __builtin_amdgcn_readlane((int)cur, D0) : 0;
    vslot = load_val(islot);       // values of step s + PF (index loaded PF steps ago)
    islot = load_idx(s + 2 * PF);  // index of step s + 2 PF
    // step-only quantities first, branch-free: they share the basic block of the forward's
    // latency chains, so the scheduler fills its bubbles with them (a branch or the barrier
    // would fence them onto the critical path)
    const uint32_t hkey = (a.seed * 0x9E3779B1u) ^ (gstep * 0x85EBCA77u);
    const uint32_t hrnd = wave_hash(hkey ^ ((uint32_t)(w * 64 + j) * 0xC2B2AE3Du));
    const bool dropped = hrnd < drop_thr;  // drop_thr == 0: never

    RSTAMP(0)
    float g[KG];
    float lb = 0.f;
    // two-class CE: the loss VALUE (a log) is not on the gradient's path - it is formed after the
    // gradient stores, where it overlaps their LDS latency
    float ce_se = 1.f, ce_off = 0.f;
    const float inv = __builtin_amdgcn_rcpf((float)(bs > 0 ? bs : 1));  // bs <= 8: exact
    if (NW == 4 || w < B) {  // waves beyond the batch (NW = 8, B <= 4) only own Adam slots
      // ---- layer 0 for this row: h = dropout(relu(W0[j] . x + b0))
      float h;
      {
        float z = pr[KB];
#pragma unroll
        for (int k = 0; k < D0; ++k) z = fmaf(pr[k], x[k], z);
        z = fmaxf(z, 0.f) * keep_scale;  // keep_scale == 1 without dropout
        h = (own1 && !dropped) ? z : 0.f;
      }
      RSTAMP(1)
      // ---- output layer: logits[c] = sum_j Wout[c][j] h_j + bout[c]  (cross-lane, wave-uniform)
      float zc[CM];
#pragma unroll
      for (int c = 0; c < CM; ++c) zc[c] = pr[KO + c] * h;
      wave_sum_bcast(zc);
#pragma unroll
      for (int c = 0; c < CM; ++c) zc[c] += rl(pr[KC], c);

      RSTAMP(2)
      // ---- loss + dlogits of this row (wave-uniform)
      float dz[CM];
      if (a.loss_kind == 0) {
        if constexpr (EX && CM == 2) {
          // two classes: softmax = logistic of the margin; one exp, one rcp (+ the deferred log)
          const float d = zc[1] - zc[0];
          const float t = __builtin_amdgcn_exp2f(-fabsf(d) * 1.4426950408889634f);  // exp(-|d|)
          const float se = 1.f + t;
          const float rs = __builtin_amdgcn_rcpf(se);
          const float p1 = d >= 0.f ? rs : t * rs;  // softmax prob of class 1
          ce_se = se;
          ce_off = fmaxf(zc[0], zc[1]) - (y == 1 ? zc[1] : zc[0]);  // lb = ce_off + log(se)
          dz[1] = (p1 - (y == 1 ? 1.f : 0.f)) * inv;
          dz[0] = -dz[1];
        } else {
          float mx = -3.402823466e+38f;
#pragma unroll
          for (int c = 0; c < CM; ++c)
            if (c < C) mx = fmaxf(mx, zc[c]);
          float e[CM], se = 0.f, zy = 0.f;
#pragma unroll
          for (int c = 0; c < CM; ++c) {
            e[c] = (c < C) ? __builtin_amdgcn_exp2f((zc[c] - mx) * 1.4426950408889634f) : 0.f;
            se += e[c];
            zy = (c == y) ? zc[c] : zy;
          }
          lb = mx + __builtin_amdgcn_logf(se) * 0.69314718055994531f - zy;
          const float rs = __builtin_amdgcn_rcpf(se);
#pragma unroll
          for (int c = 0; c < CM; ++c) dz[c] = (e[c] * rs - (c == y ? 1.f : 0.f)) * inv;
        }
      } else {
        const float sc = 2.f / (float)C;
#pragma unroll
        for (int c = 0; c < CM; ++c) {
          const float d = (c < C) ? zc[c] - (c == y ? 1.f : 0.f) : 0.f;
          lb += d * d;
          dz[c] = d * sc * inv;
        }
        lb *= 1.f / (float)C;
      }
#pragma unroll
      for (int c = 0; c < CM; ++c) dz[c] = live ? dz[c] : 0.f;
      lb = live ? lb : 0.f;

      RSTAMP(3)
      // ---- backward of this row (lane-local) -> per-row gradient of every slot
      {
        float gsum = 0.f;
#pragma unroll
        for (int c = 0; c < CM; ++c) gsum = fmaf(dz[c], pr[KO + c], gsum);
        const float dh = (h > 0.f) ? gsum * keep_scale : 0.f;
#pragma unroll
        for (int k = 0; k < D0; ++k) g[k] = dh * x[k];
        g[KB] = dh;
#pragma unroll
        for (int c = 0; c < CM; ++c) g[KO + c] = dz[c] * h;
        float gbo = 0.f;
#pragma unroll
        for (int c = 0; c < CM; ++c) gbo = (c == j) ? dz[c] : gbo;
        g[KC] = gbo;
      }
    } else {
#pragma unroll
      for (int k = 0; k < KG; ++k) g[k] = 0.f;
    }
#pragma unroll
    for (int k = 0; k < KG; ++k) gslot[par][w][k][j] = g[k];
    // off the gradient path, overlapping the stores' LDS latency: the deferred CE value and the
    // step's Adam bias-correction scalars
    if constexpr (EX && CM == 2) {
      if (a.loss_kind == 0) lb = live ? ce_off + __builtin_amdgcn_logf(ce_se) * 0.69314718055994531f : 0.f;
    }
    if (j == 0) lslot[par][w] = lb;
    const int t_adam = t0 + s + 1;
    const float step_size = a.lr * __builtin_amdgcn_rcpf(1.f - pow_t(l2b1, (float)t_adam));
    const float rbc2 = __builtin_amdgcn_rsqf(1.f - pow_t(l2b2, (float)t_adam));
    RSTAMP(4)
    __syncthreads();  // barrier 1: every row's gradients are in LDS
    RSTAMP(5)

    // ---- batch gradient of the owned slots: rows summed in order 0..NW-1
#pragma unroll
    for (int k = 0; k < KG; ++k) {
      if (owned(k)) {
        float acc = gslot[par][0][k][j];
#pragma unroll
        for (int r = 1; r < NW; ++r) acc += gslot[par][r][k][j];
        g[k] = acc;
      }
    }
    float bl = 0.f;
    if (w == 0) {
#pragma unroll
      for (int r = 0; r < NW; ++r) bl += lslot[par][r];
      bl *= inv;
    }
    bool xg_ok = true;
    if constexpr (XG) {  // rank average of the owned slots (and of the batch loss, wave 0)
      float xv[XV];
#pragma unroll
      for (int i = 0; i < XV; ++i) xv[i] = 0.f;
#pragma unroll
      for (int k = 0; k < KG; ++k)
        if (owned(k)) xv[k / NW] = g[k];
      xv[XV - 1] = bl;  // wave 0's batch loss (0 in the other waves)
      const bool timing = (w == 0) && (a.xg_ticks != nullptr);
      const unsigned long long tx = timing ? __builtin_amdgcn_s_memrealtime() : 0ull;
      xg_ok = xg_exchange_wave<XV, XWN>(xv, a, prs, rrs, gstep, j, w, NW);
      if (timing) xg_ticks_acc += __builtin_amdgcn_s_memrealtime() - tx;
#pragma unroll
      for (int k = 0; k < KG; ++k)
        if (owned(k)) g[k] = xv[k / NW];
      bl = xv[XV - 1];
    }

    RSTAMP(6)
    // ---- Adam on the owned slots (tentative with XW > 0: undone if any wave's exchange timed out)
    float bkp[KG], bkm[KG], bkv[KG];
    if constexpr (XG) {
#pragma unroll
      for (int k = 0; k < KG; ++k)
        if (owned(k)) { bkp[k] = pr[k]; bkm[k] = mr[k]; bkv[k] = vr[k]; }
    }
#pragma unroll
    for (int k = 0; k < KG; ++k) {
      if (owned(k) && slot_live(k)) adam1(pr[k], g[k], mr[k], vr[k], a.b1, a.b2, a.wd, step_size, rbc2, a.eps);
    }
    RSTAMP(7)
    if constexpr (!REP) {  // publish owned slots; read the others after the next barrier
#pragma unroll
      for (int k = 0; k < KG; ++k)
        if (owned(k)) pslot[k][j] = pr[k];
      if (XG && j == 0) xab[w] = xg_ok ? 0 : 1;
      __syncthreads();
      if constexpr (XG) {
        bool abort = false;
#pragma unroll
        for (int r = 0; r < NW; ++r) abort |= (xab[r] != 0);
        if (abort) {  // every wave sees the same flags: all leave before this step
#pragma unroll
          for (int k = 0; k < KG; ++k)
            if (owned(k)) { pr[k] = bkp[k]; mr[k] = bkm[k]; vr[k] = bkv[k]; }
          done = s;
          return false;
        }
      }
#pragma unroll
      for (int k = 0; k < KG; ++k)
        if (!owned(k)) pr[k] = pslot[k][j];
    }
    if (w == 0 && j == 0 && a.loss_out) a.loss_out[s] = bl;
    RSTAMP(8)
    return true;
  };
  // Whole PF-step groups run unconditionally, the remainder after the loop: a per-step "s < steps"
  // guard inside the loop gives the back-edge a path that skips the later steps' loads, and the
  // wait-count pass, merging that path at the loop header, then drains every load in flight
  // (vmcnt(0)) once per group.  A failed exchange leaves both loops directly (no back-edge path).
  int s0 = 0;
  for (; s0 + PF <= a.steps; s0 += PF) {
#pragma unroll
    for (int i = 0; i < PF; ++i)
      if (!step(s0 + i, vr_ring[i], ir_ring[i])) goto steps_done;
  }
#pragma unroll
  for (int i = 0; i < PF - 1; ++i)
    if (s0 + i < a.steps && !step(s0 + i, vr_ring[i], ir_ring[i])) goto steps_done;
steps_done:
#ifdef WAVE_PROF_BUILD
  if (a.prof && j == 0) {  // wave W's phase sums at prof[16 W + k]
#pragma unroll
    for (int k = 0; k < 10; ++k) a.prof[16 * W + k] = rpt[k];
  }
#endif
#undef RSTAMP
  if (w == 0 && a.step_counter && j == 0)
    __hip_atomic_store(a.step_counter, t0 + done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (XG && w == 0 && j == 0 && a.xg_ticks)
    __hip_atomic_fetch_add(a.xg_ticks, xg_ticks_acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // ---- write back: every wave holds the same parameters; each slot's moments live in its owner
#pragma unroll
  for (int k = 0; k < KG; ++k) {
    if (slot_live(k) && owned(k) && (!REP || w == 0)) {
      const int f = slot_flat(k);
      a.p[f] = pr[k]; a.m[f] = mr[k]; a.v[f] = vr[k];
    }
  }
}

template <int NW, int D0, int CM, bool EX, int XW, bool REP = false>
__global__ __launch_bounds__(64 * NW) void mlp_rows_kernel(WaveShape sh, MlpArgs a) {
  __shared__ RowsLds<NW, D0 + CM + 2, (XW > 0)> lds;
  switch (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) {
    case 0: mlp_rows_wave<NW, 0, D0, CM, EX, XW, REP>(sh, a, lds); break;
    case 1: mlp_rows_wave<NW, 1, D0, CM, EX, XW, REP>(sh, a, lds); break;
    case 2: mlp_rows_wave<NW, 2, D0, CM, EX, XW, REP>(sh, a, lds); break;
    case 3: mlp_rows_wave<NW, 3, D0, CM, EX, XW, REP>(sh, a, lds); break;
    default:
      if constexpr (NW == 8) {
        switch (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) {
          case 4: mlp_rows_wave<NW, 4, D0, CM, EX, XW, REP>(sh, a, lds); break;
          case 5: mlp_rows_wave<NW, 5, D0, CM, EX, XW, REP>(sh, a, lds); break;
          case 6: mlp_rows_wave<NW, 6, D0, CM, EX, XW, REP>(sh, a, lds); break;
          default: mlp_rows_wave<NW, 7, D0, CM, EX, XW, REP>(sh, a, lds); break;
        }
      }
  }
}

}  // namespace dct

namespace {
using dct::MlpArgs;
using dct::WaveShape;

template <int L, int BMAX, int D0, int CM, bool EX, int XW>
hipError_t launch_wave(const WaveShape& sh, const MlpArgs& a, hipStream_t st) {
  hipLaunchKernelGGL((dct::mlp_wave_kernel<L, BMAX, D0, CM, EX, XW>), dim3(1), dim3(64), 0, st, sh, a);
  return hipGetLastError();
}

template <int L, int BMAX, int XW>
hipError_t launch_wave_d0(const WaveShape& sh, const MlpArgs& a, hipStream_t st) {
  if (sh.C > 4) return hipErrorInvalidValue;
  if constexpr (L == 2)
    if (sh.d0 == 5 && sh.C == 2) return launch_wave<L, BMAX, 5, 2, true, XW>(sh, a, st);  // WeatherClassifier
  if (sh.d0 <= 8) return launch_wave<L, BMAX, 8, 4, false, XW>(sh, a, st);
  if (sh.d0 <= 16) return launch_wave<L, BMAX, 16, 4, false, XW>(sh, a, st);
  return hipErrorInvalidValue;
}

template <int D0, int CM, bool EX, int XW>
hipError_t launch_rows(const WaveShape& sh, const MlpArgs& a, hipStream_t st) {
  // B <= 4 runs 4 waves: 8 (the extra ones owning only Adam slots, two waves per SIMD) measured
  // 0.727-0.730 vs 0.710 us/step on the weather step (MI355X, round 2)
  if (a.B <= 4)
    hipLaunchKernelGGL((dct::mlp_rows_kernel<4, D0, CM, EX, XW>), dim3(1), dim3(64 * 4), 0, st, sh, a);
  else
    hipLaunchKernelGGL((dct::mlp_rows_kernel<8, D0, CM, EX, XW>), dim3(1), dim3(64 * 8), 0, st, sh, a);
  return hipGetLastError();
}

template <int XW>
hipError_t launch_rows_d0(const WaveShape& sh, const MlpArgs& a, hipStream_t st) {
  if (sh.C > 4) return hipErrorInvalidValue;
  if (sh.d0 == 5 && sh.C == 2) return launch_rows<5, 2, true, XW>(sh, a, st);  // WeatherClassifier
  if (sh.d0 <= 8) return launch_rows<8, 4, false, XW>(sh, a, st);
  if (sh.d0 <= 16) return launch_rows<16, 4, false, XW>(sh, a, st);
  return hipErrorInvalidValue;
}

// the row-parallel kernel takes plain train-mode launches of 2-layer nets
bool rows_eligible(int L, const MlpArgs& a) {
#ifdef WAVE_PROF_BUILD
  const bool prof_ok = true;  // profiling build: the rows kernel stamps its phases into a.prof
#else
  const bool prof_ok = !a.prof;
#endif
  return L == 2 && a.mode == 0 && !a.cursor && !a.pending && !a.stage && prof_ok && a.B >= 1 &&
         a.B <= 8 && a.m && a.v;
}

template <int BMAX>
hipError_t launch_wave_xg(const WaveShape& sh, const MlpArgs& a, hipStream_t st) {
  if (a.xg_world <= 2) return launch_wave_d0<2, BMAX, 2>(sh, a, st);
  if (a.xg_world <= 4) return launch_wave_d0<2, BMAX, 4>(sh, a, st);
  return launch_wave_d0<2, BMAX, 8>(sh, a, st);
}
}  // namespace

namespace dct {
// one definition each, in the mlp_wave_*.hip translation units
hipError_t wave_rows_launch_x0(const WaveShape& sh, const MlpArgs& a, hipStream_t st);
hipError_t wave_rows_launch_x2(const WaveShape& sh, const MlpArgs& a, hipStream_t st);
hipError_t wave_rows_launch_x4(const WaveShape& sh, const MlpArgs& a, hipStream_t st);
hipError_t wave_rows_launch_x8(const WaveShape& sh, const MlpArgs& a, hipStream_t st);
hipError_t wave_single_launch(const WaveShape& sh, const MlpArgs& a, hipStream_t st);
hipError_t wave_single_launch_xg(const WaveShape& sh, const MlpArgs& a, hipStream_t st);
}  // namespace dct

