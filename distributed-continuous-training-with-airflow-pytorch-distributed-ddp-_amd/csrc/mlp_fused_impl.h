// Fused tabular-MLP training kernels for MI355X (gfx950, CDNA4) - device templates.
//
// What they replace (reference jobs/train_lightning_ddp.py): the per-step hot loop of
// Lightning's fit() for WeatherClassifier (:57-62 net, :66-71 training_step, :88 Adam,
// :122 batch 4): default_collate of 4 samples, Linear/ReLU/Dropout/Linear forward,
// F.cross_entropy, autograd backward, Adam.step() - about a dozen ATen launches plus
// Python per step.  At batch 4 that step is pure latency, so here the WHOLE step lives in
// one workgroup, and - on a single rank - every step of an epoch lives in ONE launch:
//
//   [fwd layer l: relu + dropout]* (+ CE/MSE and dlogits fused into the last layer)
//   -> [dX layer l]* -> dW + Adam (moments in VGPRs, fp32 master weights in LDS),
//   while the NEXT batch's rows are already in flight from HBM into registers.
//
// Latency design (measured with the s_memtime phase stamps, tools/prof_fused.py):
//  * LDS-only barriers (s_waitcnt lgkmcnt(0); s_barrier): __syncthreads() would also wait
//    vmcnt(0), i.e. for every outstanding global load/store (the prefetch, the loss store).
//  * depth-2 register prefetch of the batch: idx for step s+2 and the X/label values of step
//    s+1 are issued at the top of step s and written into the other half of a double-buffered
//    LDS input tile at the end of it - the gather never stalls the step.
//  * compile-time layer count: every per-layer shape field has a constant index, so the
//    shape lives in SGPRs instead of being re-fetched with scalar loads in each phase.
//  * k-/o-split partial sums reduced with DPP (quad_perm, row_ror), not ds_bpermute.
//  * per-thread weight-block descriptors computed once per launch (no divisions per step);
//    1x4 blocks for small models (more threads share Adam), 4x4 for larger ones (LDS reuse);
//    Adam uses v_sqrt_f32 / v_rcp_f32.
//  * Matmuls have M = batch = 4: per CDNA guidance (GEMV / M <= 16 rows) they run on the VALU
//    from LDS with 4-output x 4-k register blocking; big-batch configs use the MFMA GEMMs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dct_common.h"
#include "mlp_fused.h"

namespace dct {

__device__ __forceinline__ uint32_t mix_hash(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t h = a * 0x9E3779B1u;
  h ^= (b + 0x7F4A7C15u) * 0x85EBCA77u;
  h ^= (c + 0x165667B1u) * 0xC2B2AE3Du;
  h ^= h >> 16;
  h *= 0x7feb352du;
  h ^= h >> 15;
  h *= 0x846ca68bu;
  h ^= h >> 16;
  return h;
}

__device__ __forceinline__ float u01(uint32_t h) { return (float)(h >> 8) * (1.0f / 16777216.0f); }

__device__ __forceinline__ float dot4(const float4& a, const float4& b) {
  return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w;
}

// Workgroup barrier for LDS traffic only (global loads/stores stay in flight across it).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), CTRL, 0xF, 0xF, false));
}

// all-reduce sum inside aligned groups of 2^ksl lanes, ksl in {0, 1, 2, 4}
template <int N>
__device__ __forceinline__ void group_sum(float (&v)[N], int ksl) {
  if (ksl >= 1) {
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] += dppf<0xB1>(v[i]);  // quad_perm [1,0,3,2]: lane ^ 1
  }
  if (ksl >= 2) {
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] += dppf<0x4E>(v[i]);  // quad_perm [2,3,0,1]: lane ^ 2
  }
  if (ksl >= 4) {
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] += dppf<0x124>(v[i]);  // row_ror:4 (next quad)
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] += dppf<0x128>(v[i]);  // row_ror:8 (other half-row)
  }
}

struct LossAcc {
  float loss;
  float correct;
};

// CE / MSE of one row of logits z[0..C) (C <= 4) with label y; writes dz[c] * inv
__device__ __forceinline__ LossAcc row_loss4(const float (&z)[4], int C, int y, int loss_kind, float inv, float* dz) {
  LossAcc r{0.f, 0.f};
  float mx = -3.402823466e+38f;
  int am = 0;
#pragma unroll
  for (int c = 0; c < 4; ++c)
    if (c < C && z[c] > mx) { mx = z[c]; am = c; }
  r.correct = (am == y) ? 1.f : 0.f;
  if (loss_kind == 0) {
    float e[4], s = 0.f, zy = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      e[c] = (c < C) ? __expf(z[c] - mx) : 0.f;
      s += e[c];
      if (c == y) zy = z[c];
    }
    r.loss = mx + __logf(s) - zy;
    const float rs = __builtin_amdgcn_rcpf(s);
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (c < C) dz[c] = (e[c] * rs - (c == y ? 1.f : 0.f)) * inv;
  } else {
    const float sc = 2.f / (float)C;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (c < C) {
        const float d = z[c] - (c == y ? 1.f : 0.f);
        r.loss += d * d;
        dz[c] = d * sc * inv;
      }
    }
    r.loss /= (float)C;
  }
  return r;
}

// ----------------------------------------------------------------------------------------
// forward of layer LI: Out[b][o] = act(sum_k W[o][k] A[b][k] + bias[o]).
// items = (rows4/4 output groups) << ksl k-splits (KS adjacent lanes per group).
// FUSE (last layer, classes <= 4): thread 0 also computes the batch loss and dZ_{L-1}.
template <int LI, int NT, int BMAX, bool FUSE>
__device__ __forceinline__ LossAcc fwd_layer(const MlpShape& sh, float* lds, const float* A, int B, int bs,
                                             bool last, bool train, float p_drop, uint32_t seed, uint32_t gstep,
                                             const int* lab, int loss_kind) {
  const int tid = threadIdx.x;
  const int K4 = sh.cols4[LI] >> 2;
  const int N = sh.dims[LI + 1];
  const int ksl = sh.f_ksl[LI];
  const int kc = sh.f_kc[LI];
  const int items = sh.f_items[LI];
  const float* W = lds + sh.w_lds[LI];
  const int ldw = sh.ldw[LI];
  const int lda = sh.lda[LI];
  float* Out = lds + sh.a_lds[LI + 1];
  const int ldo = sh.lda[LI + 1];
  const float* bias = lds + sh.b_lds[LI];
  const float scale = (train && p_drop > 0.f) ? 1.0f / (1.0f - p_drop) : 1.0f;
  LossAcc lo{0.f, 0.f};
  for (int it0 = 0; it0 < items; it0 += NT) {
    const int item = it0 + tid;
    const bool valid = item < items;
    const int g = item >> ksl;
    const int ks = item & ((1 << ksl) - 1);
    float acc[4 * BMAX];
#pragma unroll
    for (int e = 0; e < 4 * BMAX; ++e) acc[e] = 0.f;
    if (valid) {
      const int k4b = ks * kc;
      const int k4e = min(K4, k4b + kc);
      const float* wrow = W + g * 4 * ldw;
      for (int k4 = k4b; k4 < k4e; ++k4) {
        float4 w[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) w[r] = *reinterpret_cast<const float4*>(wrow + r * ldw + k4 * 4);
#pragma unroll
        for (int b = 0; b < BMAX; ++b) {  // rows >= B are zero-filled: no predicate needed
          const float4 a = *reinterpret_cast<const float4*>(A + b * lda + k4 * 4);
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[r * BMAX + b] += dot4(w[r], a);
        }
      }
    }
    group_sum(acc, ksl);
    if (FUSE) {
      if (tid == 0) {  // last layer with <= 4 classes: the single output group is item 0
        float* dZ = lds + sh.dz_lds[LI];
        const float inv = 1.0f / (float)(bs > 0 ? bs : 1);
#pragma unroll
        for (int b = 0; b < BMAX; ++b) {
          float z[4], dz[4];
#pragma unroll
          for (int c = 0; c < 4; ++c) z[c] = (c < N) ? acc[c * BMAX + b] + bias[c] : 0.f;
          const bool live = b < bs;
          const LossAcc r = row_loss4(z, N, lab[b], loss_kind, live ? inv : 0.f, dz);
#pragma unroll
          for (int c = 0; c < 4; ++c)
            if (c < N) dZ[b * 4 + c] = dz[c];
          if (live) { lo.loss += r.loss; lo.correct += r.correct; }
        }
      }
    } else if (valid && ks == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int o = g * 4 + r;
        if (o < N) {
          const float bv = bias[o];
#pragma unroll
          for (int b = 0; b < BMAX; ++b) {
            float z = acc[r * BMAX + b] + bv;
            if (!last) {
              z = fmaxf(z, 0.f);
              if (train && p_drop > 0.f) {
                const uint32_t h = mix_hash(seed, gstep, (uint32_t)((LI * 64 + b) * 65536 + o));
                z = (u01(h) < p_drop) ? 0.f : z * scale;
              }
            }
            Out[b * ldo + o] = z;
          }
        }
      }
    }
  }
  return lo;
}

// dZ_{LI-1}[b][i] = mask(A_LI[b][i]) * sum_o dZ_LI[b][o] W_LI[o][i]   (i < in)
template <int LI, int NT, int BMAX>
__device__ __forceinline__ void dx_layer(const MlpShape& sh, float* lds, int B, float dscale) {
  const int tid = threadIdx.x;
  const int in = sh.dims[LI];
  const int O4 = sh.rows4[LI] >> 2;
  const int osl = sh.d_osl[LI];
  const int oc = sh.d_oc[LI];
  const int items = sh.d_items[LI];
  const float* W = lds + sh.w_lds[LI];
  const int ldw = sh.ldw[LI];
  const float* dZ = lds + sh.dz_lds[LI];
  const int ldz = sh.rows4[LI];
  const float* A = lds + sh.a_lds[LI];
  const int lda = sh.lda[LI];
  float* dZp = lds + sh.dz_lds[LI - 1];
  const int ldzp = sh.rows4[LI - 1];
  for (int it0 = 0; it0 < items; it0 += NT) {
    const int item = it0 + tid;
    const bool valid = item < items;
    const int cg = item >> osl;
    const int os = item & ((1 << osl) - 1);
    float acc[BMAX * 4];
#pragma unroll
    for (int e = 0; e < BMAX * 4; ++e) acc[e] = 0.f;
    if (valid) {
      const int o4b = os * oc;
      const int o4e = min(O4, o4b + oc);
      for (int o4 = o4b; o4 < o4e; ++o4) {
        float4 w[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) w[r] = *reinterpret_cast<const float4*>(W + (o4 * 4 + r) * ldw + cg * 4);
#pragma unroll
        for (int b = 0; b < BMAX; ++b) {
          const float4 d = *reinterpret_cast<const float4*>(dZ + b * ldz + o4 * 4);
          acc[b * 4 + 0] += d.x * w[0].x + d.y * w[1].x + d.z * w[2].x + d.w * w[3].x;
          acc[b * 4 + 1] += d.x * w[0].y + d.y * w[1].y + d.z * w[2].y + d.w * w[3].y;
          acc[b * 4 + 2] += d.x * w[0].z + d.y * w[1].z + d.z * w[2].z + d.w * w[3].z;
          acc[b * 4 + 3] += d.x * w[0].w + d.y * w[1].w + d.z * w[2].w + d.w * w[3].w;
        }
      }
    }
    group_sum(acc, osl);
    if (valid && os == 0) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int i = cg * 4 + c;
        if (i < in) {
#pragma unroll
          for (int b = 0; b < BMAX; ++b) {
            const float av = A[b * lda + i];
            dZp[b * ldzp + i] = (av > 0.f) ? acc[b * 4 + c] * dscale : 0.f;
          }
        }
      }
    }
  }
}

// generic loss over logits A_L [B][C] (C > 4 or eval); writes dZ_{L-1}; returns sums on thread 0
template <int BMAX>
__device__ LossAcc loss_phase(const MlpShape& sh, float* lds, int B, int bs, const int* lab, int loss_kind) {
  const int tid = threadIdx.x;
  const int L = sh.L;
  const int C = sh.dims[L];
  const float* Z = lds + sh.a_lds[L];
  const int ldz_in = sh.lda[L];
  float* dZ = lds + sh.dz_lds[L - 1];
  const int ldz = sh.rows4[L - 1];
  float* red = lds + sh.red_lds;
  if (tid < B) {
    const int b = tid;
    const bool live = b < bs;
    const int y = lab[b];
    float lb = 0.f, corr = 0.f;
    float mx = -3.402823466e+38f;
    int am = 0;
    for (int c = 0; c < C; ++c) {
      const float z = Z[b * ldz_in + c];
      if (z > mx) { mx = z; am = c; }
    }
    corr = (am == y) ? 1.f : 0.f;
    const float inv = live ? 1.0f / (float)(bs > 0 ? bs : 1) : 0.f;
    if (loss_kind == 0) {
      float s = 0.f;
      for (int c = 0; c < C; ++c) s += __expf(Z[b * ldz_in + c] - mx);
      lb = mx + __logf(s) - Z[b * ldz_in + y];
      const float rs = 1.0f / s;
      for (int c = 0; c < C; ++c)
        dZ[b * ldz + c] = (__expf(Z[b * ldz_in + c] - mx) * rs - (c == y ? 1.f : 0.f)) * inv;
    } else {
      const float sc = 2.f / (float)C;
      for (int c = 0; c < C; ++c) {
        const float d = Z[b * ldz_in + c] - (c == y ? 1.f : 0.f);
        lb += d * d;
        dZ[b * ldz + c] = d * sc * inv;
      }
      lb /= (float)C;
    }
    red[b] = live ? lb : 0.f;
    red[BMAX + b] = live ? corr : 0.f;
  }
  lds_barrier();
  LossAcc r{0.f, 0.f};
  if (tid == 0) {
    for (int b = 0; b < bs; ++b) { r.loss += red[b]; r.correct += red[BMAX + b]; }
  }
  return r;
}

// direct (non-prefetched) gather of batch sb into the LDS input tile
template <int BMAX>
__device__ void gather_direct(const MlpShape& sh, float* A0, int* lab, const MlpArgs& a, int sb, int bs) {
  const int tid = threadIdx.x;
  const int d0 = sh.dims[0];
  const int lda = sh.lda[0];
  for (int e = tid; e < BMAX * lda; e += blockDim.x) {
    const int b = e / lda;
    const int k = e - b * lda;
    float x = 0.f;
    if (b < bs && k < d0) x = a.X[(size_t)a.idx[sb * a.B + b] * a.ldx + k];
    A0[e] = x;
  }
  if (tid < BMAX) lab[tid] = (tid < bs) ? a.Y[a.idx[sb * a.B + tid]] : 0;
}

// load flat torch-order params into the padded LDS layout (+ zero everything else)
__device__ void load_params_lds(const MlpShape& sh, float* lds, const float* p) {
  for (int e = threadIdx.x; e < sh.lds_floats; e += blockDim.x) lds[e] = 0.f;
  __syncthreads();
  for (int l = 0; l < sh.L; ++l) {
    const int in = sh.dims[l], out = sh.dims[l + 1];
    float* W = lds + sh.w_lds[l];
    const int ldw = sh.ldw[l];
    for (int e = threadIdx.x; e < in * out; e += blockDim.x) {
      const int o = e / in, i = e - o * in;
      W[o * ldw + i] = p[sh.woff[l] + e];
    }
    for (int e = threadIdx.x; e < out; e += blockDim.x) lds[sh.b_lds[l] + e] = p[sh.boff[l] + e];
  }
}

// weight block owned by a thread, resolved once per launch
struct BlkDesc {
  int layer;  // -1: none
  int w;      // LDS offset of W[o0][i0]
  int dz;     // LDS offset of dZ_l[0][o0]
  int a;      // offset of A_l[0][i0] (layer 0: relative to the input tile)
  int lda, ldz, ldw;
  int rows;   // valid rows in the block (<= br)
  int cols;   // valid cols (<= 4)
  int f;      // flat offset of W[o0][i0]
  int in;
};

__device__ __forceinline__ BlkDesc make_blk(const MlpShape& sh, int g) {
  BlkDesc d;
  d.layer = -1;
  if (g >= sh.nblk) return d;
  int l = 0;
#pragma unroll
  for (int j = 1; j < MLP_MAXL; ++j)
    if (j < sh.L && g >= sh.blk_start[j]) l = j;
  const int lb = g - sh.blk_start[l];
  const int cgn = sh.blk_cols[l];
  const int o0 = (lb / cgn) * sh.br, i0 = (lb % cgn) * 4;
  const int in = sh.dims[l], out = sh.dims[l + 1];
  d.layer = l;
  d.ldw = sh.ldw[l];
  d.w = sh.w_lds[l] + o0 * d.ldw + i0;
  d.ldz = sh.rows4[l];
  d.dz = sh.dz_lds[l] + o0;
  d.lda = sh.lda[l];
  d.a = (l == 0 ? 0 : sh.a_lds[l]) + i0;
  d.rows = min(sh.br, out - o0);
  d.cols = min(4, in - i0);
  d.f = sh.woff[l] + o0 * in + i0;
  d.in = in;
  return d;
}

struct BiasDesc {
  int layer;
  int dz, ldz, b, f;
};

__device__ __forceinline__ BiasDesc make_bias(const MlpShape& sh, int q) {
  BiasDesc d;
  d.layer = -1;
  if (q >= sh.nbias) return d;
  int l = 0;
#pragma unroll
  for (int j = 1; j < MLP_MAXL; ++j)
    if (j < sh.L && q >= sh.bias_start[j]) l = j;
  const int o = q - sh.bias_start[l];
  d.layer = l;
  d.dz = sh.dz_lds[l] + o;
  d.ldz = sh.rows4[l];
  d.b = sh.b_lds[l] + o;
  d.f = sh.boff[l] + o;
  return d;
}

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, float b1, float b2, float wd,
                                          float step_size, float rbc2, float eps) {
  g += wd * p;
  m = b1 * m + (1.f - b1) * g;
  v = b2 * v + (1.f - b2) * g * g;
  const float denom = __builtin_amdgcn_sqrtf(v) * rbc2 + eps;
  p -= step_size * m * __builtin_amdgcn_rcpf(denom);
}

constexpr int MLP_MAXBIAS = 2;

template <int L, int NT, int MAXQ, int BMAX, int BR>
__global__ __launch_bounds__(NT) void mlp_train_kernel(MlpShape sh, MlpArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x;
  const bool adam = (a.mode == 0);

  load_params_lds(sh, lds, a.p);
  int cur0 = 0;
  if (a.cursor) {
    cur0 = __hip_atomic_load(a.cursor, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tid == 0 && cur0 > 0 && a.loss_out) a.loss_out[cur0 - 1] = a.grad_out[sh.P];
  }
  int t0 = a.t0;
  uint32_t step_base = a.step_base;
  if (a.step_counter) {
    t0 = __hip_atomic_load(a.step_counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    step_base = (uint32_t)t0;
  }

  // ---- owned weight blocks / biases (+ Adam moments in registers for the whole launch)
  BlkDesc bd[MAXQ];
  float mw[MAXQ][4 * BR], vw[MAXQ][4 * BR];
#pragma unroll
  for (int j = 0; j < MAXQ; ++j) {
    bd[j] = make_blk(sh, tid + j * NT);
#pragma unroll
    for (int e = 0; e < 4 * BR; ++e) { mw[j][e] = 0.f; vw[j][e] = 0.f; }
    if (adam && bd[j].layer >= 0) {
#pragma unroll
      for (int r = 0; r < BR; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (r < bd[j].rows && c < bd[j].cols) {
            const int f = bd[j].f + r * bd[j].in + c;
            mw[j][r * 4 + c] = a.m[f];
            vw[j][r * 4 + c] = a.v[f];
          }
    }
  }
  BiasDesc bb[MLP_MAXBIAS];
  float mb[MLP_MAXBIAS], vb[MLP_MAXBIAS];
#pragma unroll
  for (int j = 0; j < MLP_MAXBIAS; ++j) {
    bb[j] = make_bias(sh, tid + j * NT);
    mb[j] = 0.f;
    vb[j] = 0.f;
    if (adam && bb[j].layer >= 0) { mb[j] = a.m[bb[j].f]; vb[j] = a.v[bb[j].f]; }
  }

  // ---- batch prefetch roles: thread -> (row b, feature k) or (row b, label)
  const int d0 = sh.dims[0];
  const int B = a.B;
  const int nel = B * d0;
  const bool pf = (nel + B <= NT);
  int role = 0, pb = 0, pk = 0;
  if (pf) {
    if (tid < nel) { role = 1; pb = tid / d0; pk = tid - pb * d0; }
    else if (tid < nel + B) { role = 2; pb = tid - nel; }
  }
  const int lda0 = sh.lda[0];
  int buf = 0;
  {
    const int bs0 = min(B, a.n_items - cur0 * B);
    gather_direct<BMAX>(sh, lds + sh.a0_lds[0], reinterpret_cast<int*>(lds + sh.lab_lds[0]), a, cur0, bs0);
  }
  int ridx_next = 0;  // idx of (batch cur0+1, row pb); 0 (a valid row) when out of range
  if (role && (cur0 + 1) * B + pb < a.n_items) ridx_next = a.idx[(cur0 + 1) * B + pb];
  __syncthreads();

  const float dscale = (a.dropout > 0.f) ? 1.0f / (1.0f - a.dropout) : 1.0f;
  const bool fuse = sh.fuse_loss != 0;
  const bool prof = (a.prof != nullptr) && tid == 0;
  unsigned long long tprev = 0;
  if (prof) {
    a.prof[30] = __builtin_amdgcn_s_memrealtime();
    tprev = __builtin_amdgcn_s_memtime();
  }
#define FMLP_MARK(k)                                             \
  if (prof) {                                                   \
    const unsigned long long tn = __builtin_amdgcn_s_memtime(); \
    atomicAdd(&a.prof[(k)], tn - tprev);                        \
    tprev = tn;                                                 \
  }

  for (int s = 0; s < a.steps; ++s) {
    const int sb = s + cur0;
    const int bs = min(B, a.n_items - sb * B);
    const uint32_t gstep = step_base + (uint32_t)s;
    float* A0 = lds + sh.a0_lds[buf];
    const int* lab = reinterpret_cast<const int*>(lds + sh.lab_lds[buf]);
    // issue next batch's values (idx known) and the idx of the batch after it
    const bool have_next = (s + 1 < a.steps);
    const int bs_next = have_next ? min(B, a.n_items - (sb + 1) * B) : 0;
    // branch-free: every thread issues exactly two dword loads (clamped addresses), so no
    // divergent path ever overwrites a register with a load in flight (that forced vmcnt(0))
    const uint32_t* src = (role == 1) ? reinterpret_cast<const uint32_t*>(a.X) + (size_t)ridx_next * a.ldx + pk
                                      : reinterpret_cast<const uint32_t*>(a.Y) + ridx_next;
    const uint32_t raw_next = *src;
    const int nx2 = min((sb + 2) * B + pb, a.n_items - 1);
    const int ridx_next2 = a.idx[nx2 < 0 ? 0 : nx2];
    if (!pf && s > 0) {
      gather_direct<BMAX>(sh, A0, reinterpret_cast<int*>(lds + sh.lab_lds[buf]), a, sb, bs);
      lds_barrier();
    }

    // ---- forward (+ fused loss)
    LossAcc lo{0.f, 0.f};
#pragma unroll
    for (int li = 0; li < L; ++li) {
      const float* Ain = (li == 0) ? A0 : lds + sh.a_lds[li];
      const bool last = (li == L - 1);
      if (li == 0) {
        if (L == 1 && fuse) lo = fwd_layer<0, NT, BMAX, true>(sh, lds, Ain, B, bs, last, true, a.dropout, a.seed, gstep, lab, a.loss_kind);
        else fwd_layer<0, NT, BMAX, false>(sh, lds, Ain, B, bs, last, true, a.dropout, a.seed, gstep, lab, a.loss_kind);
      } else if (li == 1) {
        if (L == 2 && fuse) lo = fwd_layer<1 % MLP_MAXL, NT, BMAX, true>(sh, lds, Ain, B, bs, last, true, a.dropout, a.seed, gstep, lab, a.loss_kind);
        else fwd_layer<1 % MLP_MAXL, NT, BMAX, false>(sh, lds, Ain, B, bs, last, true, a.dropout, a.seed, gstep, lab, a.loss_kind);
      } else if (li == 2) {
        if (L == 3 && fuse) lo = fwd_layer<2 % MLP_MAXL, NT, BMAX, true>(sh, lds, Ain, B, bs, last, true, a.dropout, a.seed, gstep, lab, a.loss_kind);
        else fwd_layer<2 % MLP_MAXL, NT, BMAX, false>(sh, lds, Ain, B, bs, last, true, a.dropout, a.seed, gstep, lab, a.loss_kind);
      } else {
        if (L == 4 && fuse) lo = fwd_layer<3, NT, BMAX, true>(sh, lds, Ain, B, bs, last, true, a.dropout, a.seed, gstep, lab, a.loss_kind);
        else fwd_layer<3, NT, BMAX, false>(sh, lds, Ain, B, bs, last, true, a.dropout, a.seed, gstep, lab, a.loss_kind);
      }
      lds_barrier();
      FMLP_MARK(1 + li);
    }
    if (!fuse) {
      lo = loss_phase<BMAX>(sh, lds, B, bs, lab, a.loss_kind);
      lds_barrier();
    }
    if (tid == 0) {
      const float bl = bs > 0 ? lo.loss / (float)bs : 0.f;
      if (a.loss_out && !a.cursor) a.loss_out[s] = bl;
      if (!adam) a.grad_out[sh.P] = bl;
    }
    FMLP_MARK(5);

    // ---- backward dX
#pragma unroll
    for (int li = L - 1; li >= 1; --li) {
      if (li == 3) dx_layer<3, NT, BMAX>(sh, lds, B, dscale);
      else if (li == 2) dx_layer<2, NT, BMAX>(sh, lds, B, dscale);
      else dx_layer<1, NT, BMAX>(sh, lds, B, dscale);
      lds_barrier();
      FMLP_MARK(6 + li);
    }

    // ---- next batch into the other half of the input tile (read after the end barrier)
    if (role) {
      const uint32_t v = (have_next && pb < bs_next) ? raw_next : 0u;
      uint32_t* dst = (role == 1) ? reinterpret_cast<uint32_t*>(lds + sh.a0_lds[buf ^ 1]) + pb * lda0 + pk
                                  : reinterpret_cast<uint32_t*>(lds + sh.lab_lds[buf ^ 1]) + pb;
      *dst = v;
    }
    ridx_next = role ? ridx_next2 : 0;

    // ---- dW (+ Adam) on owned blocks, biases
    const int t = t0 + s + 1;
    const float bc1 = 1.f - pow_t(log2f(a.b1), (float)t);
    const float bc2 = 1.f - pow_t(log2f(a.b2), (float)t);
    const float step_size = a.lr / bc1;
    const float rbc2 = __builtin_amdgcn_rsqf(bc2);
#pragma unroll
    for (int j = 0; j < MAXQ; ++j) {
      const BlkDesc& d = bd[j];
      if (d.layer >= 0) {
        const float* Ab = (d.layer == 0 ? A0 : lds) + d.a;
        float gr[16];
#pragma unroll
        for (int e = 0; e < 16; ++e) gr[e] = 0.f;
        if (BR == 4) {
#pragma unroll
          for (int b = 0; b < BMAX; ++b) {
            const float4 dz = *reinterpret_cast<const float4*>(lds + d.dz + b * d.ldz);
            const float4 x = *reinterpret_cast<const float4*>(Ab + b * d.lda);
            const float dd[4] = {dz.x, dz.y, dz.z, dz.w};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              gr[r * 4 + 0] += dd[r] * x.x;
              gr[r * 4 + 1] += dd[r] * x.y;
              gr[r * 4 + 2] += dd[r] * x.z;
              gr[r * 4 + 3] += dd[r] * x.w;
            }
          }
        } else {
#pragma unroll
          for (int b = 0; b < BMAX; ++b) {
            const float dz = lds[d.dz + b * d.ldz];
            const float4 x = *reinterpret_cast<const float4*>(Ab + b * d.lda);
            gr[0] += dz * x.x;
            gr[1] += dz * x.y;
            gr[2] += dz * x.z;
            gr[3] += dz * x.w;
          }
        }
        if (adam) {
#pragma unroll
          for (int r = 0; r < BR; ++r) {
            if (r < d.rows) {
              float* wp = lds + d.w + r * d.ldw;
              float4 w4 = *reinterpret_cast<float4*>(wp);
              float wv[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
              for (int c = 0; c < 4; ++c)
                if (c < d.cols)
                  adam_elem(wv[c], gr[r * 4 + c], mw[j][r * 4 + c], vw[j][r * 4 + c], a.b1, a.b2, a.wd, step_size,
                            rbc2, a.eps);
              *reinterpret_cast<float4*>(wp) = make_float4(wv[0], wv[1], wv[2], wv[3]);
            }
          }
        } else {
#pragma unroll
          for (int r = 0; r < BR; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c)
              if (r < d.rows && c < d.cols) a.grad_out[d.f + r * d.in + c] = gr[r * 4 + c];
        }
      }
    }
#pragma unroll
    for (int j = 0; j < MLP_MAXBIAS; ++j) {
      const BiasDesc& d = bb[j];
      if (d.layer >= 0) {
        float gg = 0.f;
#pragma unroll
        for (int b = 0; b < BMAX; ++b) gg += lds[d.dz + b * d.ldz];
        if (adam) adam_elem(lds[d.b], gg, mb[j], vb[j], a.b1, a.b2, a.wd, step_size, rbc2, a.eps);
        else a.grad_out[d.f] = gg;
      }
    }
    lds_barrier();
    FMLP_MARK(11);
    buf ^= 1;
  }
#undef FMLP_MARK
  if (prof) a.prof[31] = __builtin_amdgcn_s_memrealtime();
  if (a.cursor && tid == 0) __hip_atomic_store(a.cursor, cur0 + a.steps, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (a.step_counter && tid == 0)
    __hip_atomic_store(a.step_counter, t0 + a.steps, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (!adam) return;

  // ---- write back params + moments (flat torch order)
  __syncthreads();
  for (int l = 0; l < L; ++l) {
    const int in = sh.dims[l], out = sh.dims[l + 1];
    const float* W = lds + sh.w_lds[l];
    const int ldw = sh.ldw[l];
    for (int e = tid; e < in * out; e += NT) {
      const int o = e / in, i = e - o * in;
      a.p[sh.woff[l] + e] = W[o * ldw + i];
    }
    for (int e = tid; e < out; e += NT) a.p[sh.boff[l] + e] = lds[sh.b_lds[l] + e];
  }
#pragma unroll
  for (int j = 0; j < MAXQ; ++j) {
    if (bd[j].layer >= 0) {
#pragma unroll
      for (int r = 0; r < BR; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (r < bd[j].rows && c < bd[j].cols) {
            const int f = bd[j].f + r * bd[j].in + c;
            a.m[f] = mw[j][r * 4 + c];
            a.v[f] = vw[j][r * 4 + c];
          }
    }
  }
#pragma unroll
  for (int j = 0; j < MLP_MAXBIAS; ++j) {
    if (bb[j].layer >= 0) {
      a.m[bb[j].f] = mb[j];
      a.v[bb[j].f] = vb[j];
    }
  }
}

// Validation / inference: every workgroup stages the weights in LDS once, then walks
// BMAX-row chunks of the index list; per-row CE/MSE + argmax-correct are reduced per
// workgroup and added to eval_acc[0..1] (one atomic pair per workgroup).
template <int L, int NT, int BMAX>
__global__ __launch_bounds__(NT) void mlp_eval_kernel(MlpShape sh, MlpArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x;
  load_params_lds(sh, lds, a.p);
  __syncthreads();
  const int nchunks = (a.n_items + BMAX - 1) / BMAX;
  float wg_loss = 0.f, wg_corr = 0.f;
  const int C = sh.dims[L];
  MlpArgs ca = a;
  ca.B = BMAX;
  float* A0 = lds + sh.a0_lds[0];
  int* lab = reinterpret_cast<int*>(lds + sh.lab_lds[0]);
  for (int ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
    const int bs = min(BMAX, a.n_items - ch * BMAX);
    gather_direct<BMAX>(sh, A0, lab, ca, ch, bs);
    __syncthreads();
#pragma unroll
    for (int li = 0; li < L; ++li) {
      const float* Ain = (li == 0) ? A0 : lds + sh.a_lds[li];
      const bool last = (li == L - 1);
      if (li == 0) fwd_layer<0, NT, BMAX, false>(sh, lds, Ain, BMAX, bs, last, false, 0.f, 0u, 0u, lab, 0);
      else if (li == 1) fwd_layer<1 % MLP_MAXL, NT, BMAX, false>(sh, lds, Ain, BMAX, bs, last, false, 0.f, 0u, 0u, lab, 0);
      else if (li == 2) fwd_layer<2 % MLP_MAXL, NT, BMAX, false>(sh, lds, Ain, BMAX, bs, last, false, 0.f, 0u, 0u, lab, 0);
      else fwd_layer<3, NT, BMAX, false>(sh, lds, Ain, BMAX, bs, last, false, 0.f, 0u, 0u, lab, 0);
      __syncthreads();
    }
    if (a.logits_out) {
      const float* Z = lds + sh.a_lds[L];
      for (int e = tid; e < bs * C; e += NT) {
        const int b = e / C, c = e - b * C;
        a.logits_out[(size_t)(ch * BMAX + b) * C + c] = Z[b * sh.lda[L] + c];
      }
    }
    const LossAcc r = loss_phase<BMAX>(sh, lds, BMAX, bs, lab, a.loss_kind);
    if (tid == 0) { wg_loss += r.loss; wg_corr += r.correct; }
    __syncthreads();
  }
  if (tid == 0 && a.eval_acc) {
    atomicAdd(&a.eval_acc[0], wg_loss);
    atomicAdd(&a.eval_acc[1], wg_corr);
  }
}

template <int L, int NT, int MAXQ, int BMAX, int BR>
hipError_t launch_train_inst(const MlpShape& sh, const MlpArgs& a, hipStream_t st) {
  const size_t bytes = (size_t)sh.lds_floats * sizeof(float);
  auto fn = mlp_train_kernel<L, NT, MAXQ, BMAX, BR>;
  hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(fn, dim3(1), dim3(NT), bytes, st, sh, a);
  return hipGetLastError();
}

template <int L, int BMAX>
hipError_t launch_train_bmax(const MlpShape& sh, const MlpArgs& a, hipStream_t st) {
  if (sh.br == 1) {
    if (sh.nt == 256 && sh.maxq == 1) return launch_train_inst<L, 256, 1, BMAX, 1>(sh, a, st);
    if (sh.nt == 256 && sh.maxq == 2) return launch_train_inst<L, 256, 2, BMAX, 1>(sh, a, st);
  } else {
    if (sh.nt == 256 && sh.maxq == 1) return launch_train_inst<L, 256, 1, BMAX, 4>(sh, a, st);
    if (sh.nt == 256 && sh.maxq == 2) return launch_train_inst<L, 256, 2, BMAX, 4>(sh, a, st);
    if (sh.nt == 256 && sh.maxq == 4) return launch_train_inst<L, 256, 4, BMAX, 4>(sh, a, st);
    if (sh.nt == 512 && sh.maxq == 3) return launch_train_inst<L, 512, 3, BMAX, 4>(sh, a, st);
    if (sh.nt == 512 && sh.maxq == 4) return launch_train_inst<L, 512, 4, BMAX, 4>(sh, a, st);
  }
  return hipErrorInvalidValue;
}

template <int L>
hipError_t launch_train_L(const MlpShape& sh, const MlpArgs& a, hipStream_t st) {
  if (sh.bmax == 4) return launch_train_bmax<L, 4>(sh, a, st);
  if (sh.bmax == 16) return launch_train_bmax<L, 16>(sh, a, st);
  return hipErrorInvalidValue;
}

template <int L>
hipError_t launch_eval_L(const MlpShape& sh, const MlpArgs& a, int grid, hipStream_t st) {
  if (sh.bmax != 16) return hipErrorInvalidValue;
  const size_t bytes = (size_t)sh.lds_floats * sizeof(float);
  auto fn = mlp_eval_kernel<L, 256, 16>;
  hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(fn, dim3(grid), dim3(256), bytes, st, sh, a);
  return hipGetLastError();
}

}  // namespace dct
