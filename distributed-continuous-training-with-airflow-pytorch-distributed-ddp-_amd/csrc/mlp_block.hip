// Register-resident multi-wave trainer for 3-layer MLPs D0 -> 128 -> 128 -> C (C <= 4,
// D0 <= 32, batch <= 4): BASELINE "Weather MLP (3-layer, 128-h)" (models/mlp.py preset
// weather-mlp-3x128).  Same contract as mlp_train_kernel (mlp_fused_impl.h): one
// workgroup, every step of an epoch in one launch, identical dropout hash / loss / Adam, so
// it is a drop-in replacement selected by dct_mlp_train.
//
// Why a second design: the generic LDS kernel keeps all weights in LDS and re-streams the
// 64 KB hidden-to-hidden matrix through ds_read for the forward, the dX and the Adam phase
// (~18 us per step, LDS- and DPP-latency bound).  Here the 128x128 matrix never leaves
// VGPRs (32 weights + Adam moments per lane):
//   * forward 128->128: wave w owns the k-slice [16w, 16w+16), lane l the outputs l, l+64;
//     the activations it needs are wave-uniform broadcast reads; the 8 k-slice partials meet
//     in LDS and are summed by the (row, unit) thread that also applies bias/ReLU/dropout;
//   * dX through the same registers: each lane forms its 64 (k, row) partial products and a
//     six-level butterfly reduce-scatter (v_permlane32_swap, v_permlane16_swap, DPP row_ror,
//     ds_swizzle, DPP quad_perm), two 32-value passes, leaves each (k, row) sum in a lane pair;
//   * dW + Adam in registers with the moments; the small layers (D0x128, 128xC) are owned
//     one element per thread; the Adam second moments of the big layer live in LDS.
// Seven LDS-only barriers per step; the next batch is gathered under the step (depth-2
// register prefetch, as in the LDS kernel).
#include "mlp_fused_impl.h"

namespace dct {

namespace blk {
constexpr int H = 128, NT = 512, KS = 16, DMAX = 32, B = 4;
// LDS layout (floats); activations and gradients are stored transposed [unit][row] so one
// float4 holds a unit's 4 batch rows
constexpr int XT = 0;                    // [2][DMAX][4] input tile (double-buffered)
constexpr int LAB = XT + 2 * DMAX * 4;   // [2][4] labels (int)
constexpr int H1T = LAB + 8;             // [H][4]
constexpr int H2T = H1T + H * 4;         // [H][4]
constexpr int DZ2T = H2T + H * 4;        // [H][4]
constexpr int DZ1T = DZ2T + H * 4;       // [H][4]
constexpr int PART = DZ1T + H * 4;       // [8 waves][4 rows][H] forward k-slice partials
constexpr int W2S = PART + 8 * 4 * H;    // [4][H] last-layer weights (read by every unit)
constexpr int B0S = W2S + 4 * H;         // [H]
constexpr int B1S = B0S + H;             // [H]
constexpr int B2S = B1S + H;             // [4]
constexpr int ZP = B2S + 4;              // [8 waves][4] logit partials
constexpr int DZ3 = ZP + 32;             // [4 rows][4] dlogits
// Adam second moments of the 128x128 layer: [wave][kk][j][lane], lane-contiguous (no bank
// conflicts).  VGPRs hold W1 + m (64 per lane); a third register copy would not fit the
// 256-register budget of 2 waves/SIMD without spilling
constexpr int V1S = DZ3 + 16;
constexpr int TOTAL = V1S + 8 * KS * 2 * 64;
}  // namespace blk

__device__ __forceinline__ float sel4(const float (&v)[4], int i) {
  return i == 0 ? v[0] : (i == 1 ? v[1] : (i == 2 ? v[2] : v[3]));
}

__device__ __forceinline__ float swz_xor4(float v) {
  // ds_swizzle bit-mask mode: and 0x1f, or 0, xor 4 (within 32 lanes)
  return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), (4 << 10) | 0x1f));
}

// Reduce-scatter of 32 per-lane values over the wave: returns, in lanes l and l^1, the sum over
// all 64 lanes of value index l >> 1.  Recursive halving over lane bits 5..1 (a lane keeps the
// half of its values whose index bit equals its lane bit and adds the partner's copy of that
// half), then an all-reduce over lane bit 0.
__device__ __forceinline__ float butterfly32(float (&P)[32], int lane) {
#pragma unroll
  for (int i = 0; i < 16; ++i) {  // lane bit 5: v_permlane32_swap exchanges the two half-waves
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(P[i]), __float_as_uint(P[i + 16]), false, false);
    P[i] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {  // lane bit 4: odd/even 16-lane rows
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(P[i]), __float_as_uint(P[i + 8]), false, false);
    P[i] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
  const bool b3 = (lane >> 3) & 1, b2 = (lane >> 2) & 1, b1 = (lane >> 1) & 1;
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // lane bit 3: row_ror:8 == xor 8 inside a 16-lane row
    const float keep = b3 ? P[i + 4] : P[i], send = b3 ? P[i] : P[i + 4];
    P[i] = keep + dppf<0x128>(send);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {  // lane bit 2
    const float keep = b2 ? P[i + 2] : P[i], send = b2 ? P[i] : P[i + 2];
    P[i] = keep + swz_xor4(send);
  }
  const float keep = b1 ? P[1] : P[0], send = b1 ? P[0] : P[1];
  const float r = keep + dppf<0x4E>(send);  // lane bit 1: quad_perm [2,3,0,1]
  return r + dppf<0xB1>(r);                 // lane bit 0: all-reduce, quad_perm [1,0,3,2]
}

// ND: input slices per thread (D0 <= 4 * ND); ADAM: train mode (fused Adam) vs grad mode
// (gradients + loss to grad_out) - separate instantiations, so neither carries the other's
// loop-invariant addresses in VGPRs
template <int ND, bool ADAM>
__global__ __launch_bounds__(blk::NT, 1) void mlp_block_kernel(MlpShape sh, MlpArgs a) {
  using namespace blk;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int D0 = sh.dims[0], C = sh.dims[3];
  constexpr bool adam = ADAM;
  const int oq = tid >> 2, q = tid & 3;    // F1 / B0 roles: unit oq, input slice q (d = q + 4i)
  const int ob = tid & 127, bb = tid >> 7;  // F2r / B2 roles: (unit, row); wave w -> row w >> 1
  const int wo0 = sh.woff[0], bo0 = sh.boff[0], wo1 = sh.woff[1], bo1 = sh.boff[1];
  const int wo2 = sh.woff[2], bo2 = sh.boff[2];

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

  // ---- registers: W1 slice (+ moments), W0 slice, owned biases / last-layer weights
  float w1[2][KS], m1[2][KS];
  auto v1s = [&](int j, int kk) -> float& { return lds[V1S + ((w * KS + kk) * 2 + j) * 64 + l]; };
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      const int f = wo1 + (l + 64 * j) * H + KS * w + kk;
      w1[j][kk] = a.p[f];
      m1[j][kk] = adam ? a.m[f] : 0.f;
    }
  float w0[ND], m0[ND], v0[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) {
    const int d = q + 4 * i;
    const bool ok = d < D0;
    const int f = wo0 + oq * D0 + (ok ? d : 0);
    w0[i] = ok ? a.p[f] : 0.f;
    m0[i] = (ok && adam) ? a.m[f] : 0.f;
    v0[i] = (ok && adam) ? a.v[f] : 0.f;
  }
  // q == 0 owns b0[oq], q == 1 owns b1[oq]; (ob, bb < C) owns W2[bb][ob]; tid < C owns b2[tid]
  const int fbias = (q == 0 ? bo0 : bo1) + oq;
  float mb = 0.f, vb = 0.f;
  if (adam && q < 2) { mb = a.m[fbias]; vb = a.v[fbias]; }
  const bool own_w2 = bb < C;
  const int fw2 = wo2 + bb * H + ob;
  float pw2 = 0.f, mw2 = 0.f, vw2 = 0.f;
  if (own_w2) { pw2 = a.p[fw2]; if (adam) { mw2 = a.m[fw2]; vw2 = a.v[fw2]; } }
  float pb2 = 0.f, mb2 = 0.f, vb2 = 0.f;
  if (tid < C) { pb2 = a.p[bo2 + tid]; if (adam) { mb2 = a.m[bo2 + tid]; vb2 = a.v[bo2 + tid]; } }

  // ---- LDS: biases, last-layer weights, first batch
  for (int e = tid; e < TOTAL; e += NT) lds[e] = 0.f;
  __syncthreads();
  if (tid < H) { lds[B0S + tid] = a.p[bo0 + tid]; lds[B1S + tid] = a.p[bo1 + tid]; }
  if (adam) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) v1s(j, kk) = a.v[wo1 + (l + 64 * j) * H + KS * w + kk];
  }
  for (int e = tid; e < C * H; e += NT) lds[W2S + e] = a.p[wo2 + e];
  if (tid < C) lds[B2S + tid] = pb2;
  const int Bsz = a.B;
  {
    const int bs0 = min(Bsz, a.n_items - cur0 * Bsz);
    if (tid < B * DMAX) {
      const int b = tid & 3, d = tid >> 2;
      float x = 0.f;
      if (b < bs0 && d < D0) x = a.X[(size_t)a.idx[cur0 * Bsz + b] * a.ldx + d];
      lds[XT + d * 4 + b] = x;
    }
    if (tid < B) reinterpret_cast<int*>(lds + LAB)[tid] = (tid < bs0) ? a.Y[a.idx[cur0 * Bsz + tid]] : 0;
  }
  // prefetch roles: thread -> (row pb, feature pk) of the next batch, or (row pb, label)
  const int nel = Bsz * D0;
  int role = 0, pb = 0, pk = 0;
  if (tid < nel) { role = 1; pb = tid / D0; pk = tid - pb * D0; }
  else if (tid < nel + Bsz) { role = 2; pb = tid - nel; }
  int ridx_next = 0;
  if (role && (cur0 + 1) * Bsz + pb < a.n_items) ridx_next = a.idx[(cur0 + 1) * Bsz + pb];
  __syncthreads();

  const float p_drop = a.dropout;
  const float scale = p_drop > 0.f ? 1.0f / (1.0f - p_drop) : 1.0f;  // = dscale of the backward
  const float l2b1 = log2f(a.b1), l2b2 = log2f(a.b2);
  int buf = 0;
  for (int s = 0; s < a.steps; ++s) {
    const int sb = s + cur0;
    const int bs = min(Bsz, a.n_items - sb * Bsz);
    const uint32_t gstep = step_base + (uint32_t)s;
    const float* xT = lds + XT + buf * DMAX * 4;
    const int* lab = reinterpret_cast<const int*>(lds + LAB) + buf * 4;
    const bool have_next = (s + 1 < a.steps);
    const int bs_next = have_next ? min(Bsz, a.n_items - (sb + 1) * Bsz) : 0;
    const uint32_t* src = (role == 1) ? reinterpret_cast<const uint32_t*>(a.X) + (size_t)ridx_next * a.ldx + pk
                                      : reinterpret_cast<const uint32_t*>(a.Y) + ridx_next;
    const uint32_t raw_next = *src;
    const int nx2 = min((sb + 2) * Bsz + pb, a.n_items - 1);
    const int ridx_next2 = a.idx[nx2 < 0 ? 0 : nx2];

    // ---- F1: h1[b][oq] for b = q (quad all-reduce over the 4 input slices)
    {
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < ND; ++i) {
        if (q + 4 * i < D0) {
          const float4 x = *reinterpret_cast<const float4*>(xT + (q + 4 * i) * 4);
          acc[0] += w0[i] * x.x; acc[1] += w0[i] * x.y; acc[2] += w0[i] * x.z; acc[3] += w0[i] * x.w;
        }
      }
#pragma unroll
      for (int b = 0; b < 4; ++b) { acc[b] += dppf<0xB1>(acc[b]); acc[b] += dppf<0x4E>(acc[b]); }
      float z = fmaxf(sel4(acc, q) + lds[B0S + oq], 0.f);
      if (p_drop > 0.f) {
        const uint32_t hsh = mix_hash(a.seed, gstep, (uint32_t)((0 * 64 + q) * 65536 + oq));
        z = (u01(hsh) < p_drop) ? 0.f : z * scale;
      }
      lds[H1T + oq * 4 + q] = z;
    }
    lds_barrier();
    // ---- F2: k-slice partials of the 128x128 layer
    {
      float acc[2][4] = {};
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) {
        const float4 h = *reinterpret_cast<const float4*>(lds + H1T + (KS * w + kk) * 4);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc[j][0] += w1[j][kk] * h.x; acc[j][1] += w1[j][kk] * h.y;
          acc[j][2] += w1[j][kk] * h.z; acc[j][3] += w1[j][kk] * h.w;
        }
      }
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int b = 0; b < 4; ++b) lds[PART + (w * 4 + b) * H + l + 64 * j] = acc[j][b];
    }
    lds_barrier();
    // ---- F2r: h2[bb][ob] = act(sum of slices + b1); logit partials of this wave (row bb)
    {
      float sacc = 0.f;
#pragma unroll
      for (int ww = 0; ww < 8; ++ww) sacc += lds[PART + (ww * 4 + bb) * H + ob];
      float z = fmaxf(sacc + lds[B1S + ob], 0.f);
      if (p_drop > 0.f) {
        const uint32_t hsh = mix_hash(a.seed, gstep, (uint32_t)((1 * 64 + bb) * 65536 + ob));
        z = (u01(hsh) < p_drop) ? 0.f : z * scale;
      }
      lds[H2T + ob * 4 + bb] = z;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if (c < C) {
          const float v = wave_sum(lds[W2S + c * H + ob] * z);
          if (l == 0) lds[ZP + w * 4 + c] = v;
        }
      }
    }
    lds_barrier();
    // ---- F3 + loss: 4 lanes of wave 0, one per row
    if (tid < 4) {
      const int b = tid;
      const bool live = b < bs;
      const float inv = live ? 1.0f / (float)(bs > 0 ? bs : 1) : 0.f;
      float z[4], dz[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 4; ++c)
        z[c] = (c < C) ? lds[ZP + (2 * b) * 4 + c] + lds[ZP + (2 * b + 1) * 4 + c] + lds[B2S + c] : 0.f;
      const LossAcc r = row_loss4(z, C, lab[b], a.loss_kind, inv, dz);
#pragma unroll
      for (int c = 0; c < 4; ++c) lds[DZ3 + b * 4 + c] = dz[c];
      float lv = live ? r.loss : 0.f;
      lv += dppf<0xB1>(lv);
      lv += dppf<0x4E>(lv);
      if (tid == 0) {
        const float bl = bs > 0 ? lv / (float)bs : 0.f;
        if (a.loss_out && !a.cursor) a.loss_out[s] = bl;
        if (!adam) a.grad_out[sh.P] = bl;
      }
    }
    lds_barrier();

    const int t = t0 + s + 1;
    const float step_size = a.lr / (1.f - pow_t(l2b1, (float)t));
    const float rbc2 = __builtin_amdgcn_rsqf(1.f - pow_t(l2b2, (float)t));
    // ---- B2: dZ2 (masked), dW2 / db2 on their owners
    {
      const float4 d3 = *reinterpret_cast<const float4*>(lds + DZ3 + bb * 4);
      const float dd[4] = {d3.x, d3.y, d3.z, d3.w};
      float g = 0.f;
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (c < C) g += lds[W2S + c * H + ob] * dd[c];
      const float hv = lds[H2T + ob * 4 + bb];
      lds[DZ2T + ob * 4 + bb] = hv > 0.f ? g * scale : 0.f;
      if (own_w2) {
        const float4 h4 = *reinterpret_cast<const float4*>(lds + H2T + ob * 4);
        const float gw = lds[DZ3 + 0 * 4 + bb] * h4.x + lds[DZ3 + 1 * 4 + bb] * h4.y + lds[DZ3 + 2 * 4 + bb] * h4.z +
                         lds[DZ3 + 3 * 4 + bb] * h4.w;
        if (adam) adam_elem(pw2, gw, mw2, vw2, a.b1, a.b2, a.wd, step_size, rbc2, a.eps);
        else a.grad_out[fw2] = gw;
      }
      if (tid < C) {
        const float gb2 = lds[DZ3 + tid] + lds[DZ3 + 4 + tid] + lds[DZ3 + 8 + tid] + lds[DZ3 + 12 + tid];
        if (adam) adam_elem(pb2, gb2, mb2, vb2, a.b1, a.b2, a.wd, step_size, rbc2, a.eps);
        else a.grad_out[bo2 + tid] = gb2;
      }
    }
    lds_barrier();
    // ---- B1: dZ1 by the register butterfly; dW1 + Adam in registers
    {
      if (adam && own_w2) lds[W2S + bb * H + ob] = pw2;  // W2 / b2 were last read in B2
      if (adam && tid < C) lds[B2S + tid] = pb2;
      float4 dzj[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) dzj[j] = *reinterpret_cast<const float4*>(lds + DZ2T + (l + 64 * j) * 4);
#pragma unroll
      for (int half = 0; half < 2; ++half) {  // two 32-value passes keep the VGPR budget
        float P[32];
#pragma unroll
        for (int k2 = 0; k2 < KS / 2; ++k2) {
          const int kk = half * (KS / 2) + k2;
          P[k2 * 4 + 0] = w1[0][kk] * dzj[0].x + w1[1][kk] * dzj[1].x;
          P[k2 * 4 + 1] = w1[0][kk] * dzj[0].y + w1[1][kk] * dzj[1].y;
          P[k2 * 4 + 2] = w1[0][kk] * dzj[0].z + w1[1][kk] * dzj[1].z;
          P[k2 * 4 + 3] = w1[0][kk] * dzj[0].w + w1[1][kk] * dzj[1].w;
        }
        const float tot = butterfly32(P, l);
        if ((l & 1) == 0) {
          const int k = KS * w + half * (KS / 2) + (l >> 3), b = (l >> 1) & 3;
          const float hv = lds[H1T + k * 4 + b];
          lds[DZ1T + k * 4 + b] = hv > 0.f ? tot * scale : 0.f;
        }
      }
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) {
        const float4 h = *reinterpret_cast<const float4*>(lds + H1T + (KS * w + kk) * 4);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const float gw = dzj[j].x * h.x + dzj[j].y * h.y + dzj[j].z * h.z + dzj[j].w * h.w;
          if (adam) adam_elem(w1[j][kk], gw, m1[j][kk], v1s(j, kk), a.b1, a.b2, a.wd, step_size, rbc2, a.eps);
          else a.grad_out[wo1 + (l + 64 * j) * H + KS * w + kk] = gw;
        }
      }
    }
    lds_barrier();
    // ---- B0: dW0, db0, db1 + the next batch into the other half of the input tile
    {
      const float4 dz = *reinterpret_cast<const float4*>(lds + DZ1T + oq * 4);
#pragma unroll
      for (int i = 0; i < ND; ++i) {
        const int d = q + 4 * i;
        if (d < D0) {
          const float4 x = *reinterpret_cast<const float4*>(xT + d * 4);
          const float gw = dz.x * x.x + dz.y * x.y + dz.z * x.z + dz.w * x.w;
          if (adam) adam_elem(w0[i], gw, m0[i], v0[i], a.b1, a.b2, a.wd, step_size, rbc2, a.eps);
          else a.grad_out[wo0 + oq * D0 + d] = gw;
        }
      }
      if (q < 2) {
        const float4 g4 = *reinterpret_cast<const float4*>(lds + (q == 0 ? DZ1T : DZ2T) + oq * 4);
        const float gb = g4.x + g4.y + g4.z + g4.w;
        float* pbias = lds + (q == 0 ? B0S : B1S) + oq;
        if (adam) {
          float pv = *pbias;
          adam_elem(pv, gb, mb, vb, a.b1, a.b2, a.wd, step_size, rbc2, a.eps);
          *pbias = pv;
        } else {
          a.grad_out[fbias] = gb;
        }
      }
      if (role) {
        const uint32_t v = (have_next && pb < bs_next) ? raw_next : 0u;
        uint32_t* dst = (role == 1) ? reinterpret_cast<uint32_t*>(lds + XT + (buf ^ 1) * DMAX * 4) + pk * 4 + pb
                                    : reinterpret_cast<uint32_t*>(lds + LAB) + (buf ^ 1) * 4 + pb;
        *dst = v;
      }
      ridx_next = role ? ridx_next2 : 0;
    }
    lds_barrier();
    buf ^= 1;
  }
  if (a.cursor && tid == 0) __hip_atomic_store(a.cursor, cur0 + a.steps, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (a.step_counter && tid == 0)
    __hip_atomic_store(a.step_counter, t0 + a.steps, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (!adam) return;

  // ---- write back parameters and moments (flat torch order)
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      const int f = wo1 + (l + 64 * j) * H + KS * w + kk;
      a.p[f] = w1[j][kk];
      a.m[f] = m1[j][kk];
      a.v[f] = v1s(j, kk);
    }
#pragma unroll
  for (int i = 0; i < ND; ++i) {
    const int d = q + 4 * i;
    if (d < D0) {
      const int f = wo0 + oq * D0 + d;
      a.p[f] = w0[i];
      a.m[f] = m0[i];
      a.v[f] = v0[i];
    }
  }
  if (q < 2) {
    a.p[fbias] = lds[(q == 0 ? B0S : B1S) + oq];
    a.m[fbias] = mb;
    a.v[fbias] = vb;
  }
  if (own_w2) { a.p[fw2] = pw2; a.m[fw2] = mw2; a.v[fw2] = vw2; }
  if (tid < C) { a.p[bo2 + tid] = pb2; a.m[bo2 + tid] = mb2; a.v[bo2 + tid] = vb2; }
}

bool mlp_block_ok(const MlpShape& sh, const MlpArgs& a) {
  const char* env = getenv("DCT_MLP_BLOCK");  // "0": use the generic LDS kernel (A/B, tests)
  const bool off = env && env[0] == '0';
  return !off && sh.L == 3 && sh.dims[1] == blk::H && sh.dims[2] == blk::H && sh.dims[0] >= 1 &&
         sh.dims[0] <= blk::DMAX && sh.dims[3] >= 1 && sh.dims[3] <= 4 && a.B >= 1 && a.B <= blk::B &&
         a.prof == nullptr && a.pending == nullptr && a.stage == nullptr && a.xg_world <= 1 &&
         (a.mode == 0 || a.mode == 1);
}

hipError_t mlp_launch_block(const MlpShape& sh, const MlpArgs& a, hipStream_t st) {
  const int d0 = sh.dims[0];
  const bool tr = a.mode == 0;
  const size_t bytes = (size_t)blk::TOTAL * sizeof(float);
  static bool attr_set = false;
  if (!attr_set) {
    const void* fns[6] = {(const void*)mlp_block_kernel<2, true>, (const void*)mlp_block_kernel<2, false>,
                          (const void*)mlp_block_kernel<4, true>, (const void*)mlp_block_kernel<4, false>,
                          (const void*)mlp_block_kernel<8, true>, (const void*)mlp_block_kernel<8, false>};
    for (const void* f : fns) {
      const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
      if (e != hipSuccess) return e;
    }
    attr_set = true;
  }
#define BLK(ND)                                                                              \
  do {                                                                                       \
    if (tr) hipLaunchKernelGGL((mlp_block_kernel<ND, true>), dim3(1), dim3(blk::NT), bytes, st, sh, a);  \
    else hipLaunchKernelGGL((mlp_block_kernel<ND, false>), dim3(1), dim3(blk::NT), bytes, st, sh, a);    \
  } while (0)
  if (d0 <= 8) BLK(2);
  else if (d0 <= 16) BLK(4);
  else BLK(8);
#undef BLK
  return hipGetLastError();
}

}  // namespace dct
