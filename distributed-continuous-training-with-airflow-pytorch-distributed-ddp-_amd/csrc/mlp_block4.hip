// Sixteen-wave register-resident trainer for 3-layer MLPs D0 -> 128 -> 128 -> C (C <= 4, D0 <= 32,
// batch <= 4): BASELINE "Weather MLP (3-layer, 128-h)" (models/mlp.py preset weather-mlp-3x128;
// the reference's WeatherClassifier with a second 128-wide hidden layer,
// jobs/train_lightning_ddp.py:57-62,69,88,122).  Same contract, dropout hash, loss and Adam as
// mlp_train_kernel; selected by dct_mlp_train (DCT_MLP_BLOCK=3 / 2 select its 8-wave predecessors).
//
// Why 16 waves: on MI355X one wave issues at most one VALU op per ~5 cycles (9.6 when the next
// op depends on the previous one) while a SIMD retires one per ~2.45 (tools/probes/valu_probe.hip,
// profiles/valu_probe_r3.log).  The 8-wave kernels keep their SIMDs ~55 % busy: the step is a
// chain of reductions whose latency two waves per SIMD cannot hide.  Here every SIMD holds 4 waves
// and every wave half the k-slice, so the per-wave chain is half as long and 4 waves interleave.
//
// Per step (wave w, lane l = (hh: bit 5, u': bits 2-4, r0: bits 0-1), unit / output u = 8w + u'):
//   * W1 k-slice [8w, 8w+8) of outputs o = l, l + 64 (+ both Adam moments) in VGPRs;
//   * F1: layer 0 of unit u for row r0, input slices split between the two halves hh;
//   * F2: 4x4x1 fp32 MFMA partials of all 128 outputs over the wave's 8 k -> LDS;  BARRIER A;
//   * Phase 1: h2[u][r0] summed over the 16 partials (8 per half + permlane32), bias, ReLU, dropout;
//     the wave's logit share and the h2 > 0 mask go to LDS;  BARRIER B;
//   * Phase 2: logits = sum of the 16 shares, loss, dlogits (wave-uniform);
//   * dZ2 of all 128 outputs (old W2 from LDS + masks), owner updates of W2[:, u] / b1[u] (quad
//     reductions) and b2, dZ1 by a 32-value permlane / DPP reduce-scatter, dW0 / db0, dW1 (MFMA).
#include "mlp_block_util.h"

namespace dct {

namespace blk4 {
constexpr int H = 128, NT = 1024, NW = 16, KS = 8, DMAX = 32, B = 4;
constexpr int XT = 0;                     // [3][DMAX][4] input tile, transposed (unit-major, 4 rows)
constexpr int LAB = XT + 3 * DMAX * 4;    // [3][4] labels (int), 16 reserved
constexpr int MSK = LAB + 16;             // [2][NW] uint32: h2 > 0 of (o = 8w + b/4, row b%4)
constexpr int LOGP = MSK + 2 * NW;        // [2][NW][4 rows][4 classes] logit shares
constexpr int H1W = LOGP + 2 * NW * 16;   // [NW][KS][4] wave-private layer-1 inputs h1[k][row]
constexpr int H1X = H1W + NW * KS * 4;    // [NW][4][KS] the same tile transposed (MFMA A operands)
constexpr int PSTR = NW * 4 + 4;          // partials: [o][wave][4], padded o stride
constexpr int PART = H1X + NW * KS * 4;   // [2][H][PSTR]
constexpr int W2L = PART + 2 * H * PSTR;  // [2][H][4] W2[c][o] (o-major), published by the owners
constexpr int B2L = W2L + 2 * H * 4;      // [2][4] b2
constexpr int TOTAL = B2L + 8;
constexpr int STG = H * H;
constexpr int LDS_FLOATS = TOTAL > 2 * STG ? TOTAL : 2 * STG;  // two staging tiles (prologue/epilogue)
// VL: the second Adam moment of W1 lives in LDS (the [128][128] staging layout at offset 0, the step
// tiles after it) instead of 16 VGPRs per lane - a 16-wave workgroup has 128 VGPRs per lane
constexpr int LDS_FLOATS_VL = STG + TOTAL > 2 * STG ? STG + TOTAL : 2 * STG;
static_assert(LDS_FLOATS * 4 <= 160 * 1024 && LDS_FLOATS_VL * 4 <= 160 * 1024, "fits the CU");
static_assert((H1W % 4) == 0 && (PART % 4) == 0 && (MSK % 4) == 0 && (LAB % 4) == 0 && (W2L % 4) == 0 &&
                  (B2L % 4) == 0 && (H1X % 4) == 0 && (LOGP % 4) == 0,
              "16-B aligned tiles");
using Stg = bku::Stage<H, NT>;
}  // namespace blk4

namespace b4d {
using namespace bku;
// One pass of dZ1's reduce-scatter: 16 per-lane values, index v = 2 k' + rl (k' = 0..7, rl = row
// low bit, rows 2p + rl of pass p).  Afterwards lane l holds the wave sum of value
// 2 ((l >> 2) & 7) + (l & 1), i.e. (k' = lane bits 2-4, rl = lane bit 0); bits 1 and 5 all-reduced.
// Levels: lane bit 4 (v_permlane16_swap, no selects), 3 (row_ror 8 = lane ^ 8), 2 (row_half_mirror,
// partner lane ^ 7: bits 0-1 undecided), 0 (lane ^ 1), all-reduce over bit 1 (lane ^ 2) and bit 5.
// Two passes of 16 live values instead of one of 32: the 16-wave kernel has 128 VGPRs per lane.
__device__ __forceinline__ float rs16x(float (&P)[16], int lane) {
#pragma unroll
  for (int i = 0; i < 8; ++i) P[i] = swap16_sum(P[i], P[i + 8]);
  const bool b3 = (lane >> 3) & 1, b2 = (lane >> 2) & 1, b0 = lane & 1;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float keep = b3 ? P[i + 4] : P[i], send = b3 ? P[i] : P[i + 4];
    P[i] = keep + dpp<ROR8>(send);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const float keep = b2 ? P[i + 2] : P[i], send = b2 ? P[i] : P[i + 2];
    P[i] = keep + dpp<HMIRROR>(send);
  }
  const float keep = b0 ? P[1] : P[0], send = b0 ? P[0] : P[1];
  float r = keep + dpp<QP_X1>(send);
  r += dpp<QP_X2>(r);
  return swap32_sum(r, r);
}
}  // namespace b4d

// PROF (diagnostic instantiation, launched only when MlpArgs::prof is set): lane 0 of every wave
// sums s_memtime deltas per phase into prof[wave * 16 + phase] (tools/prof_block.py)
#define B4STAMP(k)                                              \
  if constexpr (PROF) {                                         \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    pacc[(k)] += t_ - t_last;                                   \
    t_last = t_;                                                \
  }

// NDL: input slices per lane (D0 <= 8 * NDL); CM: class capacity (2 or 4); ADAM: train mode vs grad
// mode; MF: layer-1 forward and dW1 on the 4x4x1 MFMA; WD: L2 term in Adam.
template <int NDL, int CM, bool ADAM, bool PROF = false, bool MF = false, bool WD = true, bool VL = false>
__global__ __launch_bounds__(blk4::NT, 1) void mlp_block4_kernel(MlpShape sh, MlpArgs a) {
  using namespace blk4;
  using namespace b4d;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr bool VLD = VL && ADAM;
  float* const tl = lds + (VLD ? STG : 0);  // step tiles (XT ... B2L)
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int D0 = sh.dims[0], C = sh.dims[3];
  const int hh = l >> 5, r0 = l & 3;
  const int u = KS * w + ((l >> 2) & 7);  // unit of layer 0 / output of layer 1 this lane serves
  const int wo0 = sh.woff[0], bo0 = sh.boff[0], wo1 = sh.woff[1], bo1 = sh.boff[1];
  const int wo2 = sh.woff[2], bo2 = sh.boff[2];
  unsigned long long pacc[PROF ? 11 : 1] = {};
  unsigned long long t_last = PROF ? __builtin_amdgcn_s_memtime() : 0ull;
  const unsigned long long t_kstart = t_last;

  // ---- W1 + moments: issued first, coalesced, redistributed through LDS below
  v4f sp[Stg::LD], sm[Stg::LD], sv[Stg::LD];
#pragma unroll
  for (int i = 0; i < Stg::LD; ++i) {
    const int f = wo1 + 4 * (i * NT + tid);
    sp[i] = *reinterpret_cast<const v4f*>(a.p + f);
    if (ADAM) {
      sm[i] = *reinterpret_cast<const v4f*>(a.m + f);
      sv[i] = *reinterpret_cast<const v4f*>(a.v + f);
    }
  }
  // W0[u][d] for this lane's input slices d = r0 + 4 (hh + 2i); b0[u] in every lane of the unit
  float w0[NDL], m0[NDL], v0[NDL];
#pragma unroll
  for (int i = 0; i < NDL; ++i) {
    const int d = r0 + 4 * (hh + 2 * i);
    const bool ok = d < D0;
    const int f = wo0 + u * D0 + (ok ? d : 0);
    w0[i] = ok ? a.p[f] : 0.f;
    m0[i] = (ok && ADAM) ? a.m[f] : 0.f;
    v0[i] = (ok && ADAM) ? a.v[f] : 0.f;
  }
  float pb0 = a.p[bo0 + u], mb0 = ADAM ? a.m[bo0 + u] : 0.f, vb0 = ADAM ? a.v[bo0 + u] : 0.f;
  // W2 column u (every lane of the quad, all CM classes); lanes r0 < C own W2[r0][u] (+ moments;
  // both halves update it identically, hh = 0 writes it back); b1[u] likewise; b2: wave 0, lane c
  float pw2[CM];
#pragma unroll
  for (int c = 0; c < CM; ++c) pw2[c] = c < C ? a.p[wo2 + c * H + u] : 0.f;
  const bool own_w2 = r0 < C;
  const int fw2 = wo2 + (own_w2 ? r0 : 0) * H + u;
  float mw2 = (own_w2 && ADAM) ? a.m[fw2] : 0.f, vw2 = (own_w2 && ADAM) ? a.v[fw2] : 0.f;
  float pb1 = a.p[bo1 + u], mb1 = ADAM ? a.m[bo1 + u] : 0.f, vb1 = ADAM ? a.v[bo1 + u] : 0.f;
  const bool own_b2 = w == 0 && l < C;
  const int fb2 = bo2 + (own_b2 ? l : 0);
  float pb2 = own_b2 ? a.p[fb2] : 0.f, mb2 = (own_b2 && ADAM) ? a.m[fb2] : 0.f, vb2 = (own_b2 && ADAM) ? a.v[fb2] : 0.f;

  // cursor, step counter and the first batch's row indices through the scalar cache
  const int cur0 = a.cursor ? sload(a.cursor) : 0;
  int t0 = a.t0;
  uint32_t step_base = a.step_base;
  if (a.step_counter) {
    t0 = sload(a.step_counter);
    step_base = (uint32_t)t0;
  }
  const int Bsz = a.B;
  const int bs0 = min(Bsz, a.n_items - cur0 * Bsz);
  int ridx[B];
#pragma unroll
  for (int b = 0; b < B; ++b) ridx[b] = b < bs0 ? sload(a.idx + cur0 * Bsz + b) : 0;
  float x_first = 0.f;
  int lab_first = 0;
  {
    const int b = tid & 3, d = tid >> 2;
    const int rb = ridx[0] * (b == 0) + ridx[1] * (b == 1) + ridx[2] * (b == 2) + ridx[3] * (b == 3);
    if (tid < B * DMAX && b < bs0 && d < D0) x_first = a.X[(size_t)rb * a.ldx + d];
    if (tid < B && tid < bs0) lab_first = a.Y[rb];
  }

  // ---- W1 k-slice + moments into registers through the swizzled staging tiles
  float w1[2][KS], m1[2][KS], v1[VLD ? 1 : 2][VLD ? 1 : KS];
  Stg::put(lds, sp, tid);
  if (ADAM) Stg::put(lds + STG, sm, tid);
  __syncthreads();
  Stg::get<KS>(lds, w1, l, KS / 4 * w);
  if (ADAM) {
    Stg::get<KS>(lds + STG, m1, l, KS / 4 * w);
    __syncthreads();
    if constexpr (VLD) {  // v / (1 - b2) straight into its LDS home (tile 0, staging layout)
      const float rcv = 1.f / (1.f - a.b2);
#pragma unroll
      for (int i = 0; i < Stg::LD; ++i) sv[i] *= rcv;
    }
    Stg::put(lds, sv, tid);
    if constexpr (!VLD) {
      __syncthreads();
      Stg::get<KS>(lds, v1, l, KS / 4 * w);
    }
  } else {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int k = 0; k < KS; ++k) m1[j][k] = 0.f;
#pragma unroll
    for (int j = 0; j < (VLD ? 1 : 2); ++j)
#pragma unroll
      for (int k = 0; k < (VLD ? 1 : KS); ++k) v1[j][k] = 0.f;
  }
  __syncthreads();  // staging reads done before the tiles (same LDS) are zeroed
  if (tid == 0 && cur0 > 0 && a.loss_out) a.loss_out[cur0 - 1] = a.grad_out[sh.P];

  // ---- LDS: first batch into input buffer 0, W2 / b2 into publish buffer 0
  for (int e = 4 * tid; e < TOTAL; e += 4 * NT) *reinterpret_cast<float4*>(tl + e) = make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();
  if (tid < B * DMAX) tl[XT + (tid >> 2) * 4 + (tid & 3)] = x_first;
  if (tid < B) reinterpret_cast<int*>(tl + LAB)[tid] = lab_first;
  if (own_w2 && hh == 0) tl[W2L + u * 4 + r0] = selc<CM>(pw2, r0);  // classes >= C stay 0
  if (own_b2) tl[B2L + l] = pb2;
  // prefetch roles: thread -> (row pb, feature pk) of the next batch, or (row pb, label)
  const int nel = Bsz * D0;
  int role = 0, pb = 0, pk = 0;
  if (tid < nel) { role = 1; pb = tid / D0; pk = tid - pb * D0; }
  else if (tid < nel + Bsz) { role = 2; pb = tid - nel; }
  int ridx_next = 0;
  if (role && (cur0 + 1) * Bsz + pb < a.n_items) ridx_next = a.idx[(cur0 + 1) * Bsz + pb];
  const uint32_t* pf_base = role == 1 ? reinterpret_cast<const uint32_t*>(a.X) + pk : reinterpret_cast<const uint32_t*>(a.Y);
  const int pf_stride = role == 1 ? a.ldx : (role == 2 ? 1 : 0);
  __syncthreads();

  const float p_drop = a.dropout;
  const bool drop = p_drop > 0.f;
  const float scale = drop ? 1.0f / (1.0f - p_drop) : 1.0f;
  const float l2b1 = log2f(a.b1), l2b2 = log2f(a.b2);
  const float c1 = 1.f - a.b1, c2 = 1.f - a.b2;
  const float rc1 = 1.f / c1, rc2 = 1.f / c2, sqc2 = sqrtf(c2);
  // Adam moments to the scaled form adam_scaled keeps (back on store)
  if (ADAM) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int k = 0; k < KS; ++k) {
        m1[j][k] *= rc1;
        if constexpr (!VLD) v1[j][k] *= rc2;
      }
#pragma unroll
    for (int i = 0; i < NDL; ++i) { m0[i] *= rc1; v0[i] *= rc2; }
    mb0 *= rc1; vb0 *= rc2; mw2 *= rc1; vw2 *= rc2; mb1 *= rc1; vb1 *= rc2; mb2 *= rc1; vb2 *= rc2;
  }
  float* h1w = tl + H1W + w * (KS * 4);
  float* h1x = tl + H1X + w * (KS * 4);
  int xb = 0;
  // wave priority.  Four waves share a SIMD and VALU issue goes to the oldest ready wave, so the
  // last-dispatched quarter (waves 12-15) ends up the step's critical path: it runs its
  // latency-bound loss chain ~5x slower than wave 0 while the older waves idle at barrier A
  // (profiles/block4_r3.log).  tune 1: priority = dispatch quarter (youngest highest); tune 2:
  // youngest quarter only; 0: none.
  {
    const int qw = w >> 2;
    const int tune = a.tune;
    if (tune == 1 || (tune == 2 && qw == 3)) {
      if (qw == 1) __builtin_amdgcn_s_setprio(1);
      else if (qw == 2 && tune == 1) __builtin_amdgcn_s_setprio(2);
      else if (qw == 3) __builtin_amdgcn_s_setprio(3);
    }
  }
  if constexpr (PROF) {
    t_last = __builtin_amdgcn_s_memtime();
    pacc[9] = t_last - t_kstart;  // prologue: parameters + moments in, LDS init, first batch
  }
  for (int s = 0; s < a.steps; ++s) {
    const int sb = s + cur0;
    const int bs = min(Bsz, a.n_items - sb * Bsz);
    const uint32_t gstep = step_base + (uint32_t)s;
    const int xbn = xb == 2 ? 0 : xb + 1;
    const int pbuf = s & 1, nbuf = pbuf ^ 1;
    const float* xT = tl + XT + xb * DMAX * 4;
    const bool have_next = (s + 1 < a.steps);
    const int bs_next = have_next ? min(Bsz, a.n_items - (sb + 1) * Bsz) : 0;
    const uint32_t raw_next = pf_base[(size_t)ridx_next * pf_stride];
    const int nx2 = min((sb + 2) * Bsz + pb, a.n_items - 1);
    const int ridx_next2 = a.idx[nx2 < 0 ? 0 : nx2];

    // ---- F1: h1[u][r0] (quad reduce-scatter over the input slices, permlane32 over the halves)
    float h1;
    {
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < NDL; ++i) {
        const float4 x = *reinterpret_cast<const float4*>(xT + (r0 + 4 * (hh + 2 * i)) * 4);
        acc[0] += w0[i] * x.x; acc[1] += w0[i] * x.y; acc[2] += w0[i] * x.z; acc[3] += w0[i] * x.w;
      }
      const bool qb1 = (r0 >> 1) & 1, qb0 = r0 & 1;
      const float k0 = qb1 ? acc[2] : acc[0], k1 = qb1 ? acc[3] : acc[1];
      const float s0 = qb1 ? acc[0] : acc[2], s1 = qb1 ? acc[1] : acc[3];
      const float e0 = k0 + dpp<QP_X2>(s0), e1 = k1 + dpp<QP_X2>(s1);
      const float kq = qb0 ? e1 : e0, sq = qb0 ? e0 : e1;
      const float zq = kq + dpp<QP_X1>(sq);
      float z = fmaxf(swap32_sum(zq, zq) + pb0, 0.f);
      if (drop) {
        const uint32_t hsh = mix_hash(a.seed, gstep, (uint32_t)((0 * 64 + r0) * 65536 + u));
        z = (u01(hsh) < p_drop) ? 0.f : z * scale;
      }
      h1 = z;
      if (hh == 0) {
        h1w[l] = z;                                  // [k = u'][row]
        if constexpr (MF) h1x[r0 * KS + (l >> 2)] = z;  // [row][k]
      }
    }
    bool keep2 = true;  // layer-1 dropout keep bit of this lane's Phase-1 element (row r0, unit u)
    if (drop) {
      const uint32_t hsh = mix_hash(a.seed, gstep, (uint32_t)((1 * 64 + r0) * 65536 + u));
      keep2 = u01(hsh) >= p_drop;
    }
    __builtin_amdgcn_wave_barrier();
    B4STAMP(0)
    // ---- F2: this wave's k-slice partials of all 128 outputs x 4 rows
    {
      float acc[2][4] = {};
      if constexpr (MF) {
        f32x4_t cj[2] = {(f32x4_t){0.f, 0.f, 0.f, 0.f}, (f32x4_t){0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int q = 0; q < KS / 4; ++q) {
          const float4 hq = *reinterpret_cast<const float4*>(h1x + r0 * KS + 4 * q);
          const float hv[4] = {hq.x, hq.y, hq.z, hq.w};
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int j = 0; j < 2; ++j) cj[j] = mfma4(hv[e], w1[j][4 * q + e], cj[j]);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[j][r] = cj[j][r];
      } else {
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) {
          const float4 h = *reinterpret_cast<const float4*>(h1w + kk * 4);
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            acc[j][0] += w1[j][kk] * h.x; acc[j][1] += w1[j][kk] * h.y;
            acc[j][2] += w1[j][kk] * h.z; acc[j][3] += w1[j][kk] * h.w;
          }
        }
      }
      float* part = tl + PART + pbuf * (H * PSTR);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        *reinterpret_cast<float4*>(part + (l + 64 * j) * PSTR + w * 4) =
            make_float4(acc[j][0], acc[j][1], acc[j][2], acc[j][3]);
    }
    if (role) {  // next batch into the next input buffer
      const uint32_t v = (have_next && pb < bs_next) ? raw_next : 0u;
      uint32_t* dst = (role == 1) ? reinterpret_cast<uint32_t*>(tl + XT + xbn * DMAX * 4) + pk * 4 + pb
                                  : reinterpret_cast<uint32_t*>(tl + LAB) + xbn * 4 + pb;
      *dst = v;
    }
    ridx_next = role ? ridx_next2 : 0;
    B4STAMP(1)
    lds_barrier();  // A: all partials of this step are in
    B4STAMP(2)

    // ---- Phase 1: h2[u][r0] (each half sums 8 of the 16 partials), logit share, h2 > 0 mask
    float h2;
    {
      const float* pr = tl + PART + pbuf * (H * PSTR) + u * PSTR + 32 * hh + r0;
      float z = pr[0];
#pragma unroll
      for (int i = 1; i < 8; ++i) z += pr[4 * i];
      z = fmaxf(swap32_sum(z, z) + pb1, 0.f);
      if (drop) z = keep2 ? z * scale : 0.f;
      h2 = z;
      float tsh[CM];
#pragma unroll
      for (int c = 0; c < CM; ++c) {  // sum over the 8 outputs u' (lane bits 2-4) of the half
        float t = pw2[c] * h2;
        t += dpp<ROR4>(t);
        t += dpp<ROR8>(t);
        tsh[c] = swap16_sum(t, t);
      }
      const unsigned long long msk = __ballot(h2 > 0.f);
      if (l < 4) {
        float t4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < CM; ++c) t4[c] = tsh[c];
        *reinterpret_cast<float4*>(tl + LOGP + pbuf * (NW * 16) + w * 16 + l * 4) = make_float4(t4[0], t4[1], t4[2], t4[3]);
      }
      if (l == 0) reinterpret_cast<uint32_t*>(tl + MSK)[pbuf * NW + w] = (uint32_t)msk;
    }
    B4STAMP(3)
    lds_barrier();  // B: logit shares and masks of every wave are in
    B4STAMP(4)

    // ---- Phase 2: logits (sum of the 16 shares: lane (w' = l / 4, row l % 4)), loss, dlogits
    float dz3[4][CM];
    {
      const float4 sh4 = *reinterpret_cast<const float4*>(tl + LOGP + pbuf * (NW * 16) + l * 4);
      float zs[4] = {sh4.x, sh4.y, sh4.z, sh4.w};
      const float4 t2 = *reinterpret_cast<const float4*>(tl + B2L + pbuf * 4);
      const float b2v[4] = {t2.x, t2.y, t2.z, t2.w};
      float z4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < CM; ++c) z4[c] = sum_bits2to5(zs[c]) + b2v[c];
      const int rr = r0;
      const int4 labs = *reinterpret_cast<const int4*>(tl + LAB + xb * 4);
      const int lab = (rr & 2) ? ((rr & 1) ? labs.w : labs.z) : ((rr & 1) ? labs.y : labs.x);
      const bool live = rr < bs;
      const float inv = live ? 1.0f / (float)(bs > 0 ? bs : 1) : 0.f;
      float dz[4] = {0.f, 0.f, 0.f, 0.f};
      const LossAcc lr_ = row_loss4(z4, C, lab, a.loss_kind, inv, dz);
      const float lv = live ? lr_.loss : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < CM; ++c) dz3[r][c] = (c < C) ? rl(dz[c], r) : 0.f;
      const float ltot = rl(lv, 0) + rl(lv, 1) + rl(lv, 2) + rl(lv, 3);
      const float bl = bs > 0 ? ltot / (float)bs : 0.f;
      if (tid == 0) {
        if (a.loss_out && !a.cursor) a.loss_out[s] = bl;
        if (!ADAM) a.grad_out[sh.P] = bl;
      }
    }
    B4STAMP(5)

    const int t = t0 + s + 1;
    const float step_size = a.lr / (1.f - pow_t(l2b1, (float)t));
    const float rbc2 = __builtin_amdgcn_rsqf(1.f - pow_t(l2b2, (float)t));
    const float rss = __builtin_amdgcn_rcpf(step_size);
    // adam_scaled's folded denominator (moments held as m / (1 - b1), v / (1 - b2))
    const float aA = sqc2 * rbc2 * rss * rc1, aE = a.eps * rss * rc1;
    // ---- dZ2 of every output o = l + 64j (old W2 from LDS, mask bits of the owning wave)
    float dz2[2][4];
    {
      const float* w2p = tl + W2L + pbuf * (H * 4);
      const uint32_t* mk = reinterpret_cast<const uint32_t*>(tl + MSK) + pbuf * NW;
      const int bit = 4 * (l & 7);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int o = l + 64 * j;
        float wv[CM];
        if constexpr (CM == 2) {
          const float2 t2 = *reinterpret_cast<const float2*>(w2p + o * 4);
          wv[0] = t2.x; wv[1 % CM] = t2.y;
        } else {
          const float4 t4 = *reinterpret_cast<const float4*>(w2p + o * 4);
          wv[0] = t4.x; wv[1 % CM] = t4.y; wv[2 % CM] = t4.z; wv[3 % CM] = t4.w;
        }
        const uint32_t m32 = mk[o >> 3];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float g = 0.f;
#pragma unroll
          for (int c = 0; c < CM; ++c) g += wv[c] * dz3[r][c];
          dz2[j][r] = ((m32 >> (bit + r)) & 1u) ? g * scale : 0.f;
        }
      }
    }
    // ---- owners: dW2[:, u] and db1[u] (quad reductions), W2 / b1 / b2 Adam, W2 / b2 published
    {
      float gdz = 0.f;  // this lane's own dZ2[u][r0] (old W2 column in registers)
      float gw2[CM];
#pragma unroll
      for (int c = 0; c < CM; ++c) {
        const float col[4] = {dz3[0][c], dz3[1][c], dz3[2][c], dz3[3][c]};
        const float d = selc<4>(col, r0);
        gdz += pw2[c] * d;
        gw2[c] = quad_sum(d * h2);  // dW2[c][u] = sum_r dz3[r][c] h2[u][r]
      }
      gdz = h2 > 0.f ? gdz * scale : 0.f;
      const float gb1 = quad_sum(gdz);
      const float gown = selc<CM>(gw2, r0);
      float pown = selc<CM>(pw2, r0);
      if (ADAM) {
        if (own_w2) adam_scaled<WD>(pown, gown, mw2, vw2, a.b1, a.b2, a.wd, aA, aE);
#pragma unroll
        for (int c = 0; c < CM; ++c) pw2[c] = c < C ? quad_bcast(pown, c) : 0.f;
        adam_scaled<WD>(pb1, gb1, mb1, vb1, a.b1, a.b2, a.wd, aA, aE);
      } else if (s == 0 && hh == 0) {
        if (own_w2) a.grad_out[fw2] = gown;
        if (r0 == 0) a.grad_out[bo1 + u] = gb1;
      }
      if (own_w2 && hh == 0) tl[W2L + nbuf * (H * 4) + u * 4 + r0] = pown;
      if (own_b2) {
        float gb = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) gb += CM == 2 ? (l ? dz3[r][1 % CM] : dz3[r][0]) : selc<CM>(dz3[r], l);
        if (ADAM) adam_scaled<WD>(pb2, gb, mb2, vb2, a.b1, a.b2, a.wd, aA, aE);
        else if (s == 0) a.grad_out[fb2] = gb;
        tl[B2L + nbuf * 4 + l] = pb2;
      }
    }
    B4STAMP(6)
    // ---- dZ1 = W1^T dZ2 over this wave's k-slice: (k', row r) of the reduce-scatter lands in lane
    // (hh, k', r) - the (unit, row) whose h1 this lane computed in F1
    float dz1 = 0.f;
#pragma unroll
    for (int p = 0; p < 2; ++p) {  // rows 2p, 2p + 1
      float P[16];
#pragma unroll
      for (int kk = 0; kk < KS; ++kk)
#pragma unroll
        for (int rl = 0; rl < 2; ++rl) {
          const int r = 2 * p + rl;
          P[2 * kk + rl] = w1[0][kk] * dz2[0][r] + w1[1][kk] * dz2[1][r];
        }
      const float tot = rs16x(P, l);
      if ((r0 >> 1) == p) dz1 = tot;
    }
    dz1 = h1 > 0.f ? dz1 * scale : 0.f;
    // ---- dW0 / db0: the quad holds unit u's four rows
    {
      float dq[4];
      dq[0] = dpp<QB0>(dz1); dq[1] = dpp<QB1>(dz1); dq[2] = dpp<QB2>(dz1); dq[3] = dpp<QB3>(dz1);
#pragma unroll
      for (int i = 0; i < NDL; ++i) {
        const int d = r0 + 4 * (hh + 2 * i);
        const float4 x = *reinterpret_cast<const float4*>(xT + d * 4);
        const float gw = dq[0] * x.x + dq[1] * x.y + dq[2] * x.z + dq[3] * x.w;
        if (ADAM) adam_scaled<WD>(w0[i], gw, m0[i], v0[i], a.b1, a.b2, a.wd, aA, aE);  // d >= D0: stays 0
        else if (d < D0) a.grad_out[wo0 + u * D0 + d] = gw;
      }
      const float gb = dq[0] + dq[1] + dq[2] + dq[3];
      if (ADAM) adam_scaled<WD>(pb0, gb, mb0, vb0, a.b1, a.b2, a.wd, aA, aE);
      else if (r0 == 0 && hh == 0) a.grad_out[bo0 + u] = gb;
    }
    B4STAMP(7)
    // ---- dW1 + Adam in registers
    int gb1 = wo1 + l * H + KS * w;  // grad mode: opaque per step, so the store addresses are not hoisted
    if (!ADAM) asm volatile("" : "+v"(gb1));
    if constexpr (MF) {
#pragma unroll
      for (int q = 0; q < KS / 4; ++q) {
        const float4 hq = *reinterpret_cast<const float4*>(h1w + (4 * q + r0) * 4);
        const float hv[4] = {hq.x, hq.y, hq.z, hq.w};
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          f32x4_t g = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int r = 0; r < 4; ++r) g = mfma4(hv[r], dz2[j][r], g);
          v4f* vp = reinterpret_cast<v4f*>(lds + Stg::slot(l + 64 * j, KS / 4 * w + q));
          const v4f vq = VLD ? *vp : (v4f){0.f, 0.f, 0.f, 0.f};
          float vv[4] = {vq.x, vq.y, vq.z, vq.w};
#pragma unroll
          for (int m = 0; m < 4; ++m) {
            const int kk = 4 * q + m;
            if constexpr (VLD) adam_scaled<WD>(w1[j][kk], g[m], m1[j][kk], vv[m], a.b1, a.b2, a.wd, aA, aE);
            else if (ADAM) adam_scaled<WD>(w1[j][kk], g[m], m1[j][kk], v1[j][kk], a.b1, a.b2, a.wd, aA, aE);
            else a.grad_out[gb1 + 64 * j * H + kk] = g[m];
          }
          if constexpr (VLD) *vp = (v4f){vv[0], vv[1], vv[2], vv[3]};
        }
      }
    } else {
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) {
        const float4 h = *reinterpret_cast<const float4*>(h1w + kk * 4);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const float gw = dz2[j][0] * h.x + dz2[j][1] * h.y + dz2[j][2] * h.z + dz2[j][3] * h.w;
          if constexpr (VLD) {
            float* vp = lds + Stg::slot(l + 64 * j, KS / 4 * w + kk / 4) + (kk & 3);
            float vv = *vp;
            adam_scaled<WD>(w1[j][kk], gw, m1[j][kk], vv, a.b1, a.b2, a.wd, aA, aE);
            *vp = vv;
          } else if (ADAM) {
            adam_scaled<WD>(w1[j][kk], gw, m1[j][kk], v1[j][kk], a.b1, a.b2, a.wd, aA, aE);
          } else {
            a.grad_out[gb1 + 64 * j * H + kk] = gw;
          }
        }
      }
    }
    __builtin_amdgcn_wave_barrier();  // the next step rewrites this wave's h1 tile
    B4STAMP(8)
    xb = xbn;
  }
  if (a.cursor && tid == 0) __hip_atomic_store(a.cursor, cur0 + a.steps, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (a.step_counter && tid == 0)
    __hip_atomic_store(a.step_counter, t0 + a.steps, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (!ADAM) return;

  // ---- write back parameters and moments (flat torch order); opaque bases, see mlp_block3.hip
  int lo = l, uo = u, to = tid;
  asm volatile("" : "+v"(lo), "+v"(uo), "+v"(to));
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      m1[j][k] *= c1;
      if constexpr (!VLD) v1[j][k] *= c2;
    }
#pragma unroll
  for (int i = 0; i < NDL; ++i) { m0[i] *= c1; v0[i] *= c2; }
  mb0 *= c1; vb0 *= c2; mw2 *= c1; vw2 *= c2; mb1 *= c1; vb1 *= c2; mb2 *= c1; vb2 *= c2;
  __syncthreads();  // every wave is past its last use of the step tiles (the staging aliases them)
  if constexpr (VLD) {  // v: LDS home -> global (times 1 - b2), then the same tile stages w1
#pragma unroll
    for (int i = 0; i < Stg::LD; ++i) {
      const int g = i * NT + to;
      const v4f t4 = *reinterpret_cast<const v4f*>(lds + Stg::slot(g / (H / 4), g % (H / 4)));
      *reinterpret_cast<v4f*>(a.v + wo1 + 4 * g) = t4 * c2;
    }
    __syncthreads();
  }
  Stg::own<KS>(lds, w1, lo, KS / 4 * w);
  Stg::own<KS>(lds + STG, m1, lo, KS / 4 * w);
  __syncthreads();
  Stg::store(a.p + wo1, lds, to);
  Stg::store(a.m + wo1, lds + STG, to);
  if constexpr (!VLD) {
    __syncthreads();
    Stg::own<KS>(lds, v1, lo, KS / 4 * w);
    __syncthreads();
    Stg::store(a.v + wo1, lds, to);
  }
#pragma unroll
  for (int i = 0; i < NDL; ++i) {
    const int d = r0 + 4 * (hh + 2 * i);
    if (d < D0) {
      const int f = wo0 + uo * D0 + d;
      a.p[f] = w0[i];
      a.m[f] = m0[i];
      a.v[f] = v0[i];
    }
  }
  if (r0 == 0 && hh == 0) {
    a.p[bo0 + uo] = pb0; a.m[bo0 + uo] = mb0; a.v[bo0 + uo] = vb0;
    a.p[bo1 + uo] = pb1; a.m[bo1 + uo] = mb1; a.v[bo1 + uo] = vb1;
  }
  if (own_w2 && hh == 0) {
    const int f = wo2 + r0 * H + uo;
    a.p[f] = selc<CM>(pw2, r0); a.m[f] = mw2; a.v[f] = vw2;
  }
  if (own_b2) { a.p[fb2] = pb2; a.m[fb2] = mb2; a.v[fb2] = vb2; }
  if constexpr (PROF) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    pacc[10] = __builtin_amdgcn_s_memtime() - t_last;  // epilogue: write-back issued and retired
    if (l == 0) {
#pragma unroll
      for (int i = 0; i < 11; ++i) atomicAdd(a.prof + w * 16 + i, pacc[i]);
    }
  }
}
#undef B4STAMP

bool mlp_block4_ok(const MlpShape& sh, const MlpArgs& a) {
  // opt-in (DCT_MLP_BLOCK=4) until validated on the GPU; "3" / "2": the 8-wave kernels, "0" / "v1": others
  const char* env = getenv("DCT_MLP_BLOCK");
  if (!(env && env[0] == '4')) return false;
  const bool prof_ok = a.prof == nullptr || (sh.dims[0] <= 8 && sh.dims[3] <= 2 && a.mode == 0);
  const bool aligned = (sh.woff[1] % 4) == 0 && ((uintptr_t)a.p & 15) == 0 &&
                       (a.mode != 0 || (((uintptr_t)a.m | (uintptr_t)a.v) & 15) == 0);
  return prof_ok && aligned && sh.L == 3 && sh.dims[1] == blk4::H && sh.dims[2] == blk4::H && sh.dims[0] >= 1 &&
         sh.dims[0] <= blk4::DMAX && sh.dims[3] >= 1 && sh.dims[3] <= 4 && a.B >= 1 && a.B <= blk4::B &&
         a.pending == nullptr && a.stage == nullptr && a.xg_world <= 1 && (a.mode == 0 || a.mode == 1);
}

template <int NDL, int CM, bool ADAM, bool PROF = false, bool MF = false, bool WD = true, bool VL = false>
static void b4_launch(hipStream_t st, const MlpShape& sh, const MlpArgs& a) {
  const size_t bytes = (size_t)((VL && ADAM) ? blk4::LDS_FLOATS_VL : blk4::LDS_FLOATS) * sizeof(float);
  static const hipError_t attr = hipFuncSetAttribute((const void*)mlp_block4_kernel<NDL, CM, ADAM, PROF, MF, WD, VL>,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  (void)attr;
  hipLaunchKernelGGL((mlp_block4_kernel<NDL, CM, ADAM, PROF, MF, WD, VL>), dim3(1), dim3(blk4::NT), bytes, st, sh, a);
}

hipError_t mlp_launch_block4(const MlpShape& sh, const MlpArgs& a, hipStream_t st) {
  const int d0 = sh.dims[0], C = sh.dims[3];
  const bool tr = a.mode == 0;
  const char* mfe = getenv("DCT_MLP_BLOCK_MF");
  const bool mf = !(mfe && mfe[0] == '0') && d0 <= 8 && C <= 2;
  const bool wd = a.wd != 0.f;
  const char* vle = getenv("DCT_B4_VL");  // "0": W1's second moment in VGPRs (spills at 128 / lane)
  const bool vl = !(vle && vle[0] == '0');
  const char* pe = getenv("DCT_B4_PRIO");
  MlpArgs a2 = a;
  a2.tune = pe ? atoi(pe) : a.tune;
  if (a.prof) {
    if (mf) b4_launch<1, 2, true, true, true, true, true>(st, sh, a2);
    else b4_launch<1, 2, true, true, false, true, true>(st, sh, a2);
  } else if (mf) {
    if (!tr) b4_launch<1, 2, false, false, true>(st, sh, a2);
    else if (wd) {
      if (vl) b4_launch<1, 2, true, false, true, true, true>(st, sh, a2);
      else b4_launch<1, 2, true, false, true, true, false>(st, sh, a2);
    } else {
      if (vl) b4_launch<1, 2, true, false, true, false, true>(st, sh, a2);
      else b4_launch<1, 2, true, false, true, false, false>(st, sh, a2);
    }
  } else {
#define B4K(NDL, CM)                                                \
  do {                                                              \
    if (tr) b4_launch<NDL, CM, true, false, false, true, true>(st, sh, a2); \
    else b4_launch<NDL, CM, false>(st, sh, a2);                      \
  } while (0)
    if (d0 <= 8) {
      if (C <= 2) B4K(1, 2); else B4K(1, 4);
    } else {
      if (C <= 2) B4K(4, 2); else B4K(4, 4);
    }
#undef B4K
  }
  return hipGetLastError();
}

}  // namespace dct
