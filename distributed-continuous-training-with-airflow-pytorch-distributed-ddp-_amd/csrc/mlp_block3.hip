// Two-barrier register-resident trainer for 3-layer MLPs D0 -> 128 -> 128 -> C (C <= 4, D0 <= 32,
// batch <= 4): BASELINE "Weather MLP (3-layer, 128-h)" (models/mlp.py preset weather-mlp-3x128;
// the reference's WeatherClassifier with a second 128-wide hidden layer,
// jobs/train_lightning_ddp.py:57-62,69,88,122).  Same contract as mlp_train_kernel: one workgroup
// runs every step of a launch with the same dropout hash, loss and Adam, so it is a drop-in
// replacement selected by dct_mlp_train (mlp_block2.hip, its one-barrier predecessor, stays
// selectable with DCT_MLP_BLOCK=2 for A/B).
//
// Per step, 8 waves (2 per SIMD):
//   * wave w owns the k-slice [16w, 16w+16) of W1 (lane l: outputs o = l and l + 64, weights and
//     both Adam moments in VGPRs); lane (unit 16w + l/4, row l%4) computes layer 0 for that slice;
//   * layer 1: each wave's k-slice partials of all 128 outputs (4x4x1 fp32 MFMA) go to LDS;
//     BARRIER A; wave w then reduces only ITS 16 outputs (lane = (o, row): eight 4-B reads), adds
//     the bias, ReLU, dropout and forms its share of the logits (W2 column o in registers, all-
//     reduce over the 16 o-lanes), published with the 64-bit h2 > 0 mask;
//     BARRIER B; every wave sums the 8 logit shares (one read per lane), runs the loss and makes
//     dlogits wave-uniform.  The predecessor summed all 8 partials of all 128 outputs in every wave
//     (128 KB of LDS reads per step instead of 16 KB) and reduced the logits over 64 lanes.
//   * wave w owns W2[:, o] and b1[o] of its 16 outputs: the quad of lanes of output o reduces dW2 /
//     db1 with two DPP adds, lane c updates W2[c][o] (quad-broadcast back), b1 is updated in every
//     lane of the quad; the new W2 is published to LDS for the other waves' dZ2 of the next step.
//   * dZ1 = W1^T dZ2 over the wave's k-slice (permlane / DPP reduce-scatter, no LDS), dW0 / db0
//     via quad DPP broadcasts, dW1 on the 4x4x1 MFMA (D0 <= 8, C <= 2) or the VALU, Adam in VGPRs.
#include "mlp_block_util.h"

namespace dct {

namespace blk3 {
constexpr int H = 128, NT = 512, NW = 8, KS = 16, DMAX = 32, B = 4;
constexpr int XT = 0;                     // [3][DMAX][4] input tile, transposed (unit-major, 4 rows)
constexpr int LAB = XT + 3 * DMAX * 4;    // [3][4] labels (int), 16 reserved
constexpr int MSK = LAB + 16;             // [2][NW] uint64: h2 > 0 of (o = 16w + b/4, row b%4)
constexpr int LOGP = MSK + 2 * NW * 2;    // [2][NW][4 rows][4 classes] logit shares
constexpr int H1W = LOGP + 2 * NW * 16;   // [NW][KS][4] wave-private layer-1 inputs h1[k][row]
constexpr int H1X = H1W + NW * KS * 4;    // [NW][4][KS] the same tile transposed (MFMA A operands)
constexpr int PSTR = 36;                  // partials: [o][wave][4] with a 36-float o stride
constexpr int PART = H1X + NW * KS * 4;   // [2][H][PSTR]
constexpr int W2L = PART + 2 * H * PSTR;  // [2][H][4] W2[c][o] (o-major), published by the owners
constexpr int B2L = W2L + 2 * H * 4;      // [2][4] b2
constexpr int TOTAL = B2L + 8;
constexpr int STG = H * H;
constexpr int LDS_FLOATS = TOTAL > 2 * STG ? TOTAL : 2 * STG;  // two staging tiles (prologue/epilogue)
static_assert(LDS_FLOATS * 4 <= 160 * 1024, "fits the CU");
static_assert((H1W % 4) == 0 && (PART % 4) == 0 && (MSK % 4) == 0 && (LAB % 4) == 0 && (W2L % 4) == 0 &&
                  (B2L % 4) == 0 && (H1X % 4) == 0 && (LOGP % 4) == 0,
              "16-B aligned tiles");
using Stg = bku::Stage<H, NT>;
}  // namespace blk3

// PROF (diagnostic instantiation, launched only when MlpArgs::prof is set): lane 0 of every wave
// sums s_memtime deltas per phase into prof[wave * 16 + phase] (tools/prof_block.py)
#define B3STAMP(k)                                              \
  if constexpr (PROF) {                                         \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    pacc[(k)] += t_ - t_last;                                   \
    t_last = t_;                                                \
  }

// ND: input slices per lane (D0 <= 4 * ND); CM: class capacity (2 or 4); ADAM: train mode vs grad
// mode (gradients + loss to grad_out); MF: layer-1 forward and dW1 on the 4x4x1 MFMA; WD: L2 term.
template <int ND, int CM, bool ADAM, bool PROF = false, bool MF = false, bool WD = true>
__global__ __launch_bounds__(blk3::NT, 1) void mlp_block3_kernel(MlpShape sh, MlpArgs a) {
  using namespace blk3;
  using namespace bku;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int D0 = sh.dims[0], C = sh.dims[3];
  const int r0 = l & 3;                 // layer-0 role: row r0, unit u = KS w + l / 4, input slice r0
  const int u = KS * w + (l >> 2);      // ... and the layer-1 role: output o = u, row r0
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
  // W0 slices of unit u (input d = r0 + 4i), b0[u]
  float w0[ND], m0[ND], v0[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) {
    const int d = r0 + 4 * i;
    const bool ok = d < D0;
    const int f = wo0 + u * D0 + (ok ? d : 0);
    w0[i] = ok ? a.p[f] : 0.f;
    m0[i] = (ok && ADAM) ? a.m[f] : 0.f;
    v0[i] = (ok && ADAM) ? a.v[f] : 0.f;
  }
  float pb0 = a.p[bo0 + u], mb0 = ADAM ? a.m[bo0 + u] : 0.f, vb0 = ADAM ? a.v[bo0 + u] : 0.f;
  // W2 column o = u (every lane of the quad holds all CM classes), lane r0 < C owns W2[r0][u]
  // (+ moments); b1[u] in every lane of the quad; b2 owned by wave 0, lane c
  float pw2[CM];
#pragma unroll
  for (int c = 0; c < CM; ++c) pw2[c] = c < C ? a.p[wo2 + c * H + u] : 0.f;
  const bool own_w2 = r0 < C;
  const int fw2 = wo2 + (own_w2 ? r0 : 0) * H + u;
  float mw2 = (own_w2 && ADAM) ? a.m[fw2] : 0.f, vw2 = (own_w2 && ADAM) ? a.v[fw2] : 0.f;
  float pb1 = a.p[bo1 + u], mb1 = ADAM ? a.m[bo1 + u] : 0.f, vb1 = ADAM ? a.v[bo1 + u] : 0.f;
  const bool own_b2 = w == 0 && l < C;  // an old wave: the young half is the step's critical path
  const int fb2 = bo2 + (own_b2 ? l : 0);
  float pb2 = own_b2 ? a.p[fb2] : 0.f, mb2 = (own_b2 && ADAM) ? a.m[fb2] : 0.f, vb2 = (own_b2 && ADAM) ? a.v[fb2] : 0.f;

  // cursor, step counter and the first batch's row indices through the scalar cache: their round
  // trips overlap the W1 loads instead of queueing behind them in vmcnt
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
  float w1[2][KS], m1[2][KS], v1[2][KS];
  Stg::put(lds, sp, tid);
  if (ADAM) Stg::put(lds + STG, sm, tid);
  __syncthreads();
  Stg::get<KS>(lds, w1, l, KS / 4 * w);
  if (ADAM) {
    Stg::get<KS>(lds + STG, m1, l, KS / 4 * w);
    __syncthreads();
    Stg::put(lds, sv, tid);
    __syncthreads();
    Stg::get<KS>(lds, v1, l, KS / 4 * w);
  } else {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int k = 0; k < KS; ++k) m1[j][k] = v1[j][k] = 0.f;
  }
  __syncthreads();  // staging reads done before the tiles (same LDS) are zeroed
  if (tid == 0 && cur0 > 0 && a.loss_out) a.loss_out[cur0 - 1] = a.grad_out[sh.P];

  // ---- LDS: first batch into input buffer 0, W2 / b2 into publish buffer 0
  for (int e = 4 * tid; e < TOTAL; e += 4 * NT) *reinterpret_cast<float4*>(lds + e) = make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();
  if (tid < B * DMAX) lds[XT + (tid >> 2) * 4 + (tid & 3)] = x_first;
  if (tid < B) reinterpret_cast<int*>(lds + LAB)[tid] = lab_first;
  if (own_w2) lds[W2L + u * 4 + r0] = selc<CM>(pw2, r0);  // classes >= C stay 0 (zeroed above)
  if (own_b2) lds[B2L + l] = pb2;
  // prefetch roles: thread -> (row pb, feature pk) of the next batch, or (row pb, label)
  const int nel = Bsz * D0;
  int role = 0, pb = 0, pk = 0;
  if (tid < nel) { role = 1; pb = tid / D0; pk = tid - pb * D0; }
  else if (tid < nel + Bsz) { role = 2; pb = tid - nel; }
  int ridx_next = 0;
  if (role && (cur0 + 1) * Bsz + pb < a.n_items) ridx_next = a.idx[(cur0 + 1) * Bsz + pb];
  // per-thread source of its prefetch element: base + row index * stride (no per-step branch)
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
      for (int k = 0; k < KS; ++k) { m1[j][k] *= rc1; v1[j][k] *= rc2; }
#pragma unroll
    for (int i = 0; i < ND; ++i) { m0[i] *= rc1; v0[i] *= rc2; }
    mb0 *= rc1; vb0 *= rc2; mw2 *= rc1; vw2 *= rc2; mb1 *= rc1; vb1 *= rc2; mb2 *= rc1; vb2 *= rc2;
  }
  float* h1w = lds + H1W + w * (KS * 4);
  float* h1x = lds + H1X + w * (KS * 4);
  int xb = 0;
  // wave priority: the second-dispatched half (waves 4-7) loses VALU arbitration to its SIMD
  // partner and ends up the step's critical path while the older half idles at barrier A
  // (profiles/block3_r3.log); tune 1 raises the young half, 2 the old half (A/B)
  if (a.tune == 1 && w >= NW / 2) __builtin_amdgcn_s_setprio(1);
  if (a.tune == 2 && w < NW / 2) __builtin_amdgcn_s_setprio(1);
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
    const float* xT = lds + XT + xb * DMAX * 4;
    const bool have_next = (s + 1 < a.steps);
    const int bs_next = have_next ? min(Bsz, a.n_items - (sb + 1) * Bsz) : 0;
    const uint32_t raw_next = pf_base[(size_t)ridx_next * pf_stride];
    const int nx2 = min((sb + 2) * Bsz + pb, a.n_items - 1);
    const int ridx_next2 = a.idx[nx2 < 0 ? 0 : nx2];

    // ---- F1: h1[u][r0] (quad all-reduce over the input slices) -> wave-private tile
    float h1;
    {
      // input slices d >= D0 hold zeros in the tile (and zero weights): no guards, no branches
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < ND; ++i) {
        const float4 x = *reinterpret_cast<const float4*>(xT + (r0 + 4 * i) * 4);
        acc[0] += w0[i] * x.x; acc[1] += w0[i] * x.y; acc[2] += w0[i] * x.z; acc[3] += w0[i] * x.w;
      }
      // quad reduce-scatter over the input slices: lane r0 keeps row r0
      const bool qb1 = (r0 >> 1) & 1, qb0 = r0 & 1;
      const float k0 = qb1 ? acc[2] : acc[0], k1 = qb1 ? acc[3] : acc[1];
      const float s0 = qb1 ? acc[0] : acc[2], s1 = qb1 ? acc[1] : acc[3];
      const float e0 = k0 + dpp<QP_X2>(s0), e1 = k1 + dpp<QP_X2>(s1);
      const float kq = qb0 ? e1 : e0, sq = qb0 ? e0 : e1;
      float z = fmaxf(kq + dpp<QP_X1>(sq) + pb0, 0.f);
      if (drop) {
        const uint32_t hsh = mix_hash(a.seed, gstep, (uint32_t)((0 * 64 + r0) * 65536 + u));
        z = (u01(hsh) < p_drop) ? 0.f : z * scale;
      }
      h1 = z;
      h1w[l] = z;  // [k = l / 4][row = l % 4]
      if constexpr (MF) h1x[r0 * KS + (l >> 2)] = z;  // [row][k]
    }
    // layer-1 dropout keep bit of this lane's Phase-1 element (row r0, unit u): hashed off the
    // critical path, while the F2 partials are in flight
    bool keep2 = true;
    if (drop) {
      const uint32_t hsh = mix_hash(a.seed, gstep, (uint32_t)((1 * 64 + r0) * 65536 + u));
      keep2 = u01(hsh) >= p_drop;
    }
    __builtin_amdgcn_wave_barrier();
    B3STAMP(0)
    // ---- F2: this wave's k-slice partials of all 128 outputs x 4 rows
    {
      float acc[2][4] = {};
      if constexpr (MF) {
        // out[o = l + 64j][r] = sum_k h[k][r] W[o][k]: A = h[k][lane % 4] (the transposed tile),
        // B = this lane's own weight, C lands as acc[j][r] of output o = l + 64j
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
          if ((kk & 3) == 0) __builtin_amdgcn_sched_barrier(0);  // bound the hoisted tile loads (VGPRs)
          const float4 h = *reinterpret_cast<const float4*>(h1w + kk * 4);
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            acc[j][0] += w1[j][kk] * h.x; acc[j][1] += w1[j][kk] * h.y;
            acc[j][2] += w1[j][kk] * h.z; acc[j][3] += w1[j][kk] * h.w;
          }
        }
      }
      float* part = lds + PART + pbuf * (H * PSTR);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        *reinterpret_cast<float4*>(part + (l + 64 * j) * PSTR + w * 4) =
            make_float4(acc[j][0], acc[j][1], acc[j][2], acc[j][3]);
    }
    // next batch into the next input buffer (its last readers finished before the previous barrier B)
    if (role) {
      const uint32_t v = (have_next && pb < bs_next) ? raw_next : 0u;
      uint32_t* dst = (role == 1) ? reinterpret_cast<uint32_t*>(lds + XT + xbn * DMAX * 4) + pk * 4 + pb
                                  : reinterpret_cast<uint32_t*>(lds + LAB) + xbn * 4 + pb;
      *dst = v;
    }
    ridx_next = role ? ridx_next2 : 0;
    B3STAMP(1)
    lds_barrier();  // A: all partials of this step are in
    B3STAMP(2)

    // ---- Phase 1: h2[u][r0] of this wave's 16 outputs, its share of the logits, the h2 > 0 mask
    float h2, tsh[CM];
    {
      const float* pr = lds + PART + pbuf * (H * PSTR) + u * PSTR + r0;
      float z = pr[0];
#pragma unroll
      for (int ww = 1; ww < NW; ++ww) z += pr[4 * ww];
      z = fmaxf(z + pb1, 0.f);
      if (drop) z = keep2 ? z * scale : 0.f;
      h2 = z;
#pragma unroll
      for (int c = 0; c < CM; ++c) tsh[c] = sum_bits2to5(pw2[c] * h2);  // lane: row r0's share
      const unsigned long long msk = __ballot(h2 > 0.f);
      if (l < 4) {
        float t4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < CM; ++c) t4[c] = tsh[c];
        *reinterpret_cast<float4*>(lds + LOGP + pbuf * (NW * 16) + w * 16 + l * 4) = make_float4(t4[0], t4[1], t4[2], t4[3]);
      }
      if (l == 0)
        *reinterpret_cast<uint2*>(lds + MSK + pbuf * (NW * 2) + w * 2) = make_uint2((uint32_t)msk, (uint32_t)(msk >> 32));
    }
    B3STAMP(3)
    lds_barrier();  // B: logit shares and masks of every wave are in
    B3STAMP(4)

    // ---- Phase 2: logits (sum of the 8 shares), loss, dlogits (wave-uniform)
    float dz3[4][CM];
    float bl;
    {
      // lane (w' = l / 8, row rr = (l / 2) % 4, class pair cp = l % 2) reads 2 classes of one share
      const int rr = (l >> 1) & 3, cp = l & 1;
      const float2 sh2 = *reinterpret_cast<const float2*>(lds + LOGP + pbuf * (NW * 16) + (l >> 3) * 16 + rr * 4 + 2 * cp);
      float zs[2] = {sh2.x, sh2.y};
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        zs[i] += dpp<ROR8>(zs[i]);   // waves w' and w' ^ 1 (lane bit 3)
        zs[i] = swap16_sum(zs[i], zs[i]);
        zs[i] = swap32_sum(zs[i], zs[i]);
      }
      const float ox0 = dpp<QP_X1>(zs[0]), ox1 = dpp<QP_X1>(zs[1]);  // the other class pair
      const float4 t2 = *reinterpret_cast<const float4*>(lds + B2L + pbuf * 4);
      float z4[4];
      z4[0] = (cp ? ox0 : zs[0]) + t2.x;
      z4[1] = (cp ? ox1 : zs[1]) + t2.y;
      z4[2] = (cp ? zs[0] : ox0) + t2.z;
      z4[3] = (cp ? zs[1] : ox1) + t2.w;
      const int4 labs = *reinterpret_cast<const int4*>(lds + LAB + xb * 4);
      const int lab = (rr & 2) ? ((rr & 1) ? labs.w : labs.z) : ((rr & 1) ? labs.y : labs.x);
      const bool live = rr < bs;
      const float inv = live ? 1.0f / (float)(bs > 0 ? bs : 1) : 0.f;
      float dz[4] = {0.f, 0.f, 0.f, 0.f};
      const LossAcc lr_ = row_loss4(z4, C, lab, a.loss_kind, inv, dz);
      const float lv = live ? lr_.loss : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < CM; ++c) dz3[r][c] = (c < C) ? rl(dz[c], 2 * r) : 0.f;
      const float ltot = rl(lv, 0) + rl(lv, 2) + rl(lv, 4) + rl(lv, 6);
      bl = bs > 0 ? ltot / (float)bs : 0.f;
      if (tid == 0) {
        if (a.loss_out && !a.cursor) a.loss_out[s] = bl;
        if (!ADAM) a.grad_out[sh.P] = bl;
      }
    }
    B3STAMP(5)

    const int t = t0 + s + 1;
    const float step_size = a.lr / (1.f - pow_t(l2b1, (float)t));
    const float rbc2 = __builtin_amdgcn_rsqf(1.f - pow_t(l2b2, (float)t));
    const float rss = __builtin_amdgcn_rcpf(step_size);
    // adam_scaled's folded denominator (moments held as m / (1 - b1), v / (1 - b2))
    const float aA = sqc2 * rbc2 * rss * rc1, aE = a.eps * rss * rc1;
    // ---- dZ2 of every output o = l + 64j (old W2 from LDS, mask bits of the owning wave)
    float dz2[2][4];
    {
      const float* w2p = lds + W2L + pbuf * (H * 4);
      const uint32_t* mk = reinterpret_cast<const uint32_t*>(lds + MSK + pbuf * (NW * 2));
      const int bit = 4 * (l & 15);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int o = l + 64 * j;
        float wv[CM];
        if constexpr (CM == 2) {
          const float2 t = *reinterpret_cast<const float2*>(w2p + o * 4);
          wv[0] = t.x; wv[1 % CM] = t.y;
        } else {
          const float4 t = *reinterpret_cast<const float4*>(w2p + o * 4);
          wv[0] = t.x; wv[1 % CM] = t.y; wv[2 % CM] = t.z; wv[3 % CM] = t.w;
        }
        const uint2 mw = *reinterpret_cast<const uint2*>(mk + 2 * (o >> 4));
        const unsigned long long m64 = ((unsigned long long)mw.y << 32) | mw.x;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float g = 0.f;
#pragma unroll
          for (int c = 0; c < CM; ++c) g += wv[c] * dz3[r][c];
          dz2[j][r] = ((m64 >> (bit + r)) & 1ull) ? g * scale : 0.f;
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
        const float d = selc<4>(col, r0);  // dlogit of (row r0, class c)
        gdz += pw2[c] * d;
        gw2[c] = quad_sum(d * h2);  // dW2[c][u] = sum_r dz3[r][c] h2[u][r]
      }
      gdz = h2 > 0.f ? gdz * scale : 0.f;
      const float gb1 = quad_sum(gdz);
      const float gown = selc<CM>(gw2, r0);
      if (ADAM) {
        float pown = selc<CM>(pw2, r0);
        if (own_w2) adam_scaled<WD>(pown, gown, mw2, vw2, a.b1, a.b2, a.wd, aA, aE);
#pragma unroll
        for (int c = 0; c < CM; ++c) pw2[c] = c < C ? quad_bcast(pown, c) : 0.f;
        adam_scaled<WD>(pb1, gb1, mb1, vb1, a.b1, a.b2, a.wd, aA, aE);
        if (own_w2) lds[W2L + nbuf * (H * 4) + u * 4 + r0] = pown;
      } else {
        if (s == 0) {
          if (own_w2) a.grad_out[fw2] = gown;
          if (r0 == 0) a.grad_out[bo1 + u] = gb1;
        }
        if (own_w2) lds[W2L + nbuf * (H * 4) + u * 4 + r0] = selc<CM>(pw2, r0);
      }
      if (own_b2) {
        float gb = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) gb += CM == 2 ? (l ? dz3[r][1 % CM] : dz3[r][0]) : selc<CM>(dz3[r], l);
        if (ADAM) adam_scaled<WD>(pb2, gb, mb2, vb2, a.b1, a.b2, a.wd, aA, aE);
        else if (s == 0) a.grad_out[fb2] = gb;
        lds[B2L + nbuf * 4 + l] = pb2;
      }
    }
    B3STAMP(6)
    // ---- dZ1 = W1^T dZ2 over this wave's k-slice: one 16-value reduce-scatter per batch row
    // (pass p = row p leaves unit k's sum in lanes 4k..4k+3), lane l keeps pass l & 3 - exactly
    // the (unit, row) whose h1 (and ReLU/dropout mask) it computed in F1
    float dz1 = 0.f;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      float P[16];
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) P[kk] = w1[0][kk] * dz2[0][p] + w1[1][kk] * dz2[1][p];
      const float tot = rs_small<16>(P, l);
      if (r0 == p) dz1 = tot;
    }
    dz1 = h1 > 0.f ? dz1 * scale : 0.f;
    // ---- dW0 / db0: the quad holds unit u's four rows
    {
      float dq[4];
      dq[0] = dpp<QB0>(dz1); dq[1] = dpp<QB1>(dz1); dq[2] = dpp<QB2>(dz1); dq[3] = dpp<QB3>(dz1);
#pragma unroll
      for (int i = 0; i < ND; ++i) {
        const int d = r0 + 4 * i;
        const float4 x = *reinterpret_cast<const float4*>(xT + d * 4);
        const float gw = dq[0] * x.x + dq[1] * x.y + dq[2] * x.z + dq[3] * x.w;
        if (ADAM) adam_scaled<WD>(w0[i], gw, m0[i], v0[i], a.b1, a.b2, a.wd, aA, aE);  // d >= D0: stays 0
        else if (d < D0) a.grad_out[wo0 + u * D0 + d] = gw;
      }
      const float gb = dq[0] + dq[1] + dq[2] + dq[3];
      if (ADAM) adam_scaled<WD>(pb0, gb, mb0, vb0, a.b1, a.b2, a.wd, aA, aE);
      else if (r0 == 0) a.grad_out[bo0 + u] = gb;
    }
    B3STAMP(7)
    // ---- dW1 + Adam in registers
    int gb1 = wo1 + l * H + KS * w;  // grad mode: opaque per step, so 32 store addresses are not hoisted
    if (!ADAM) asm volatile("" : "+v"(gb1));
    if constexpr (MF) {
      // dW1[o = l + 64j][k = 4q + m] = sum_r h1[k][r] dZ2[o][r]: A = h1[4q + lane % 4][r] (one b128 of
      // the tile per q), B = this lane's dZ2, C register m = the gradient of its own w1[j][4q + m]
#pragma unroll
      for (int q = 0; q < KS / 4; ++q) {
        const float4 hq = *reinterpret_cast<const float4*>(h1w + (4 * q + r0) * 4);
        const float hv[4] = {hq.x, hq.y, hq.z, hq.w};
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          f32x4_t g = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int r = 0; r < 4; ++r) g = mfma4(hv[r], dz2[j][r], g);
#pragma unroll
          for (int m = 0; m < 4; ++m) {
            const int kk = 4 * q + m;
            if (ADAM) adam_scaled<WD>(w1[j][kk], g[m], m1[j][kk], v1[j][kk], a.b1, a.b2, a.wd, aA, aE);
            else a.grad_out[gb1 + 64 * j * H + kk] = g[m];
          }
        }
      }
    } else {
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) {
        if ((kk & 3) == 0) __builtin_amdgcn_sched_barrier(0);
        const float4 h = *reinterpret_cast<const float4*>(h1w + kk * 4);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const float gw = dz2[j][0] * h.x + dz2[j][1] * h.y + dz2[j][2] * h.z + dz2[j][3] * h.w;
          if (ADAM) adam_scaled<WD>(w1[j][kk], gw, m1[j][kk], v1[j][kk], a.b1, a.b2, a.wd, aA, aE);
          else a.grad_out[gb1 + 64 * j * H + kk] = gw;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();  // the next step rewrites this wave's h1 tile
    B3STAMP(8)
    xb = xbn;
  }
  if (a.cursor && tid == 0) __hip_atomic_store(a.cursor, cur0 + a.steps, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (a.step_counter && tid == 0)
    __hip_atomic_store(a.step_counter, t0 + a.steps, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (!ADAM) return;

  // ---- write back parameters and moments (flat torch order).  The bases are made opaque so the
  // compiler recomputes these addresses here instead of keeping the prologue's live across the loop.
  int lo = l, uo = u, to = tid;
  asm volatile("" : "+v"(lo), "+v"(uo), "+v"(to));
  // moments back to torch's scale
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int k = 0; k < KS; ++k) { m1[j][k] *= c1; v1[j][k] *= c2; }
#pragma unroll
  for (int i = 0; i < ND; ++i) { m0[i] *= c1; v0[i] *= c2; }
  mb0 *= c1; vb0 *= c2; mw2 *= c1; vw2 *= c2; mb1 *= c1; vb1 *= c2; mb2 *= c1; vb2 *= c2;
  // W1 + moments leave through the same LDS staging as they came in: coalesced 16-byte stores
  __syncthreads();  // every wave is past its last use of the step tiles (the staging aliases them)
  Stg::own<KS>(lds, w1, lo, KS / 4 * w);
  Stg::own<KS>(lds + STG, m1, lo, KS / 4 * w);
  __syncthreads();
  Stg::store(a.p + wo1, lds, to);
  Stg::store(a.m + wo1, lds + STG, to);
  __syncthreads();
  Stg::own<KS>(lds, v1, lo, KS / 4 * w);
  __syncthreads();
  Stg::store(a.v + wo1, lds, to);
#pragma unroll
  for (int i = 0; i < ND; ++i) {
    const int d = r0 + 4 * i;
    if (d < D0) {
      const int f = wo0 + uo * D0 + d;
      a.p[f] = w0[i];
      a.m[f] = m0[i];
      a.v[f] = v0[i];
    }
  }
  if (r0 == 0) {
    a.p[bo0 + uo] = pb0; a.m[bo0 + uo] = mb0; a.v[bo0 + uo] = vb0;
    a.p[bo1 + uo] = pb1; a.m[bo1 + uo] = mb1; a.v[bo1 + uo] = vb1;
  }
  if (own_w2) {
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
#undef B3STAMP

bool mlp_block3_ok(const MlpShape& sh, const MlpArgs& a) {
  if (sh.mlp_block == 0) return false;  // DCT_MLP_BLOCK=0 (plan-time copy): the generic LDS trainer
  // a profiling launch is served for the weather shape (D0 <= 8, C <= 2, train mode) only
  const bool prof_ok = a.prof == nullptr || (sh.dims[0] <= 8 && sh.dims[3] <= 2 && a.mode == 0);
  // 16-byte W1 row loads / stores
  const bool aligned = (sh.woff[1] % 4) == 0 && ((uintptr_t)a.p & 15) == 0 &&
                       (a.mode != 0 || (((uintptr_t)a.m | (uintptr_t)a.v) & 15) == 0);
  return prof_ok && aligned && sh.L == 3 && sh.dims[1] == blk3::H && sh.dims[2] == blk3::H && sh.dims[0] >= 1 &&
         sh.dims[0] <= blk3::DMAX && sh.dims[3] >= 1 && sh.dims[3] <= 4 && a.B >= 1 && a.B <= blk3::B &&
         a.pending == nullptr && a.stage == nullptr && a.xg_world <= 1 && (a.mode == 0 || a.mode == 1);
}

// one launch of an instantiation; its dynamic-LDS limit (two 64-KB staging tiles) is raised once
template <int ND, int CM, bool ADAM, bool PROF = false, bool MF = false, bool WD = true>
static void b3_launch(size_t bytes, hipStream_t st, const MlpShape& sh, const MlpArgs& a) {
  static const hipError_t attr = hipFuncSetAttribute((const void*)mlp_block3_kernel<ND, CM, ADAM, PROF, MF, WD>,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  (void)attr;
  hipLaunchKernelGGL((mlp_block3_kernel<ND, CM, ADAM, PROF, MF, WD>), dim3(1), dim3(blk3::NT), bytes, st, sh, a);
}

hipError_t mlp_launch_block3(const MlpShape& sh, const MlpArgs& a, hipStream_t st) {
  const int d0 = sh.dims[0], C = sh.dims[3];
  const bool tr = a.mode == 0;
  const size_t bytes = (size_t)blk3::LDS_FLOATS * sizeof(float);
  // weather shape (D0 <= 8, C <= 2): layer-1 forward and dW1 on the 4x4x1 fp32 MFMA (the VALU form
  // for other shapes); train mode without weight decay drops the L2 term from every Adam update
  const bool mf = d0 <= 8 && C <= 2;
  const bool wd = a.wd != 0.f;
  const MlpArgs& a2 = a;
  if (a.prof) {
    if (mf) b3_launch<2, 2, true, true, true>(bytes, st, sh, a2);
    else b3_launch<2, 2, true, true>(bytes, st, sh, a2);
  } else if (mf) {
    if (!tr) b3_launch<2, 2, false, false, true>(bytes, st, sh, a2);
    else if (wd) b3_launch<2, 2, true, false, true, true>(bytes, st, sh, a2);
    else b3_launch<2, 2, true, false, true, false>(bytes, st, sh, a2);
  } else {
#define B3K(ND, CM)                                          \
  do {                                                       \
    if (tr) b3_launch<ND, CM, true>(bytes, st, sh, a2);       \
    else b3_launch<ND, CM, false>(bytes, st, sh, a2);         \
  } while (0)
    if (d0 <= 8) {
      if (C <= 2) B3K(2, 2); else B3K(2, 4);
    } else {
      if (C <= 2) B3K(8, 2); else B3K(8, 4);
    }
#undef B3K
  }
  return hipGetLastError();
}

}  // namespace dct
