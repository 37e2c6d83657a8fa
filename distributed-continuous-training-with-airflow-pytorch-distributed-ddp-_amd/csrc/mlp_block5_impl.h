// mlp_block5 device code (the kernel template and its helpers), shared by the two instantiation
// units: mlp_block5.hip (one-rank launches: train, grad mode, profiling) and mlp_block5_xg.hip
// (the data-parallel launches) - separate units so each gets its own code-generation flags
// (_build.py FILE_FLAGS) and they compile in parallel.
#pragma once
// Lean two-barrier trainer for BASELINE's weather MLP exactly: D0 -> 128 -> 128 -> 2 (D0 <= 8,
// batch <= 4, train mode, CE or MSE) - models/mlp.py preset weather-mlp-3x128, the reference's
// WeatherClassifier with a second 128-wide hidden layer (jobs/train_lightning_ddp.py:57-62,69,88,
// 122).  Same contract and work split as mlp_block3.hip (which keeps serving every other shape and
// the grad mode); this one removes latency from the step's serial chain, which the per-phase stamps
// of block3 showed is where the time goes (profiles/block3_r3.log: the loss alone ~1700 cycles per
// wave, the layer-0 forward ~870, the W2 owners ~1780 for a handful of updates):
//   * dropout factors of the NEXT step are hashed during this step's Adam (throughput-bound) instead
//     of heading the layer-0 forward and the h2 reduction;
//   * two-class loss in one lane per (row, class): logits all-reduced over the 8 wave shares with
//     one linear LDS read (lane = wave' * 8 + class * 4 + row) and three cross-lane adds, the other
//     class by one row rotation, softmax as rcp(1 + exp(z_other - z)) - no max / log / division on
//     the path to dlogits (the reported loss is a softplus off that path), no IEEE divisions at all;
//   * every LDS operand of the backward (W2 of the previous publish, b2, labels) is read before
//     barrier B; the W2 owners take dlogit(row, class) from their own lane and one DPP rotation;
//   * the input tile of the layer-0 forward stays in registers for dW0;
//   * W1 Adam pairs its two rows per k (o and o + 64) on one reciprocal: 1/d0 = d1 / (d0 d1).
// Step layout per wave w (8 waves, 2 per SIMD), lane l, unit u = 16 w + l / 4, row r0 = l % 4:
//   F1 (h1[u][r0]) -> F2 k-slice partials (4x4x1 MFMA) -> BARRIER A -> h2 of the wave's 16 outputs,
//   logit shares, h2 > 0 ballot -> BARRIER B -> loss -> dZ2, W2 / b1 / b2 Adam -> dZ1 (reduce-
//   scatter) -> W0 / b0 Adam -> dW1 (MFMA) + W1 Adam.
#include <type_traits>

#include "mlp_block_util.h"

namespace dct {

namespace blk5 {
// B: rows of one micro-batch (the quad's four row lanes); a step of per-rank batch <= 4 MB runs MB of them
constexpr int H = 128, NT = 512, NW = 8, KS = 16, DMAX = 8, B = 4, C = 2, MBMAX = 2, BMAX = B * MBMAX;
constexpr int PSTR = 36;                  // partials: [o][wave][4] with a 36-float o stride
// LDS layout of the MB-micro-batch kernel (MB = 1: batch <= 4, the reference's; MB = 2: batch <= 8)
template <int MB>
struct Lds {
  static constexpr int RB = B * MB;                        // rows of one step
  static constexpr int XT = 0;                             // [3][DMAX][RB] input tiles, feature-major
  static constexpr int LAB = XT + 3 * DMAX * RB;           // [3][RB] labels (int)
  static constexpr int MSK = LAB + (MB == 1 ? 16 : 32);    // [2][NW] uint64: h2 > 0 of (o = 16w + b/4, row b%4)
  static constexpr int LOGP = MSK + 2 * NW * 2;            // [2][NW][C][4] logit shares (wave, class, row)
  static constexpr int H1W = LOGP + 2 * NW * 8;            // [MB][NW][KS][4] wave-private h1[k][row] per micro-batch
  static constexpr int H1X = H1W + MB * NW * KS * 4;       // [NW][4][KS] the same tile transposed (MFMA A operands)
  static constexpr int PART = H1X + NW * KS * 4;           // [2][H][PSTR]
  static constexpr int W2L = PART + 2 * H * PSTR;          // [2][H][C] W2[c][o] (o-major), published by the owners
  static constexpr int B2L = W2L + 2 * H * C;              // [2][4] b2
  static constexpr int ABT = B2L + 8;                      // [4] data-parallel launches: a wave's exchange timed out
  static constexpr int TOTAL = ABT + 4;
  static_assert((H1W % 4) == 0 && (PART % 4) == 0 && (MSK % 4) == 0 && (LAB % 4) == 0 && (W2L % 4) == 0 &&
                    (B2L % 4) == 0 && (H1X % 4) == 0 && (LOGP % 4) == 0,
                "16-B aligned tiles");
};
static_assert(Lds<1>::TOTAL == 11036, "the batch <= 4 layout is round 5's");
constexpr int STG = H * H;
constexpr int LDS_FLOATS = Lds<MBMAX>::TOTAL > 2 * STG ? Lds<MBMAX>::TOTAL : 2 * STG;  // two staging tiles (prologue/epilogue)
static_assert(LDS_FLOATS * 4 <= 160 * 1024, "fits the CU");
using Stg = bku::Stage<H, NT>;
constexpr float LOG2E = 1.4426950408889634f, LN2 = 0.6931471805599453f;
}  // namespace blk5

// ---- data parallelism inside the persistent launch (XW = 2 / 4 / 8 ranks, one per GPU) ---------
// The reference averages every rank's gradients each step (DDP, jobs/train_lightning_ddp.py:136)
// and logs the cross-rank mean loss (sync_dist, :70).  Here that happens in the trainer's own
// launch, over receive buffers every rank maps from its peers (IPC over xGMI, parallel/xgmi.py),
// as a reduce-scatter + all-gather with the optimizer state SHARDED by it (ZeRO-1 style):
//   * every lane holds 16 W1 pairs (rows l, l + 64 x 8 k-pairs of its wave's k-slice, pair
//     i = 8 j + h) and 2 small pairs ({W0[u][r0], W0[u][r0 + 4]}, {W2[r0 & 1][u], its bias: b0[u],
//     b1[u] or b2[l & 1] by r0}); rank i % XW owns W1 pair i of every lane, rank w % XW the small
//     pairs of wave w - so one CU pushes 2 x 16 (XW-1)/XW granules per lane per step instead of
//     16 (XW - 1) for a full all-reduce, and runs 1/XW of the W1 Adam;
//   * RS: each gradient pair is pushed, as it leaves the MFMA, to its owner's slot [src][slot];
//     the owner polls its slots, sums the XW contributions IN RANK ORDER, applies Adam;
//   * AG: the owner pushes the new parameter pair into every peer's slot [pair]; everyone polls
//     the pairs it does not own.  Replicas are bit-identical by construction (one writer each);
//   * the batch loss rides in one granule per rank (rank-ordered mean = sync_dist's);
//   * at launch end the owned Adam moments are all-gathered the same way, so p / m / v in HBM
//     are complete and identical on every rank (checkpoints, resume and fallbacks see one state).
// Granules are 16-B {value, tag, value, tag} write-through stores (the data IS the flag, each
// 8-B half tag-checked); tag = global step + 1, two parity slabs: a rank rewrites a slab of
// step s + 2 only after every peer's step s + 1 granules reached it, i.e. after they finished
// reading step s.  Spins are bounded (xg_timeout): a timeout records the tag in xg_status, the
// workgroup leaves at the next barrier and the launch writes NOTHING back (HBM keeps the state
// the launch started from; the engine re-syncs or raises).
namespace b5x {
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
constexpr int SYS = 17;              // sc0 | sc1: write-through stores, L2-bypassing loads
constexpr int NP = 16, NS = 2;       // W1 pairs / small pairs per lane
constexpr int G = blk5::NT * 16;     // bytes of one slot: one 16-B granule per thread
template <int XW>
struct Lay {
  static constexpr int NO = (NP + XW - 1) / XW;            // W1 pair slots a rank owns per lane (pair
                                                           // XW t + rank; beyond NP when XW does not divide 16)
  static constexpr int RSS = NO + NS;                      // RS slots per (parity, source)
  // RS slots are indexed by the source's distance from the owner, (src - owner) mod XW (1..XW-1),
  // so a rank polls its sources without knowing their absolute index
  static constexpr int AG = 2 * XW * RSS * G;              // [2][NP + NS] all-gather slots
  static constexpr int LS = AG + 2 * (NP + NS) * G;        // [2][XW] loss granules
  static constexpr int EP = LS + ((2 * XW * 16 + 255) & ~255);  // [NP + NS][m, v] launch-end moments
  static constexpr int BYTES = EP + (NP + NS) * 2 * G;
  static __device__ __forceinline__ int rs(int par, int src, int slot) { return ((par * XW + src) * RSS + slot) * G; }
  static __device__ __forceinline__ int ag(int par, int slot) { return AG + (par * (NP + NS) + slot) * G; }
  static __device__ __forceinline__ int ls(int par, int src) { return LS + (par * XW + src) * 16; }
  static __device__ __forceinline__ int ep(int slot, int mv) { return EP + (slot * 2 + mv) * G; }
};
__device__ __forceinline__ void put(__amdgpu_buffer_rsrc_t rs, int off, float x, float y, uint32_t tag) {
  v4u d;
  d.x = __float_as_uint(x);
  d.y = tag;
  d.z = __float_as_uint(y);
  d.w = tag;
  __builtin_amdgcn_raw_buffer_store_b128(d, rs, off, 0, SYS);
}
__device__ __forceinline__ bool get(__amdgpu_buffer_rsrc_t rs, int off, uint32_t tag, float& x, float& y) {
  const v4u d = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, SYS);
  x = __uint_as_float(d.x);
  y = __uint_as_float(d.z);
  return (d.y == tag) & (d.w == tag);
}
// v[XW t + rank] out of v[XW t .. XW t + XW - 1] for a wave-uniform rank: XW - 1 selects on an
// SGPR condition, no branch and no dynamically indexed register
template <int XW, class T>
__device__ __forceinline__ T pick(const T* v, int rank) {
  T r = v[0];
#pragma unroll
  for (int k = 1; k < XW; ++k) r = rank == k ? v[k] : r;
  return r;
}
template <int V>
using IC = std::integral_constant<int, V>;
// f(IC<0>), ..., f(IC<N - 1>)
template <int N, int I = 0, class F>
__device__ __host__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(IC<I>{});
    static_for<N, I + 1>(f);
  }
}
}  // namespace b5x

#define B5STAMP(k)                                              \
  if constexpr (PROF) {                                         \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    pacc[(k)] += t_ - t_last;                                   \
    t_last = t_;                                                \
  }

// dropout factor of element (layer li, row r, unit u) at global step gstep: 0 or 1 / (1 - p).  Same
// bits as mix_hash(seed, gstep, (li * 64 + r) * 65536 + u) (mlp_fused_impl.h), split into the
// wave-uniform step part (scalar ALU), the lane's constant element part (b5_elem, once per launch)
// and the per-element finalizer: two vector multiplies per mask instead of five
__device__ __forceinline__ uint32_t b5_elem(int li, int r, int u) {
  return ((uint32_t)((li * 64 + r) * 65536 + u) + 0x165667B1u) * 0xC2B2AE3Du;
}
__device__ __forceinline__ float b5_drop(uint32_t seed, uint32_t gstep, uint32_t elem, float p, float scale) {
  uint32_t h = (seed * 0x9E3779B1u) ^ ((gstep + 0x7F4A7C15u) * 0x85EBCA77u);
  h ^= elem;
  h ^= h >> 16;
  h *= 0x7feb352du;
  h ^= h >> 15;
  h *= 0x846ca68bu;
  h ^= h >> 16;
  return u01(h) < p ? 0.f : scale;
}

// Adam (scaled moments, bku::adam_scaled) of two parameters sharing one reciprocal
template <bool WD>
__device__ __forceinline__ void adam_pair(float& p0, float g0, float& m0, float& v0, float& p1, float g1, float& m1,
                                          float& v1, float b1, float b2, float wd, float A, float E) {
  if constexpr (WD) { g0 = fmaf(wd, p0, g0); g1 = fmaf(wd, p1, g1); }
  m0 = fmaf(b1, m0, g0);
  m1 = fmaf(b1, m1, g1);
  v0 = fmaf(b2, v0, g0 * g0);
  v1 = fmaf(b2, v1, g1 * g1);
  const float d0 = fmaf(__builtin_amdgcn_sqrtf(v0), A, E), d1 = fmaf(__builtin_amdgcn_sqrtf(v1), A, E);
  const float R = __builtin_amdgcn_rcpf(d0 * d1);
  p0 = fmaf(-m0, d1 * R, p0);
  p1 = fmaf(-m1, d0 * R, p1);
}

// 4x4 transpose across a quad on the 4x4x1 MFMA: lane m holds v[i'] = A[m][i'] -> lane n gets
// A[0..3][n].  Call i' multiplies column i' by the one-hot e[i'] = (lane % 4 == i'), so the products
// land in lane i' only (C[b][m][n] = A[m][i'] delta(n, i')) and 4 accumulating calls assemble the
// transpose exactly (x * 1 + 0); no VALU work.
__device__ __forceinline__ bku::f32x4_t quad_transpose_mf(const float (&v)[4], const float (&e)[4]) {
  bku::f32x4_t t = (bku::f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 4; ++i) t = bku::mfma4(v[i], e[i], t);
  return t;
}

// reduce-scatter of 16 per-lane values over lane bits 2..5 (the 16 lanes sharing lane % 4): lane l
// ends with the sum of value l >> 2.  Levels: bit 5 (permlane32 swap), bit 4 (permlane16 swap),
// bit 3 (row rotation by 8 = lane ^ 8), bit 2 (row rotations by 4 / 12 = lane ^ 4 inside the row).
__device__ __forceinline__ float rs_bits2to5(float (&P)[16], int lane) {
  using namespace bku;
#pragma unroll
  for (int i = 0; i < 8; ++i) P[i] = swap32_sum(P[i], P[i + 8]);
#pragma unroll
  for (int i = 0; i < 4; ++i) P[i] = swap16_sum(P[i], P[i + 4]);
  const bool b3 = (lane >> 3) & 1, b2 = (lane >> 2) & 1;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const float keep = b3 ? P[i + 2] : P[i], send = b3 ? P[i] : P[i + 2];
    P[i] = keep + dpp<ROR8>(send);
  }
  const float keep = b2 ? P[1] : P[0], send = b2 ? P[0] : P[1];
  // lane ^ 4 inside the row: row_ror:N makes lane i read lane (i - N) % 16 (tools/probes/dpp_dir_probe),
  // so lanes with bit 2 clear read i + 4 through row_ror:12, the others i - 4 through row_ror:4
  const float t4 = dpp<ROR4>(send), t12 = dpp<0x12C>(send);
  return keep + (b2 ? t4 : t12);
}

// Adam (scaled moments) of two parameters held as one 64-bit register pair: the moment / parameter
// updates are packed fp32 (v_pk_fma / v_pk_mul: one issue for both lanes of the pair), the two
// square roots scalar, one reciprocal for the pair as in adam_pair
typedef float v2f __attribute__((ext_vector_type(2)));
template <bool WD>
__device__ __forceinline__ void adam_v2(v2f& p, v2f g, v2f& m, v2f& v, float b1, float b2, float wd, float A, float E) {
  if constexpr (WD) g = (v2f)(wd) * p + g;
  m = (v2f)(b1) * m + g;
  v = (v2f)(b2) * v + g * g;
  const v2f sq = (v2f){__builtin_amdgcn_sqrtf(v.x), __builtin_amdgcn_sqrtf(v.y)};
  const v2f d = sq * (v2f)(A) + (v2f)(E);
  const float R = __builtin_amdgcn_rcpf(d.x * d.y);
  p = p - m * ((v2f){d.y, d.x} * R);
}

// MB: micro-batches of B = 4 rows per step (MB = 2: per-rank batch 5..8): every micro-batch runs the
// forward and backward of its four rows on the same lanes (rows r0 + 4 mb), its gradients accumulate
// in registers (dZ2 / the h1 tile stay for the one dW1 pass), the last one applies Adam to the sums.
// LK: 0 = cross-entropy, 1 = MSE against the one-hot label; WD: L2 term in the update; ADAM = false:
// grad mode (the DDP step: ONE step at the device batch cursor, gradients + batch loss to grad_out,
// the previous step's all-reduced loss to loss_out[cursor - 1]; no moments read or written);
// XW > 1: train mode of one rank of XW data-parallel ranks (b5x above); RK >= 0: that rank as a
// compile-time constant (every ownership test folds, the all-gather loads land straight in the W1
// registers; fewer live registers and spills than the runtime-rank kernel, RK = -1)
template <bool WD, int LK, bool PROF = false, bool DXM = true, bool ADAM = true, int XW = 1, int RK = -1, int MB = 1>
__global__ __launch_bounds__(blk5::NT, 1) void mlp_block5_kernel(MlpShape sh, MlpArgs a) {
  using namespace blk5;
  using namespace bku;
  static_assert(XW == 1 || (ADAM && XW >= 2 && XW <= 8), "exchange: train mode, 2..8 ranks");
  static_assert(MB >= 1 && MB <= MBMAX, "micro-batches per step");
  using LY = Lds<MB>;
  constexpr int RB = LY::RB, XT = LY::XT, LAB = LY::LAB, MSK = LY::MSK, LOGP = LY::LOGP, H1W = LY::H1W;
  constexpr int H1X = LY::H1X, PART = LY::PART, W2L = LY::W2L, B2L = LY::B2L, ABT = LY::ABT, TOTAL = LY::TOTAL;
  constexpr int PS = XW > 1 ? 32 : 16;  // PROF: stamp slots per wave (XW > 1: the exchange phases 15..20)
  using XL = b5x::Lay<XW>;
  constexpr int NO = XL::NO;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int D0 = sh.dims[0];
  const int r0 = l & 3;                 // layer-0 / layer-1 role: row r0 of unit u
  const int u = KS * w + (l >> 2);
  const int wo0 = sh.woff[0], bo0 = sh.boff[0], wo1 = sh.woff[1], bo1 = sh.boff[1];
  const int wo2 = sh.woff[2], bo2 = sh.boff[2];
  unsigned long long pacc[PROF ? PS : 1] = {};
  unsigned long long t_last = PROF ? __builtin_amdgcn_s_memtime() : 0ull;
  const unsigned long long t_kstart = t_last;

  // ---- batch indices first: the first batch's row of lane tid < 32 (row fb, feature fd) and the next
  // batch's prefetch element, as VECTOR loads (a scalar load's wait would stall the whole prologue
  // behind it, lgkmcnt is shared with the LDS staging); the dependent X / Y gathers follow the W1 loads
  const int Bsz = a.B;
  const int fb = tid & (RB - 1), fd = tid / RB;  // (RB: a power of two)
  // prefetch roles: thread -> (row pb, feature pk) of the next batch, or (row pb, label)
  const int nel = Bsz * D0;
  int role = 0, pb = 0, pk = 0;
  if (tid < nel) { role = 1; pb = tid / D0; pk = tid - pb * D0; }
  else if (tid < nel + Bsz) { role = 2; pb = tid - nel; }
  // grad mode with a staging buffer (the DDP step path, one launch per step): the previous launch
  // left this launch's batch in a.stage ([0] = batch index + 1, [64 + role slot] = x / label
  // words), so the first batch is one load issued with nothing in front of it instead of the
  // cursor -> idx -> x chain of three dependent round trips
  const bool stp = !ADAM && a.stage != nullptr;
  uint32_t st_tag = 0u, st_x = 0u, st_lab = 0u;
  if (stp) {
    st_tag = a.stage[0];
    if (tid < RB * DMAX && fd < D0 && fb < Bsz) st_x = a.stage[64 + fb * D0 + fd];
    if (tid < Bsz) st_lab = a.stage[64 + nel + tid];
  }
  const int cur0 = (!ADAM && a.cursor) ? sload(a.cursor) : 0;  // grad mode: batch index from the device cursor
  const int bs0 = min(Bsz, a.n_items - cur0 * Bsz);
  const bool first_ok = tid < RB * DMAX && fb < bs0;
  // unconditional load at a clamped index, masked after: a load behind the first_ok branch compiled
  // to a branch with `s_waitcnt vmcnt(0)` inside it - one full memory round trip at kernel start,
  // before a single W1 load was issued
  const int rb_raw = a.idx[max(0, min(cur0 * Bsz + (first_ok ? fb : 0), a.n_items - 1))];
  const int rb_first = (first_ok && !stp) ? rb_raw : 0;
  int ridx_next = 0;
  if (!stp && role && (cur0 + 1) * Bsz + pb < a.n_items) ridx_next = a.idx[(cur0 + 1) * Bsz + pb];

  // ---- W1 + moments: coalesced, redistributed through LDS below
  // (p and m first, v last: the first staging round waits only for the p / m loads - vmcnt counts in
  // issue order - while v is still arriving)
  v4f sp[Stg::LD], sm[Stg::LD], sv[Stg::LD];
#pragma unroll
  for (int i = 0; i < Stg::LD; ++i) {
    const int f = wo1 + 4 * (i * NT + tid);
    sp[i] = *reinterpret_cast<const v4f*>(a.p + f);
    if constexpr (ADAM) sm[i] = *reinterpret_cast<const v4f*>(a.m + f);
  }
  if constexpr (ADAM) {
#pragma unroll
    for (int i = 0; i < Stg::LD; ++i) sv[i] = *reinterpret_cast<const v4f*>(a.v + wo1 + 4 * (i * NT + tid));
  }
  // W0 slices of unit u (inputs d = r0 and r0 + 4), b0[u]
  float w0[2], m0[2], v0[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int d = r0 + 4 * i;
    const bool ok = d < D0;
    const int f = wo0 + u * D0 + (ok ? d : 0);
    w0[i] = ok ? a.p[f] : 0.f;
    m0[i] = (ok && ADAM) ? a.m[f] : 0.f;
    v0[i] = (ok && ADAM) ? a.v[f] : 0.f;
  }
  float pb0 = a.p[bo0 + u], mb0 = ADAM ? a.m[bo0 + u] : 0.f, vb0 = ADAM ? a.v[bo0 + u] : 0.f;
  // W2 column u (both classes in every lane of the quad); lane r0 < 2 owns W2[r0][u] (+ moments);
  // b1[u] in every lane of the quad; b2 owned by wave 0, lanes 0 / 1
  float pw2[C];
#pragma unroll
  for (int c = 0; c < C; ++c) pw2[c] = a.p[wo2 + c * H + u];
  const bool own_w2 = r0 < C;
  // (XW > 1: every lane updates W2[r0 & 1][u] - quad lanes 2 / 3 duplicate lanes 0 / 1)
  const int fw2 = wo2 + (XW > 1 ? (r0 & 1) : (own_w2 ? r0 : 0)) * H + u;
  float mw2 = ((own_w2 || XW > 1) && ADAM) ? a.m[fw2] : 0.f, vw2 = ((own_w2 || XW > 1) && ADAM) ? a.v[fw2] : 0.f;
  float pb1 = a.p[bo1 + u], mb1 = ADAM ? a.m[bo1 + u] : 0.f, vb1 = ADAM ? a.v[bo1 + u] : 0.f;
  const bool own_b2 = w == 0 && l < C;
  const int fb2 = bo2 + (own_b2 ? l : 0);
  float pb2 = own_b2 ? a.p[fb2] : 0.f, mb2 = (own_b2 && ADAM) ? a.m[fb2] : 0.f, vb2 = (own_b2 && ADAM) ? a.v[fb2] : 0.f;
  // XW > 1: the bias this lane updates in its second small pair: b0[u] (r0 0), b1[u] (r0 1), b2[l & 1]
  const int fbx = r0 == 0 ? bo0 + u : (r0 == 1 ? bo1 + u : bo2 + (l & 1));
  float pbx = 0.f, mbx = 0.f, vbx = 0.f;
  if constexpr (XW > 1) {
    pbx = a.p[fbx];
    mbx = a.m[fbx];
    vbx = a.v[fbx];
  }

  // step counter and the first batch's row indices through the scalar cache (their round trips
  // overlap the W1 loads)
  int t0 = a.t0;
  uint32_t step_base = a.step_base;
  if (a.step_counter) {
    t0 = sload(a.step_counter);
    step_base = (uint32_t)t0;
  }
  float x_first = 0.f;
  int lab_first = 0;
  if (stp) {
    // the next batch's indices (its x / label words are fetched in the step and staged for the
    // next launch); issued behind the parameter loads
    if (role && (cur0 + 1) * Bsz + pb < a.n_items) ridx_next = a.idx[(cur0 + 1) * Bsz + pb];
    if ((int)st_tag == cur0 + 1) {  // wave-uniform: staged by the launch before, for this batch
      if (first_ok && fd < D0) x_first = __uint_as_float(st_x);
      if (tid < RB && tid < bs0) lab_first = (int)st_lab;
    } else {  // first launch of a run / after a reset: the gather
      const int rb = first_ok ? a.idx[cur0 * Bsz + fb] : 0;
      if (first_ok && fd < D0) x_first = a.X[(size_t)rb * a.ldx + fd];
      if (tid < RB && tid < bs0) lab_first = a.Y[rb];
    }
  } else {
    if (first_ok && fd < D0) x_first = a.X[(size_t)rb_first * a.ldx + fd];
    if (tid < RB && tid < bs0) lab_first = a.Y[rb_first];  // tid < RB: fb = tid
  }

  // ---- W1 k-slice + moments into registers through the swizzled staging tiles
  float w1[2][KS], m1[2][KS], v1[2][KS];
  if constexpr (PROF) pacc[11] = __builtin_amdgcn_s_memtime() - t_kstart;  // loads issued
  Stg::put(lds, sp, tid);
  if constexpr (ADAM) Stg::put(lds + STG, sm, tid);
  lds_barrier();
  if constexpr (PROF) pacc[12] = __builtin_amdgcn_s_memtime() - t_kstart;  // W1 + m staged
  Stg::get<KS>(lds, w1, l, KS / 4 * w);
  if constexpr (ADAM) {
    Stg::get<KS>(lds + STG, m1, l, KS / 4 * w);
    lds_barrier();
    Stg::put(lds, sv, tid);
    lds_barrier();
    Stg::get<KS>(lds, v1, l, KS / 4 * w);
  } else {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int k = 0; k < KS; ++k) m1[j][k] = v1[j][k] = 0.f;
  }
  lds_barrier();  // staging reads done before the tiles (same LDS) are zeroed
  if constexpr (PROF) pacc[13] = __builtin_amdgcn_s_memtime() - t_kstart;  // all three in registers
  // grad mode: the previous DDP step's all-reduced loss (still in grad_out[P]) to its slot
  if (!ADAM && tid == 0 && cur0 > 0 && a.loss_out) a.loss_out[cur0 - 1] = a.grad_out[sh.P];

  // ---- LDS: first batch into input buffer 0, W2 / b2 into publish buffer 0
  for (int e = 4 * tid; e < TOTAL; e += 4 * NT) *reinterpret_cast<float4*>(lds + e) = make_float4(0.f, 0.f, 0.f, 0.f);
  lds_barrier();
  if (tid < RB * DMAX) lds[XT + fd * RB + fb] = x_first;
  if (tid < RB) reinterpret_cast<int*>(lds + LAB)[tid] = lab_first;
  if (own_w2) lds[W2L + u * C + r0] = r0 ? pw2[1] : pw2[0];
  if (own_b2) lds[B2L + l] = pb2;
  const uint32_t* pf_base = role == 1 ? reinterpret_cast<const uint32_t*>(a.X) + pk : reinterpret_cast<const uint32_t*>(a.Y);
  const int pf_stride = role == 1 ? a.ldx : (role == 2 ? 1 : 0);
  lds_barrier();

  if constexpr (PROF) pacc[14] = __builtin_amdgcn_s_memtime() - t_kstart;  // LDS init + first batch
  // data-parallel launches take these launch constants from the host (kernarg -> scalar registers):
  // derived here, the compiler re-materialises their divisions / logarithms inside the step loop.
  // Measured (profiles/b5_host_constants_ab_r4.log): 8 ranks 17.3 -> 16.4 us/step, but the one-rank
  // kernel 3.90 -> 3.98 us/step despite 7 % fewer loop instructions (its schedule overlaps the
  // re-materialised work with the MFMA chains), so XW = 1 keeps deriving them
  const float p_drop = a.dropout;
  const bool drop = p_drop > 0.f;
  const float scale = XW > 1 ? a.k_drop_scale : (drop ? 1.0f / (1.0f - p_drop) : 1.0f);
  const float l2b1 = XW > 1 ? a.k_l2b1 : log2f(a.b1), l2b2 = XW > 1 ? a.k_l2b2 : log2f(a.b2);
  const float c1 = 1.f - a.b1, c2 = 1.f - a.b2;
  const float rc1 = XW > 1 ? a.k_rc1 : 1.f / c1, rc2 = XW > 1 ? a.k_rc2 : 1.f / c2;
  const float sqc2 = XW > 1 ? a.k_sqc2 : sqrtf(c2);
  // Adam moments to the scaled form adam_scaled keeps (back on store)
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int k = 0; k < KS; ++k) { m1[j][k] *= rc1; v1[j][k] *= rc2; }
#pragma unroll
  for (int i = 0; i < 2; ++i) { m0[i] *= rc1; v0[i] *= rc2; }
  mb0 *= rc1; vb0 *= rc2; mw2 *= rc1; vw2 *= rc2; mb1 *= rc1; vb1 *= rc2; mb2 *= rc1; vb2 *= rc2;
  mbx *= rc1; vbx *= rc2;
  // the step loop keeps W1 and its moments as 64-bit pairs of consecutive k (packed Adam; the dW1 MFMA
  // accumulators come out in the same pairs)
  v2f W[2][KS / 2], Mo[2][KS / 2], Vo[2][KS / 2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int h = 0; h < KS / 2; ++h) {
      W[j][h] = (v2f){w1[j][2 * h], w1[j][2 * h + 1]};
      Mo[j][h] = (v2f){m1[j][2 * h], m1[j][2 * h + 1]};
      Vo[j][h] = (v2f){v1[j][2 * h], v1[j][2 * h + 1]};
    }
  // ---- XW > 1: the moments of the owned W1 pairs only (slot t = pair rank + XW t), the exchange's
  // buffer descriptors, this rank's small-pair ownership
  const int xrank = XW > 1 ? (RK >= 0 ? RK : a.xg_rank) : 0;
  v2f MoO[NO], VoO[NO];
  __amdgpu_buffer_rsrc_t xrr = __builtin_amdgcn_make_buffer_rsrc((void*)a.xg_recv, 0, 0, 0x00020000), xpr[XW];
  // (the wave index through readfirstlane: a scalar condition, uniform branches)
  const bool sown = XW == 1 || (__builtin_amdgcn_readfirstlane(w) % XW) == xrank;
  bool xbad = false;  // this wave's exchange timed out
  unsigned long long xticks = 0;
  if constexpr (XW > 1) {
#pragma unroll
    for (int t = 0; t < NO; ++t) {
      v2f cm[XW], cv[XW];
#pragma unroll
      for (int k = 0; k < XW; ++k) {
        const int i = XW * t + k < b5x::NP ? XW * t + k : 0;  // (slots past pair 15: never used)
        cm[k] = Mo[i >> 3][i & 7];
        cv[k] = Vo[i >> 3][i & 7];
      }
      MoO[t] = b5x::pick<XW>(cm, xrank);
      VoO[t] = b5x::pick<XW>(cv, xrank);
    }
  }
  if constexpr (XW > 1) {
    xrr = __builtin_amdgcn_make_buffer_rsrc((void*)a.xg_recv, 0, XL::BYTES, 0x00020000);
#pragma unroll
    for (int q = 0; q < XW; ++q)
      xpr[q] = __builtin_amdgcn_make_buffer_rsrc((void*)sload_ptr(a.xg_peers, q), 0, XL::BYTES, 0x00020000);
  }
  // bounded spin of one wave until sweep() (this lane's loads of one pass, true when all tags
  // match) holds in every lane; false after xg_timeout (the tag is recorded in xg_status)
  auto xwait = [&](uint32_t tag, auto&& sweep) -> bool {
    const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
    for (int spin = 0;; ++spin) {
      asm volatile("" ::: "memory");  // every pass re-issues its loads
      if (__all(sweep())) return true;
      if ((spin & 15) == 15 && (long long)(__builtin_amdgcn_s_memrealtime() - t_start) > a.xg_timeout) {
        if (l == 0) __hip_atomic_store(a.xg_status, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return false;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  };
  const int tb = tid * 16;  // this thread's granule inside a slot
  // dropout factors of this lane's (row r0 + 4 mb, unit u) elements at the first step
  uint32_t el0[MB], el1[MB];
  float f1[MB], f2[MB];
#pragma unroll
  for (int hf = 0; hf < MB; ++hf) {
    el0[hf] = b5_elem(0, r0 + B * hf, u);
    el1[hf] = b5_elem(1, r0 + B * hf, u);
    f1[hf] = b5_drop(a.seed, step_base, el0[hf], p_drop, scale);
    f2[hf] = b5_drop(a.seed, step_base, el1[hf], p_drop, scale);
  }
  float* h1x = lds + H1X + w * (KS * 4);
  float eye[4];  // one-hot of lane % 4 (B operands of the MFMA quad transposes)
#pragma unroll
  for (int i = 0; i < 4; ++i) eye[i] = r0 == i ? 1.f : 0.f;
  const int cb = (l >> 2) & 1;  // loss role: class cb of row r0 (wave share l / 8)
  int xb = 0;
  if (a.tune == 1 && w >= NW / 2) __builtin_amdgcn_s_setprio(1);
  if (a.tune == 2 && w < NW / 2) __builtin_amdgcn_s_setprio(1);
  if constexpr (PROF) {
    t_last = __builtin_amdgcn_s_memtime();
    pacc[9] = t_last - t_kstart;
  }
  for (int s = 0; s < a.steps; ++s) {
    const int sb = s + cur0;  // batch index (grad mode: at the device cursor)
    const int bs = min(Bsz, a.n_items - sb * Bsz);
    const uint32_t gstep = step_base + (uint32_t)s;
    const int xbn = xb == 2 ? 0 : xb + 1;
    const int pbuf = s & 1, nbuf = pbuf ^ 1;
    const float* xT = lds + XT + xb * DMAX * RB;
    const bool have_next = (s + 1 < a.steps);
    const int bs_next = have_next ? min(Bsz, a.n_items - (sb + 1) * Bsz) : 0;
    const uint32_t raw_next = pf_base[(size_t)ridx_next * pf_stride];
    const int nx2 = min((sb + 2) * Bsz + pb, a.n_items - 1);
    const int ridx_next2 = a.idx[nx2 < 0 ? 0 : nx2];
    const uint32_t xtag = gstep + 1u;  // XW > 1: this step's exchange tag and parity slab
    const int xpar = (int)(gstep & 1u);
    const int t = t0 + s + 1;
    // per micro-batch state that outlives it: dZ2 (the one dW1 pass runs over every micro-batch), and
    // the gradient sums of the small parameters (the last micro-batch applies Adam to them)
    float dz2m[MB][2][4];
    float dz = 0.f, xbl = 0.f, tls = 0.f;  // last micro-batch's dlogit; XW > 1: batch loss; loss sum
    float h2 = 0.f, h1 = 0.f;
    float gw0s = 0.f, gw1s = 0.f, gb1s = 0.f, gbs = 0.f, g0s = 0.f, g1s = 0.f, db0s = 0.f;
    float aA = 0.f, aE = 0.f;
    v2f GO[NO];  // XW > 1 (reduce-scatter): gradients of the W1 pairs this rank owns
#pragma unroll
    for (int t2 = 0; t2 < NO; ++t2) GO[t2] = (v2f){0.f, 0.f};
    float xg_own = 0.f, xg_bx = 0.f;  // XW > 1: this lane's second small gradient pair
    v2f xs_g0 = (v2f){0.f, 0.f}, xs_g1 = (v2f){0.f, 0.f};  // XW > 1: the small gradient pairs
    bool abort_step = false;
    // ---- dW1 pass (see its call sites)
    auto dw1_pass = [&]() {
      // ---- dW1 (MFMA: A = h1[4q + lane % 4][r], B = this lane's dZ2, C register m = the gradient of
      // its own w1[j][4q + m], summed over every micro-batch's rows) + packed Adam on pairs of consecutive k
#pragma unroll
      for (int q = 0; q < KS / 4; ++q) {
        f32x4_t g[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) g[j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int hf = 0; hf < MB; ++hf) {
          const float4 hq = *reinterpret_cast<const float4*>(lds + H1W + (hf * NW + w) * (KS * 4) + (4 * q + r0) * 4);
          const float hv[4] = {hq.x, hq.y, hq.z, hq.w};
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) g[j] = mfma4(hv[r], dz2m[hf][j][r], g[j]);
        }

        if constexpr (ADAM && XW > 1) {
          // pair i = 8 j + 2 q + h to its owner i % XW (slot i / XW there), or kept if owned here
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const int i = 8 * j + 2 * q + h;
              const float gx = g[j][2 * h], gy = g[j][2 * h + 1];
              if ((i % XW) == xrank) GO[i / XW] = (v2f){gx, gy};
              else b5x::put(xpr[i % XW], XL::rs(xpar, (xrank - i % XW + XW) % XW, i / XW) + tb, gx, gy, xtag);
            }
        } else if constexpr (ADAM) {
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int h = 0; h < 2; ++h)
              adam_v2<WD>(W[j][2 * q + h], (v2f){g[j][2 * h], g[j][2 * h + 1]}, Mo[j][2 * q + h], Vo[j][2 * q + h], a.b1,
                          a.b2, a.wd, aA, aE);
        } else {  // dW1[o = l + 64 j][16 w + 4 q .. + 3]: one 16-byte store per (j, q)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            *reinterpret_cast<float4*>(a.grad_out + wo1 + (l + 64 * j) * H + KS * w + 4 * q) =
                make_float4(g[j][0], g[j][1], g[j][2], g[j][3]);
        }
      }
    };

#pragma unroll
    for (int hf = 0; hf < MB; ++hf) {
      const bool last = hf == MB - 1;    // (constant once unrolled)
      const int mpar = MB == 1 ? pbuf : hf;  // PART / LOGP / MSK buffer of this micro-batch
      float* h1w = lds + H1W + (hf * NW + w) * (KS * 4);

      // ---- F1: h1[u][r0] (quad reduce-scatter over the input slices); the tile stays for dW0
      const float4 xa = *reinterpret_cast<const float4*>(xT + r0 * RB + B * hf);
      const float4 xc = *reinterpret_cast<const float4*>(xT + (r0 + 4) * RB + B * hf);
      {
        const float acc0 = w0[0] * xa.x + w0[1] * xc.x, acc1 = w0[0] * xa.y + w0[1] * xc.y;
        const float acc2 = w0[0] * xa.z + w0[1] * xc.z, acc3 = w0[0] * xa.w + w0[1] * xc.w;
        const bool qb1 = (r0 >> 1) & 1, qb0 = r0 & 1;
        const float k0 = qb1 ? acc2 : acc0, k1 = qb1 ? acc3 : acc1;
        const float s0 = qb1 ? acc0 : acc2, s1 = qb1 ? acc1 : acc3;
        const float e0 = k0 + dpp<QP_X2>(s0), e1 = k1 + dpp<QP_X2>(s1);
        const float kq = qb0 ? e1 : e0, sq = qb0 ? e0 : e1;
        h1 = fmaxf(kq + dpp<QP_X1>(sq) + pb0, 0.f) * f1[hf];
        h1w[l] = h1;                    // [k = l / 4][row = l % 4]
        h1x[r0 * KS + (l >> 2)] = h1;   // [row][k]
      }
      __builtin_amdgcn_wave_barrier();
      B5STAMP(0)
      // ---- F2: this wave's k-slice partials of all 128 outputs x 4 rows (4x4x1 MFMA: A = h[k][lane % 4],
      // B = the lane's own weight; C lands as acc[j][row] of output o = l + 64 j)
      {
        // one accumulator per (j, q): chains of 4 dependent MFMAs (40 cycles each) instead of 16
        f32x4_t cq[2][KS / 4];
#pragma unroll
        for (int q = 0; q < KS / 4; ++q) {
          const float4 hq = *reinterpret_cast<const float4*>(h1x + r0 * KS + 4 * q);
          const float hv[4] = {hq.x, hq.y, hq.z, hq.w};
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            cq[j][q] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int e = 0; e < 4; ++e) cq[j][q] = mfma4(hv[e], W[j][2 * q + (e >> 1)][e & 1], cq[j][q]);
          }
        }
        f32x4_t cj[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) cj[j] = (cq[j][0] + cq[j][1]) + (cq[j][2] + cq[j][3]);
        float* part = lds + PART + mpar * (H * PSTR);
#pragma unroll
        for (int j = 0; j < 2; ++j)
          *reinterpret_cast<float4*>(part + (l + 64 * j) * PSTR + w * 4) = make_float4(cj[j][0], cj[j][1], cj[j][2], cj[j][3]);
      }
      if (hf == 0) {
        if (stp) {  // grad mode: hand the next batch to the next launch (tag last, 0 = nothing staged)
          const int bs_st = min(Bsz, a.n_items - (sb + 1) * Bsz);
          if (role) a.stage[64 + tid] = pb < bs_st ? raw_next : 0u;
          if (tid == 0) a.stage[0] = bs_st > 0 ? (uint32_t)(sb + 2) : 0u;
        }
        // next batch into the next input buffer (its last readers finished before the previous barrier B)
        if (role) {
          const uint32_t v = (have_next && pb < bs_next) ? raw_next : 0u;
          uint32_t* dst = (role == 1) ? reinterpret_cast<uint32_t*>(lds + XT + xbn * DMAX * RB) + pk * RB + pb
                                      : reinterpret_cast<uint32_t*>(lds + LAB) + xbn * RB + pb;
          *dst = v;
        }
        ridx_next = role ? ridx_next2 : 0;
      }
      B5STAMP(1)
      lds_barrier();  // A: all partials of this step are in (and W2 / b2 of the previous publish)
      B5STAMP(2)
      if constexpr (XW > 1) {
        // a wave's exchange of the previous step timed out (flag written before this barrier):
        // the whole workgroup leaves together, the epilogue writes nothing back
        if (lds[ABT] != 0.f) {
          abort_step = true;
          break;
        }
      }

      // ---- backward operands published before A: W2 columns l, l + 64 (dZ2), b2 of class cb, the
      // label of row r0 - issued first, consumed after barrier B
      const float2 wv0 = *reinterpret_cast<const float2*>(lds + W2L + pbuf * (H * C) + l * C);
      const float2 wv1 = *reinterpret_cast<const float2*>(lds + W2L + pbuf * (H * C) + (l + 64) * C);
      const float b2c = lds[B2L + pbuf * 4 + cb];
      const int lab = reinterpret_cast<const int*>(lds + LAB)[xb * RB + B * hf + r0];
      // ---- h2[u][r0] of this wave's 16 outputs, its logit shares, the h2 > 0 mask
      {
        const float* pr = lds + PART + mpar * (H * PSTR) + u * PSTR + r0;
        float q[NW];
#pragma unroll
        for (int ww = 0; ww < NW; ++ww) q[ww] = pr[4 * ww];
        const float z = ((q[0] + q[1]) + (q[2] + q[3])) + ((q[4] + q[5]) + (q[6] + q[7]));
        h2 = fmaxf(z + pb1, 0.f) * f2[hf];
        const float t0s = sum_bits2to5(pw2[0] * h2), t1s = sum_bits2to5(pw2[1] * h2);  // row r0's shares
        const unsigned long long msk = __ballot(h2 > 0.f);
        if (l < 8) lds[LOGP + mpar * (NW * 8) + w * 8 + l] = cb ? t1s : t0s;  // [wave][class][row]
        if (l == 0)
          *reinterpret_cast<uint2*>(lds + MSK + mpar * (NW * 2) + w * 2) = make_uint2((uint32_t)msk, (uint32_t)(msk >> 32));
      }
      B5STAMP(3)
      lds_barrier();  // B: logit shares and masks of every wave are in
      B5STAMP(4)

      // ---- loss: lane (share l / 8, class cb, row r0) -> logit (r0, cb) of the micro-batch
      const uint2 mw0 = *reinterpret_cast<const uint2*>(lds + MSK + mpar * (NW * 2) + 2 * (l >> 4));
      const uint2 mw1 = *reinterpret_cast<const uint2*>(lds + MSK + mpar * (NW * 2) + 2 * ((l >> 4) + 4));
      float lv;
      {
        float lg = lds[LOGP + mpar * (NW * 8) + l];
        lg += dpp<ROR8>(lg);          // shares w', w' ^ 1 (lane bit 3)
        lg = swap16_sum(lg, lg);      // lane bit 4
        lg = swap32_sum(lg, lg);      // lane bit 5
        const float z = lg + b2c;
        const float zo = dpp<ROR4>(z);  // the other class of the same row (lane bit 2 flipped in the
                                        // row-replicated copies)
        const bool live = r0 + B * hf < bs;
        const float invb = __builtin_amdgcn_rcpf((float)(bs > 0 ? bs : 1));
        const float inv = live ? invb : 0.f;
        const float y = (cb == lab) ? 1.f : 0.f;
        if constexpr (LK == 0) {
          const float tt = zo - z;
          const float e = __builtin_amdgcn_exp2f(tt * LOG2E);
          const float pc = __builtin_amdgcn_rcpf(1.f + e);  // softmax of class cb
          dz = (pc - y) * inv;
          // row loss (lane of the labelled class): softplus(z_other - z_label), off the dz path
          const float sp = fmaxf(tt, 0.f) + LN2 * __builtin_amdgcn_logf(1.f + __builtin_amdgcn_exp2f(-fabsf(tt) * LOG2E));
          lv = (live && cb == lab) ? sp : 0.f;
        } else {
          const float d = z - y;
          dz = d * inv;               // d (2 / C) / bs
          lv = live ? 0.5f * d * d : 0.f;  // / C
        }
      }
      // dlogits of the micro-batch, wave-uniform: dz3[r][c] lives in lane 4c + r
      float dz3[4][C];
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < C; ++c) dz3[r][c] = rl(dz, 4 * c + r);
      if (w == 0) {  // batch loss: lanes 0..7 hold (class, row) terms
        float tl = lv + dpp<QP_X1>(lv);
        tl += dpp<QP_X2>(tl);
        tl += dpp<ROR4>(tl);
        tls = hf == 0 ? tl : tls + tl;
        if (last) {
          const float bl = bs > 0 ? tls * __builtin_amdgcn_rcpf((float)bs) : 0.f;
          if constexpr (ADAM && XW > 1) {
            // sync_dist: one granule to every peer now, the rank-ordered mean after the all-gather
            xbl = rl(bl, 0);
            if (l == 0) {
#pragma unroll
              for (int q = 0; q < XW; ++q)
                if (q != xrank) b5x::put(xpr[q], XL::ls(xpar, xrank), xbl, 0.f, xtag);
            }
          } else if constexpr (ADAM) {
            if (l == 0 && a.loss_out) a.loss_out[s] = bl;
          } else {
            if (l == 0) a.grad_out[sh.P] = bl;
          }
        }
      }
      B5STAMP(5)

      if (last) {
        const float step_size = a.lr * __builtin_amdgcn_rcpf(1.f - pow_t(l2b1, (float)t));
        const float rbc2 = __builtin_amdgcn_rsqf(1.f - pow_t(l2b2, (float)t));
        const float rss = __builtin_amdgcn_rcpf(step_size);
        aA = sqc2 * rbc2 * rss * rc1;
        aE = a.eps * rss * rc1;
      }
      // ---- dZ2 of outputs o = l + 64 j, the micro-batch's rows (old W2, mask bits of the owning wave)
      {
        const int sh4 = 4 * (l & 15);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const float2 wv = j ? wv1 : wv0;
          const uint2 mw = j ? mw1 : mw0;
          const uint32_t nib = ((sh4 < 32 ? mw.x : mw.y) >> (sh4 & 31)) & 15u;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float g = wv.x * dz3[r][0] + wv.y * dz3[r][1];
            dz2m[hf][j][r] = ((nib >> r) & 1u) ? g * scale : 0.f;
          }
        }
      }
      if constexpr (XW > 1) {
        if (last) {
          dw1_pass();
          B5STAMP(15)  // dW1 MFMA + gradient pushes
        }
      }
      // ---- owners: dW2[:, u], db1[u] (quad sums), W2 / b1 / b2 Adam, W2 / b2 published
      {
        const float d_own = dz, d_oth = dpp<ROR4>(dz);  // dlogit (r0, cb), (r0, 1 - cb)
        const float dr0 = cb ? d_oth : d_own, dr1 = cb ? d_own : d_oth;
        const float gw0 = quad_sum(dr0 * h2), gw1 = quad_sum(dr1 * h2);
        float gdz = pw2[0] * dr0 + pw2[1] * dr1;
        gdz = h2 > 0.f ? gdz * scale : 0.f;
        const float gb1 = quad_sum(gdz);
        const float gbh = (l & 1) ? (dz3[0][1] + dz3[1][1]) + (dz3[2][1] + dz3[3][1])
                                  : (dz3[0][0] + dz3[1][0]) + (dz3[2][0] + dz3[3][0]);
        gw0s = hf == 0 ? gw0 : gw0s + gw0;
        gw1s = hf == 0 ? gw1 : gw1s + gw1;
        gb1s = hf == 0 ? gb1 : gb1s + gb1;
        gbs = hf == 0 ? gbh : gbs + gbh;
        if (last) {
          // updates run in every lane (no control flow around loop-carried registers: a conditional update
          // costs a register copy per value at the loop back edge); only the owners' results are kept
          // (W2[r0][u] is broadcast from quad lanes 0 / 1, b2 published by wave 0's lanes 0 / 1)
          float pown = (r0 & 1) ? pw2[1] : pw2[0];
          const float gown = (r0 & 1) ? gw1s : gw0s;
          const float gb = gbs;
          if constexpr (ADAM && XW > 1) {  // exchanged with the W0 gradients below
            xg_own = gown;
            xg_bx = r0 == 1 ? gb1s : gb;  // (r0 0: db0, known after dZ1)
          } else if constexpr (ADAM) {
            adam_pair<WD>(pown, gown, mw2, vw2, pb1, gb1s, mb1, vb1, a.b1, a.b2, a.wd, aA, aE);
            pw2[0] = dpp<QB0>(pown);
            pw2[1] = dpp<QB1>(pown);
            if (own_w2) lds[W2L + nbuf * (H * C) + u * C + r0] = pown;
            adam_scaled<WD>(pb2, gb, mb2, vb2, a.b1, a.b2, a.wd, aA, aE);
            if (own_b2) lds[B2L + nbuf * 4 + l] = pb2;
          } else {  // grad mode (one step): dW2[r0][u], db1[u], db2 to the flat gradient
            if (own_w2) a.grad_out[fw2] = gown;
            if (r0 == 0) a.grad_out[bo1 + u] = gb1s;
            if (own_b2) a.grad_out[fb2] = gb;
          }
        }
      }
      B5STAMP(6)
      // ---- dZ1 = W1^T dZ2 over this wave's k-slice, lane l keeps its own (unit u, row r0)
      float dz1 = 0.f;
      if constexpr (DXM) {
        // on the 4x4x1 MFMA: each quad's 4x4 blocks of W1 (rows o = 4b + i + 64 j, columns k = 4q + m)
        // and of dZ2 are transposed across the quad (MFMA, exact), so the call index runs over the block's 8
        // outputs and lane (b, n) accumulates sum_o W1[o][4q + m] dZ2[o][n] for m = 0..3; the 16
        // blocks' partials are then reduce-scattered over lane bits 2..5 to lane (b' = k, n)
        float dzt[2][4];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const f32x4_t tq = quad_transpose_mf(dz2m[hf][j], eye);
#pragma unroll
          for (int i = 0; i < 4; ++i) dzt[j][i] = tq[i];
        }
        float P[16];
#pragma unroll
        for (int q = 0; q < KS / 4; ++q) {
          f32x4_t acc[2];  // one chain per j (4 dependent MFMAs each)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const float wq[4] = {W[j][2 * q].x, W[j][2 * q].y, W[j][2 * q + 1].x, W[j][2 * q + 1].y};
            const f32x4_t wt = quad_transpose_mf(wq, eye);
            acc[j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[j] = mfma4(wt[i], dzt[j][i], acc[j]);
          }
          const f32x4_t at = acc[0] + acc[1];
#pragma unroll
          for (int m = 0; m < 4; ++m) P[4 * q + m] = at[m];
        }
        dz1 = rs_bits2to5(P, l);
      } else {
        // one 16-value reduce-scatter per batch row (pass p leaves unit k's sum in lanes 4k..4k+3)
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          float P[16];
#pragma unroll
          for (int kk = 0; kk < KS; ++kk)
            P[kk] = W[0][kk >> 1][kk & 1] * dz2m[hf][0][p] + W[1][kk >> 1][kk & 1] * dz2m[hf][1][p];
          const float tot = rs_small<16>(P, l);
          if (r0 == p) dz1 = tot;
        }
      }
      dz1 = h1 > 0.f ? dz1 * scale : 0.f;
      // ---- dW0 / db0 (the quad holds unit u's four rows; inputs from the F1 tile in registers)
      {
        const float dq0 = dpp<QB0>(dz1), dq1 = dpp<QB1>(dz1), dq2 = dpp<QB2>(dz1), dq3 = dpp<QB3>(dz1);
        const float g0h = dq0 * xa.x + dq1 * xa.y + dq2 * xa.z + dq3 * xa.w;
        const float g1h = dq0 * xc.x + dq1 * xc.y + dq2 * xc.z + dq3 * xc.w;
        const float dbh = (dq0 + dq1) + (dq2 + dq3);
        g0s = hf == 0 ? g0h : g0s + g0h;
        g1s = hf == 0 ? g1h : g1s + g1h;
        db0s = hf == 0 ? dbh : db0s + dbh;
        if (last) {
          const float g0 = g0s, g1 = g1s;
          if constexpr (ADAM && XW > 1) {
            // the two small pairs go to the wave's owner rank now (its Adam runs after the dW1 loop)
            if (r0 == 0) xg_bx = db0s;
            xs_g0 = (v2f){g0, g1};
            xs_g1 = (v2f){xg_own, xg_bx};
            if (!sown) {
#pragma unroll
              for (int q = 0; q < XW; ++q)
                if (q == __builtin_amdgcn_readfirstlane(w) % XW) {  // (scalar: the descriptor stays in SGPRs)
                  const int rel = (xrank - q + XW) % XW;
                  b5x::put(xpr[q], XL::rs(xpar, rel, NO) + tb, g0, g1, xtag);
                  b5x::put(xpr[q], XL::rs(xpar, rel, NO + 1) + tb, xg_own, xg_bx, xtag);
                }
            }
          } else if constexpr (ADAM) {
            adam_pair<WD>(w0[0], g0, m0[0], v0[0], w0[1], g1, m0[1], v0[1], a.b1, a.b2, a.wd, aA, aE);  // d >= D0: stays 0
            adam_scaled<WD>(pb0, db0s, mb0, vb0, a.b1, a.b2, a.wd, aA, aE);
          } else {
            if (r0 < D0) a.grad_out[wo0 + u * D0 + r0] = g0;
            if (r0 + 4 < D0) a.grad_out[wo0 + u * D0 + r0 + 4] = g1;
            if (r0 == 0) a.grad_out[bo0 + u] = db0s;
          }
        }
      }
    }
    if constexpr (XW > 1) {
      if (abort_step) break;
    }
    // next step's dropout factors (independent work for the Adam stream below)
#pragma unroll
    for (int hf = 0; hf < MB; ++hf) {
      f1[hf] = b5_drop(a.seed, gstep + 1u, el0[hf], p_drop, scale);  // p_drop = 0: always 1
      f2[hf] = b5_drop(a.seed, gstep + 1u, el1[hf], p_drop, scale);
    }
    B5STAMP(7)
    // dW1 + packed Adam (one rank) / + reduce-scatter pushes here, after dZ1 and dW0 (XW > 1: issued
    // earlier, right behind dZ2 - its pushes then travel while dZ1 / dW0 compute)
    if constexpr (XW == 1) dw1_pass();
      // ---- the owner's part: reduce-scatter poll, rank-ordered sums, Adam, all-gather pushes;
      // then the all-gather poll of every pair owned elsewhere (specialised per rank: all
      // register indices are constants)
    if constexpr (ADAM && XW > 1) {
      const unsigned long long xt0 = __builtin_amdgcn_s_memrealtime();
      const float invw = 1.f / (float)XW;
      do {
        // reduce-scatter poll: slots of sources at distance 1..XW-1 (the sum starts at the owner's
        // own gradient and follows the ranks after it: a fixed order, so runs are reproducible)
        float rv[XW][NO][2], sv[XW][2][2];
        if (!xwait(xtag, [&]() -> bool {
              bool k = true;
#pragma unroll
              for (int q = 1; q < XW; ++q)
#pragma unroll
                for (int t = 0; t < NO; ++t)
                  k &= b5x::get(xrr, XL::rs(xpar, q, t) + tb, xtag, rv[q][t][0], rv[q][t][1]) | (XW * t + xrank >= b5x::NP);
              return k;
            })) {
          xbad = true;
          break;
        }
        B5STAMP(16)  // reduce-scatter poll wait
        // the small pairs' slots (owner waves only; pushed before the W1 pairs, so normally in):
        // first pass issued here, checked after the W1 Adam - their registers are not in flight
        // together with the W1 slots'
        auto small_sweep = [&]() -> bool {
          bool k = true;
#pragma unroll
          for (int q = 1; q < XW; ++q) {
            k &= b5x::get(xrr, XL::rs(xpar, q, NO) + tb, xtag, sv[q][0][0], sv[q][0][1]);
            k &= b5x::get(xrr, XL::rs(xpar, q, NO + 1) + tb, xtag, sv[q][1][0], sv[q][1][1]);
          }
          return k;
        };
        bool sok = true;
        if (sown) sok = small_sweep();
        // Adam on the owned W1 pairs (slot t = pair XW t + rank), pushed to every peer
        v2f WO[NO];
#pragma unroll
        for (int t = 0; t < NO; ++t) {
          v2f cw[XW];
#pragma unroll
          for (int k = 0; k < XW; ++k) {
            const int i = XW * t + k < b5x::NP ? XW * t + k : 0;
            cw[k] = W[i >> 3][i & 7];
          }
          WO[t] = b5x::pick<XW>(cw, xrank);
          v2f gs = GO[t];
#pragma unroll
          for (int q = 1; q < XW; ++q) gs += (v2f){rv[q][t][0], rv[q][t][1]};
          adam_v2<WD>(WO[t], gs * (v2f)(invw), MoO[t], VoO[t], a.b1, a.b2, a.wd, aA, aE);
          const int agoff = XL::ag(xpar, XW * t + xrank) + tb;
          if (XW * t + xrank < b5x::NP) {
#pragma unroll
            for (int q = 0; q < XW; ++q)
              if (q != xrank) b5x::put(xpr[q], agoff, WO[t].x, WO[t].y, xtag);
          }
        }
        B5STAMP(17)  // owned W1 Adam + all-gather pushes
        if (sown && !__all(sok) && !xwait(xtag, small_sweep)) {
          xbad = true;
          break;
        }
        if (sown) {
          v2f s0 = xs_g0, s1 = xs_g1;
#pragma unroll
          for (int q = 1; q < XW; ++q) {
            s0 += (v2f){sv[q][0][0], sv[q][0][1]};
            s1 += (v2f){sv[q][1][0], sv[q][1][1]};
          }
          s0 *= (v2f)(invw);
          s1 *= (v2f)(invw);
          adam_pair<WD>(w0[0], s0.x, m0[0], v0[0], w0[1], s0.y, m0[1], v0[1], a.b1, a.b2, a.wd, aA, aE);
          float pown = (r0 & 1) ? pw2[1] : pw2[0];
          adam_pair<WD>(pown, s1.x, mw2, vw2, pbx, s1.y, mbx, vbx, a.b1, a.b2, a.wd, aA, aE);
          xs_g1.x = pown;  // the new W2 element (broadcast below)
#pragma unroll
          for (int q = 0; q < XW; ++q)
            if (q != xrank) {
              b5x::put(xpr[q], XL::ag(xpar, b5x::NP) + tb, w0[0], w0[1], xtag);
              b5x::put(xpr[q], XL::ag(xpar, b5x::NP + 1) + tb, pown, pbx, xtag);
            }
        }
        B5STAMP(18)  // small pairs: wait, Adam, all-gather pushes
        // all-gather poll: every pair slot (the owned ones are not checked), the small pairs of a
        // wave owned elsewhere, and in wave 0 the losses (lane q: rank q's)
        float av[b5x::NP][2], sa[2][2], lq = 0.f, lq1;
        const int lsrc = l < XW ? l : 0;
        const bool lskip = w != 0 || l >= XW || l == xrank;
        if (!xwait(xtag, [&]() -> bool {
              bool k = true;
#pragma unroll
              for (int i = 0; i < b5x::NP; ++i)
                k &= b5x::get(xrr, XL::ag(xpar, i) + tb, xtag, av[i][0], av[i][1]) | ((i % XW) == xrank);
              if (!sown) {
                k &= b5x::get(xrr, XL::ag(xpar, b5x::NP) + tb, xtag, sa[0][0], sa[0][1]);
                k &= b5x::get(xrr, XL::ag(xpar, b5x::NP + 1) + tb, xtag, sa[1][0], sa[1][1]);
              }
              if (w == 0) k &= b5x::get(xrr, XL::ls(xpar, lsrc), xtag, lq, lq1) | lskip;
              return k;
            })) {
          xbad = true;
          break;
        }
        B5STAMP(19)  // all-gather poll wait
#pragma unroll
        for (int i = 0; i < b5x::NP; ++i)
          W[i >> 3][i & 7] = (i % XW) == xrank ? WO[i / XW] : (v2f){av[i][0], av[i][1]};
        if (!sown) {
          w0[0] = sa[0][0];
          w0[1] = sa[0][1];
          xs_g1.x = sa[1][0];
          pbx = sa[1][1];
        }
        if (w == 0) {  // sync_dist: the rank-ordered mean of the XW batch losses
          float tot = 0.f;
#pragma unroll
          for (int q = 0; q < XW; ++q) tot += (q == xrank) ? xbl : rl(lq, q);
          if (l == 0 && a.loss_out) a.loss_out[s] = tot * invw;
        }
      } while (false);
      if (xbad) {
        if (l == 0) lds[ABT] = 1.f;  // read by every wave behind the next barrier A
      } else {
        // W2[r0 & 1][u], b0[u], b1[u] to the quad; W2 / b2 published for the next step
        const float pown = xs_g1.x;
        pw2[0] = dpp<QB0>(pown);
        pw2[1] = dpp<QB1>(pown);
        pb0 = dpp<QB0>(pbx);
        pb1 = dpp<QB1>(pbx);
        if (own_w2) lds[W2L + nbuf * (H * C) + u * C + r0] = pown;
        if (w == 0 && (l == 2 || l == 3)) lds[B2L + nbuf * 4 + (l & 1)] = pbx;
      }
      xticks += __builtin_amdgcn_s_memrealtime() - xt0;
      B5STAMP(20)  // all-gather unpack, loss mean, W2 / b2 publish
    }
    __builtin_amdgcn_wave_barrier();  // the next step rewrites this wave's h1 tiles
    B5STAMP(8)
    xb = xbn;
  }

  if constexpr (XW > 1) {
    if (a.xg_ticks && tid == 0) atomicAdd(a.xg_ticks, xticks);
    lds_barrier();
    if (lds[ABT] != 0.f) return;  // an exchange timed out: HBM keeps the launch's starting state
    // ---- all-gather of the owned Adam moments (scaled form on every rank alike), so m / v in HBM
    // are complete on every rank; launch-unique tag (high bit: never a step tag)
    const uint32_t etag = 0x80000000u | (step_base + (uint32_t)a.steps);
    do {
#pragma unroll
      for (int t = 0; t < NO; ++t) {
        const int o0 = XL::ep(XW * t + xrank, 0) + tb, o1 = XL::ep(XW * t + xrank, 1) + tb;
#pragma unroll
        for (int q = 0; q < XW; ++q)
          if (q != xrank && XW * t + xrank < b5x::NP) {
            b5x::put(xpr[q], o0, MoO[t].x, MoO[t].y, etag);
            b5x::put(xpr[q], o1, VoO[t].x, VoO[t].y, etag);
          }
      }
      if (sown) {
#pragma unroll
        for (int q = 0; q < XW; ++q)
          if (q != xrank) {
            b5x::put(xpr[q], XL::ep(b5x::NP, 0) + tb, m0[0], m0[1], etag);
            b5x::put(xpr[q], XL::ep(b5x::NP, 1) + tb, v0[0], v0[1], etag);
            b5x::put(xpr[q], XL::ep(b5x::NP + 1, 0) + tb, mw2, mbx, etag);
            b5x::put(xpr[q], XL::ep(b5x::NP + 1, 1) + tb, vw2, vbx, etag);
          }
      }
      // every moment register is (re)defined on every path, so none of the prologue's full-width
      // moments stays live across the step loop
      float em[b5x::NP][2][2], es[2][2][2];
      const bool ok = xwait(etag, [&]() -> bool {
        bool k = true;
#pragma unroll
        for (int i = 0; i < b5x::NP; ++i) {
          const bool own = (i % XW) == xrank;
          k &= b5x::get(xrr, XL::ep(i, 0) + tb, etag, em[i][0][0], em[i][0][1]) | own;
          k &= b5x::get(xrr, XL::ep(i, 1) + tb, etag, em[i][1][0], em[i][1][1]) | own;
        }
        if (!sown) {
#pragma unroll
          for (int k2 = 0; k2 < 2; ++k2)
#pragma unroll
            for (int mv = 0; mv < 2; ++mv)
              k &= b5x::get(xrr, XL::ep(b5x::NP + k2, mv) + tb, etag, es[k2][mv][0], es[k2][mv][1]);
        }
        return k;
      });
#pragma unroll
      for (int i = 0; i < b5x::NP; ++i) {
        const bool own = (i % XW) == xrank;
        Mo[i >> 3][i & 7] = own ? MoO[i / XW] : (v2f){em[i][0][0], em[i][0][1]};
        Vo[i >> 3][i & 7] = own ? VoO[i / XW] : (v2f){em[i][1][0], em[i][1][1]};
      }
      if (!ok) {
        xbad = true;
        break;
      }
      if (!sown) {
        m0[0] = es[0][0][0]; m0[1] = es[0][0][1];
        v0[0] = es[0][1][0]; v0[1] = es[0][1][1];
        mw2 = es[1][0][0]; mbx = es[1][0][1];
        vw2 = es[1][1][0]; vbx = es[1][1][1];
      }
    } while (false);
    if (xbad) lds[ABT] = 1.f;
    lds_barrier();
    if (lds[ABT] != 0.f) return;
    mbx *= c1;
    vbx *= c2;
  }
  if (a.step_counter && tid == 0)
    __hip_atomic_store(a.step_counter, t0 + a.steps, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if constexpr (!ADAM) {
    if (a.cursor && tid == 0) __hip_atomic_store(a.cursor, cur0 + a.steps, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;  // parameters unchanged
  }

  // ---- write back parameters and moments (flat torch order); opaque bases so the prologue's
  // addresses are recomputed here instead of being kept live across the loop
  int lo = l, uo = u, to = tid;
  asm volatile("" : "+v"(lo), "+v"(uo), "+v"(to));
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int h = 0; h < KS / 2; ++h) {
      w1[j][2 * h] = W[j][h].x; w1[j][2 * h + 1] = W[j][h].y;
      m1[j][2 * h] = Mo[j][h].x; m1[j][2 * h + 1] = Mo[j][h].y;
      v1[j][2 * h] = Vo[j][h].x; v1[j][2 * h + 1] = Vo[j][h].y;
    }
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int k = 0; k < KS; ++k) { m1[j][k] *= c1; v1[j][k] *= c2; }
#pragma unroll
  for (int i = 0; i < 2; ++i) { m0[i] *= c1; v0[i] *= c2; }
  mb0 *= c1; vb0 *= c2; mw2 *= c1; vw2 *= c2; mb1 *= c1; vb1 *= c2; mb2 *= c1; vb2 *= c2;
  lds_barrier();  // every wave is past its last use of the step tiles (the staging aliases them)
  Stg::own<KS>(lds, w1, lo, KS / 4 * w);
  Stg::own<KS>(lds + STG, m1, lo, KS / 4 * w);
  lds_barrier();
  Stg::store(a.p + wo1, lds, to);
  Stg::store(a.m + wo1, lds + STG, to);
  lds_barrier();
  Stg::own<KS>(lds, v1, lo, KS / 4 * w);
  lds_barrier();
  Stg::store(a.v + wo1, lds, to);
  const int r0o = lo & 3;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int d = r0o + 4 * i;
    if (d < D0) {
      const int f = wo0 + uo * D0 + d;
      a.p[f] = w0[i];
      a.m[f] = m0[i];
      a.v[f] = v0[i];
    }
  }
  if constexpr (XW > 1) {  // the second small pair: W2[r0 & 1][u] (lanes 0 / 1) and its bias
    if (r0o < 2 || (w == 0 && (lo == 2 || lo == 3))) {
      a.p[fbx] = pbx; a.m[fbx] = mbx; a.v[fbx] = vbx;
    }
    if (own_w2) {
      const int f = wo2 + r0o * H + uo;
      a.p[f] = (r0o & 1) ? pw2[1] : pw2[0]; a.m[f] = mw2; a.v[f] = vw2;
    }
  } else {
    if (r0o == 0) {
      a.p[bo0 + uo] = pb0; a.m[bo0 + uo] = mb0; a.v[bo0 + uo] = vb0;
      a.p[bo1 + uo] = pb1; a.m[bo1 + uo] = mb1; a.v[bo1 + uo] = vb1;
    }
    if (own_w2) {
      const int f = wo2 + r0o * H + uo;
      a.p[f] = (r0o & 1) ? pw2[1] : pw2[0]; a.m[f] = mw2; a.v[f] = vw2;
    }
    if (own_b2) { a.p[fb2] = pb2; a.m[fb2] = mb2; a.v[fb2] = vb2; }
  }
  if constexpr (PROF) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    pacc[10] = __builtin_amdgcn_s_memtime() - t_last;
    if (l == 0) {
#pragma unroll
      for (int i = 0; i < PS - 1; ++i) atomicAdd(a.prof + w * PS + i, pacc[i]);
    }
  }
}
#undef B5STAMP

// one launch of an instantiation; its dynamic-LDS limit (two 64-KB staging tiles) is raised once
template <bool WD, int LK, bool PROF = false, bool DXM = true, bool ADAM = true, int XW = 1, int RK = -1, int MB = 1>
inline void b5_launch(size_t bytes, hipStream_t st, const MlpShape& sh, const MlpArgs& a) {
  static const hipError_t attr = hipFuncSetAttribute((const void*)mlp_block5_kernel<WD, LK, PROF, DXM, ADAM, XW, RK, MB>,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  (void)attr;
  hipLaunchKernelGGL((mlp_block5_kernel<WD, LK, PROF, DXM, ADAM, XW, RK, MB>), dim3(1), dim3(blk5::NT), bytes, st, sh, a);
}


}  // namespace dct
