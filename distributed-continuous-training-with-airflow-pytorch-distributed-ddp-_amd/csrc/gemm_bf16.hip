// bf16 MFMA GEMM with fused bias/activation epilogue for gfx950.
//
//   C[M,N] (+)= op(A)[M,K] . op(B)[K,N]  (+ bias[N], act)      fp32 accumulate
//   A: trans_a=0 -> stored [M][K] (lda), trans_a=1 -> stored [K][M]
//   B: trans_b=1 -> stored [N][K] (ldb)  (torch Linear weight), trans_b=0 -> stored [K][N]
//
// The three products of a Linear layer map onto it as
//   forward  Y  = X W^T + b  : A=X (0),   B=W (1)   epilogue bias(+relu/gelu), bf16 out (+aux)
//   backward dX = dZ W       : A=dZ (0),  B=W (0)   bf16 out
//   backward dW = dZ^T X     : A=dZ (1),  B=X (0)   fp32 out accumulated into the flat
//                                                    gradient buffer (a DDP bucket view)
//
// Structure (CDNA4 guide §5 "standard MFMA GEMM main loop"): 128x128 block tile, BK=64,
// 256 threads = 4 waves in 2x2, each wave 64x64 = 4x4 tiles of v_mfma_f32_16x16x32_bf16
// (64 fp32 accumulators/lane); LDS images [rows][BK+8] with k contiguous so every A/B
// fragment is one ds_read_b128 (row stride 144 B: the 16 rows of a fragment read land on
// 16 distinct 16-B slots); global->LDS by register staging (16-B loads) double-buffered,
// one barrier per K-step, next tile's loads issued before the current tile's MFMAs.
// Transposed operands are transposed in the staging write (8 x ds_write_b16 per 16-B load).
// Block index -> tile is remapped so blocks sharing an A row-panel run on one XCD (T1).
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include <algorithm>
#include <stdint.h>

#include "dct_common.h"
#include "adam_impl.h"
#include "kernels.h"
#include "knobs.h"

namespace dct {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int GBM = 128, GBN = 128, GBK = 64, GPAD = 8, GLD = GBK + GPAD, GNT = 256;


// Stage one BMxBK (or BNxBK) tile of an operand into registers.
// Non-transposed: chunk c -> row c/8, k-chunk c%8 (8 bf16 each)  [storage [R][K]]
// Transposed:     chunk c -> k c/16, row-chunk c%16               [storage [K][R]]
template <bool TRANS>
__device__ __forceinline__ void stage_load(const uint16_t* __restrict__ G, int ld, int R, int K, int r0, int k0,
                                           bool vec, uint4 (&reg)[4]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = tid + q * GNT;
    int row, kk;
    if (!TRANS) {
      row = r0 + (c >> 3);
      kk = k0 + (c & 7) * 8;
    } else {
      kk = k0 + (c >> 4);
      row = r0 + (c & 15) * 8;
    }
    uint4 v = make_uint4(0, 0, 0, 0);
    if (!TRANS) {
      if (row < R) {
        const uint16_t* src = G + (size_t)row * ld + kk;
        if (vec && kk + 8 <= K) {
          v = *reinterpret_cast<const uint4*>(src);
        } else {
          uint16_t t[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) t[j] = (kk + j < K) ? src[j] : (uint16_t)0;
          v.x = t[0] | ((uint32_t)t[1] << 16); v.y = t[2] | ((uint32_t)t[3] << 16);
          v.z = t[4] | ((uint32_t)t[5] << 16); v.w = t[6] | ((uint32_t)t[7] << 16);
        }
      }
    } else {
      if (kk < K) {
        const uint16_t* src = G + (size_t)kk * ld + row;
        if (vec && row + 8 <= R) {
          v = *reinterpret_cast<const uint4*>(src);
        } else {
          uint16_t t[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) t[j] = (row + j < R) ? src[j] : (uint16_t)0;
          v.x = t[0] | ((uint32_t)t[1] << 16); v.y = t[2] | ((uint32_t)t[3] << 16);
          v.z = t[4] | ((uint32_t)t[5] << 16); v.w = t[6] | ((uint32_t)t[7] << 16);
        }
      }
    }
    reg[q] = v;
  }
}

template <bool TRANS>
__device__ __forceinline__ void stage_store(uint16_t* S, const uint4 (&reg)[4]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = tid + q * GNT;
    if (!TRANS) {
      const int row = c >> 3, kc = (c & 7) * 8;
      *reinterpret_cast<uint4*>(S + row * GLD + kc) = reg[q];
    } else {
      const int kk = c >> 4, r8 = (c & 15) * 8;
      const uint32_t w[4] = {reg[q].x, reg[q].y, reg[q].z, reg[q].w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        S[(r8 + 2 * j) * GLD + kk] = (uint16_t)(w[j] & 0xffff);
        S[(r8 + 2 * j + 1) * GLD + kk] = (uint16_t)(w[j] >> 16);
      }
    }
  }
}

template <bool TA, bool TB>
__global__ __launch_bounds__(GNT, 2) void gemm_bf16_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  // LDS: A[2][GBM][GLD] then B[2][GBN][GLD]
  uint16_t* const As0 = smem;
  uint16_t* const Bs0 = smem + 2 * GBM * GLD;

  // XCD-aware bijective remap: consecutive tiles (same A panel) onto one XCD group
  const int nwg = gridDim.x;
  const int orig = blockIdx.x;
  const int xcd = orig & 7;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int tiles_n = (g.N + GBN - 1) / GBN;
  const int tm = wgid / tiles_n, tn = wgid % tiles_n;
  const int m0 = tm * GBM, n0 = tn * GBN;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = (g.K + GBK - 1) / GBK;
  uint4 ra[4], rb[4];
  stage_load<TA>(g.A, g.lda, g.M, g.K, m0, 0, g.vec_a, ra);
  stage_load<!TB>(g.B, g.ldb, g.N, g.K, n0, 0, g.vec_b, rb);
  stage_store<TA>(As0, ra);
  stage_store<!TB>(Bs0, rb);
  __syncthreads();

  const int frow = lane & 15;
  const int fk = (lane >> 4) * 8;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool has_next = kt + 1 < nk;
    if (has_next) {
      stage_load<TA>(g.A, g.lda, g.M, g.K, m0, (kt + 1) * GBK, g.vec_a, ra);
      stage_load<!TB>(g.B, g.ldb, g.N, g.K, n0, (kt + 1) * GBK, g.vec_b, rb);
    }
    const uint16_t* a_base = As0 + cur * GBM * GLD + (wr * 64 + frow) * GLD + fk;
    const uint16_t* b_base = Bs0 + cur * GBN * GLD + (wc * 64 + frow) * GLD + fk;
#pragma unroll
    for (int ks = 0; ks < GBK / 32; ++ks) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const bf16x8*>(a_base + i * 16 * GLD + ks * 32);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(b_base + j * 16 * GLD + ks * 32);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (has_next) {
      stage_store<TA>(As0 + (cur ^ 1) * GBM * GLD, ra);
      stage_store<!TB>(Bs0 + (cur ^ 1) * GBN * GLD, rb);
    }
    __syncthreads();
  }

  // ---- epilogue: C layout col = lane&15, row = (lane>>4)*4 + r
  const int ccol = lane & 15;
  const int crow = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = n0 + wc * 64 + j * 16 + ccol;
      if (col >= g.N) continue;
      const float bv = (g.bias && g.epilogue >= EPI_BIAS && g.epilogue <= EPI_BIAS_GELU) ? g.bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wr * 64 + i * 16 + crow + r;
        if (row >= g.M) continue;
        float z = acc[i][j][r] * g.alpha + bv;
        const size_t o = (size_t)row * g.ldc + col;
        if (g.residual) z += g.residual[o];
        if (g.aux && g.epilogue == EPI_BIAS_GELU) reinterpret_cast<uint16_t*>(g.aux)[o] = f32_to_bf16(z);
        if (g.epilogue == EPI_BIAS_RELU) z = fmaxf(z, 0.f);
        else if (g.epilogue == EPI_BIAS_GELU) z = gelu_f(z);
        else if (g.epilogue == EPI_RELU_MASK) z = bf16_to_f32(reinterpret_cast<const uint16_t*>(g.aux)[o]) > 0.f ? z : 0.f;
        else if (g.epilogue == EPI_GELU_GRAD) z *= gelu_grad_f(bf16_to_f32(reinterpret_cast<const uint16_t*>(g.aux)[o]));
        if (g.out_f32) {
          float* C = reinterpret_cast<float*>(g.C);
          C[o] = g.accumulate ? C[o] + z : z;
        } else {
          uint16_t* C = reinterpret_cast<uint16_t*>(g.C);
          if (g.accumulate) z += bf16_to_f32(C[o]);
          C[o] = f32_to_bf16(z);
        }
      }
    }
  }
}


// ================================================================== fast path (v2)
// Same tile geometry, but the operands reach LDS by global_load_lds (16-B LDS-DMA, no VGPR
// staging) as verbatim copies of global memory, and transposed operands are transposed by
// the hardware on the way OUT of LDS (ds_read_b64_tr_b16) instead of by 8 ds_write_b16 per
// 16-B chunk on the way in.  Two LDS images:
//   KC ("k contiguous", A row-major / B = W[N][K]): [128 rows][64 k], 16-B chunk c of row r at
//      physical chunk c ^ (r & 7); fragments by ds_read_b128.
//   MC ("rows contiguous", A stored [K][M] / B stored [K][N]): [64 k][128 rows], chunk c of
//      k-row k at c ^ f(k), f(k) = ((k & 3) | ((k >> 1) & 4)) << 1, which spreads the 8 k-rows a
//      32-lane half reads per ds_read_b64_tr_b16 over all 64 banks.
// Split-K (fp32 output, few tiles, e.g. dW = dZ^T X with K = batch): slices accumulate with
// float atomics into C (zeroed by the launcher unless accumulating).
constexpr int G2_BYTES = GBM * GBK * 2;  // one operand image (16 KB)

typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ int mc_swz(int k) { return ((k & 3) | ((k >> 1) & 4)) << 1; }

// one ROWS x KT operand tile -> LDS image (the MC image is 128 wide, KT k-rows of 256 B).  KT = 64:
// row-major (KC) rows of 128 B; KT = 128: rows of 256 B (16 chunks, swizzled by r & 15)
template <bool MC, int ROWS = 128, int NT = 256, int KT = 64>
__device__ __forceinline__ void g2_fill(const uint16_t* __restrict__ G, int ld, int R, int r0, int k0, char* img) {
  static_assert(ROWS == 128 || !MC, "k-major (MC) images are 128 columns wide");
  constexpr int CPR = KT / 8;  // 16-B chunks per KC row
  constexpr int CH = (MC ? KT * 16 : ROWS * CPR) / NT;  // 16-B chunks per thread
  static_assert(CH >= 1 && CH * NT == (MC ? KT * 16 : ROWS * CPR), "whole chunks per thread");
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
#pragma unroll
  for (int q = 0; q < CH; ++q) {
    const int L = q * NT + wave * 64 + lane;  // linear 16-B chunk of the image
    const uint16_t* src;
    if (!MC) {
      const int r = L / CPR, pc = L % CPR;
      const int c = pc ^ (r & (CPR - 1));
      int row = r0 + r;
      row = row < R ? row : R - 1;
      src = G + (size_t)row * ld + k0 + c * 8;
    } else {
      const int k = L >> 4, pc = L & 15;
      const int c = pc ^ mc_swz(k);
      int col = r0 + c * 8;
      col = col + 8 <= R ? col : R - 8;
      src = G + (size_t)(k0 + k) * ld + col;
    }
    // LDS-DMA in inline asm: hipcc would otherwise wait vmcnt(0) before every later ds_read
    // (it cannot prove the DMA does not alias them), serialising the prefetch with the MFMAs.
    // Completion is counted by hand: the k-loop's "s_waitcnt vmcnt(0)" before its barrier.
    const uint32_t dst = __builtin_amdgcn_readfirstlane(
        (uint32_t)(uintptr_t)(lds_void*)(img + (q * NT + wave * 64) * 16));
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(src), "s"(dst)
        : "memory");
  }
}

// The KC fill of g2_fill<false, ROWS, NT, KT> with a row pointer per chunk (rows[q]: the source row
// of this thread's chunk q) - the gathered A operand of dct_gemm_bf16_gather_fwd
template <int ROWS, int NT, int KT, int CH>
__device__ __forceinline__ void g2_fill_rows(const uint16_t* const (&rows)[CH], int k0, char* img) {
  constexpr int CPR = KT / 8;
  static_assert(CH * NT == ROWS * CPR, "whole chunks per thread");
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
#pragma unroll
  for (int q = 0; q < CH; ++q) {
    const int L = q * NT + wave * 64 + lane;
    const int r = L / CPR, pc = L % CPR;
    const uint16_t* src = rows[q] + k0 + (pc ^ (r & (CPR - 1))) * 8;
    const uint32_t dst = __builtin_amdgcn_readfirstlane(
        (uint32_t)(uintptr_t)(lds_void*)(img + (q * NT + wave * 64) * 16));
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(src), "s"(dst)
        : "memory");
  }
}

__device__ __forceinline__ int gather_row(const GatherFwd& ga, int c, int m) {
  int q = c * ga.stride + m;
  q = q < ga.n_items ? q : (ga.n_items > 0 ? q % ga.n_items : 0);
  return ga.idx[q];
}

// 16 x 32 operand fragment (rows rb..rb+15, k-slice ks) in the MFMA A/B layout
template <bool MC, int KT = 64>
__device__ __forceinline__ bf16x8 g2_frag(const char* img, int rb, int ks, int lane) {
  if (!MC) {
    const int row = rb + (lane & 15);
    const int c = ks * 4 + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(img + row * (2 * KT) + ((c ^ (row & (KT / 8 - 1))) << 4));
  } else {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int k = ks * 32 + 8 * g + q;
    const int c = (rb >> 3) + (p >> 1);
    const int k2 = k + 4;
    const char* a0 = img + k * 256 + ((c ^ mc_swz(k)) << 4) + (p & 1) * 8;
    const char* a1 = img + k2 * 256 + ((c ^ mc_swz(k2)) << 4) + (p & 1) * 8;
    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) bf16x4*)(a0));
    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) bf16x4*)(a1));
    bf16x8 r;
    r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
    r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
    return r;
  }
}

// SPLIT: split-K slices reduce with float atomics.  Those keep the MFMA's natural C layout
// (lane = column) so every atomic instruction covers 16 consecutive columns of 4 rows (restaging
// through LDS into 256-byte row runs measured 0-20 % SLOWER on every dW shape:
// profiles/gemm_splitk_lds_restage_ab_r1.log); the
// plain-store kernels swap the MFMA operands instead (lane = row, 4 consecutive columns per
// lane -> 8/16-byte row stores).
// BM = 64: half-height tiles for small-K / few-tile shapes (K <= 256 with M in the tens of
// thousands: the transformer's projections).  Twice the workgroups and half the epilogue per
// thread, and with a single k-tile only one LDS stage (32 KB) -> 4 resident workgroups per CU,
// so one tile's global loads overlap another's epilogue.
// Pipeline depth S (LDS stages of 2 x 16 KB).  With one 128x128 tile per CU (the 4096 x 1024 x 1024
// MLP layers: 256 tiles on 256 CUs) a single wave per SIMD cannot hide an L2/HBM round trip
// behind ONE k-step of MFMAs (~0.2 us), so S = 4 keeps three k-tiles in flight (128 KB LDS, one
// workgroup per CU); grids with several tiles per CU keep S = 2 and hide latency with a second
// resident workgroup.  The prefetch stays in flight ACROSS the k-step barrier: the barrier is a
// raw s_barrier (__syncthreads' fence would emit vmcnt(0) and drain the LDS-DMA queue) preceded
// by a counted vmcnt - every fill issues FILL_OPS loads per thread and loads retire in order, so
// "stage i landed" = at most FILL_OPS x (fills issued after it) still pending.
template <int N>
__device__ __forceinline__ void wait_vm_le() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int FILL_OPS, int S>
__device__ __forceinline__ void wait_stage(int newer_fills) {
  static_assert(S == 2 || S == 4, "pipeline depth 2 or 4");
  if (S == 2 || newer_fills <= 0) wait_vm_le<0>();
  else if (newer_fills == 1) wait_vm_le<FILL_OPS>();
  else wait_vm_le<2 * FILL_OPS>();
}

// workgroup barrier that leaves LDS-DMA loads in flight (this wave's LDS reads retired first)
__device__ __forceinline__ void raw_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// bijective XCD-aware remap: consecutive work ids land on the same XCD (shared L2)
__device__ __forceinline__ int xcd_wgid() {
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
}

// WM: waves along M (2: 256 threads, 2 x 2 waves; 4: 512 threads, 4 x 2 waves - two waves per SIMD
// on a one-tile-per-CU grid, so one wave's LDS reads / waits overlap the other's MFMAs).
// KT: k per LDS stage.  128 (8-wave tiles only): each KC row contributes 256 contiguous bytes per
// stage instead of 128 - the one-tile-per-CU grids are bound by the CU's global -> LDS rate, which the
// longer row segments raise (tools/probes/gemm_probe.hip: 4096 x 1024 x 1024 NT 14.3 -> 12.7 us).
// GA: A is gathered dataset rows (dct_gemm_bf16_gather_fwd, ga: its GatherFwd)
template <bool TA, bool TB, bool SPLIT, int BM, int S, int WM = 2, int KT = 64, bool GA = false>
__device__ __forceinline__ void gemm2_body(const GemmArgs& g, int splits, int wgid, const GatherFwd* ga = nullptr) {
  static_assert(!GA || (!TA && TB && !SPLIT), "gathered A: the forward (NT) kernels");
  static_assert(BM == 128 || (BM == 64 && !TA), "BM = 64 needs a row-major (KC) A image");
  static_assert(WM == 2 || (WM == 4 && BM == 128), "8-wave tiles: 128 x 128");
  static_assert(KT == 64 || (KT == 128 && WM == 4 && S == 2), "128-deep k stages: 8-wave tiles, 2 stages");
  constexpr int IMG = 128 * 2 * KT;  // bytes of one 128-row (or MC 128-column) operand image
  constexpr int NT = 128 * WM;
  constexpr int IM = BM / (16 * WM);  // 16-row MFMA tiles per wave (WM x 2 waves)
  extern __shared__ __attribute__((aligned(16))) char smem2[];
  // [buf][A,B] images of 16 KB each
  constexpr bool AMC = TA, BMC = !TB;
  const int tile = wgid / splits, split = wgid - tile * splits;
  const int tiles_n = (g.N + GBN - 1) / GBN;
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int m0 = tm * BM, n0 = tn * GBN;
  const int nk_all = g.K / KT;
  const int per = (nk_all + splits - 1) / splits;
  const int kt0 = split * per;
  const int kt1 = min(nk_all, kt0 + per);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  f32x4 acc[IM][4];
#pragma unroll
  for (int i = 0; i < IM; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // colsum: one wave column (wc == 0) of the first N tile sums its A rows
  const bool do_cs = g.colsum != nullptr && tn == 0 && wc == 0;
  float cs[IM] = {};
  auto img = [&](int buf, int op) -> char* { return smem2 + (buf * 2 + op) * IMG; };
  // GA: the dataset row of each A chunk this thread loads (the same rows in every k stage)
  constexpr int ACH = GA ? BM * (KT / 8) / NT : 1;
  const uint16_t* arow[ACH];
  int gcur = 0;
  int glab = 0, glab_r = -1;  // GA: this thread's label (row glab_r), loaded before the k loop, stored after
  if constexpr (GA) {
    gcur = ga->cursor[0];
    const int t = wgid * NT + tid;
    if (ga->ydst && t < g.M) {
      glab_r = t;
      glab = ga->Y[gather_row(*ga, gcur, t)];
    }
#pragma unroll
    for (int q = 0; q < ACH; ++q) {
      const int r = (q * NT + tid) / (KT / 8);
      arow[q] = g.A + (size_t)gather_row(*ga, gcur, min(m0 + r, g.M - 1)) * g.lda;
    }
  }
  auto fill = [&](int buf, int kt) {
    const int k0 = kt * KT;
    if constexpr (GA) g2_fill_rows<BM, NT, KT, ACH>(arow, k0, img(buf, 0));
    else if (!TA) g2_fill<false, BM, NT, KT>(g.A, g.lda, g.M, m0, k0, img(buf, 0));
    else g2_fill<true, 128, NT, KT>(g.A, g.lda, g.M, m0, k0, img(buf, 0));
    if (TB) g2_fill<false, 128, NT, KT>(g.B, g.ldb, g.N, n0, k0, img(buf, 1));
    else g2_fill<true, 128, NT, KT>(g.B, g.ldb, g.N, n0, k0, img(buf, 1));
  };
  // global_load_lds per thread per fill (A + B)
  constexpr int FILL_OPS = ((TA ? 16 * KT : BM * KT / 8) + 16 * KT) / NT;
  const int n = kt1 - kt0;
  if (n > 0) {
    // GA: every LDS buffer is filled up front (gathered rows are HBM round trips, not L2 hits: one
    // latency for all the stages that fit instead of one per stage); otherwise S - 1 stages
    constexpr int PRE = GA ? S : S - 1;
#pragma unroll
    for (int s = 0; s < PRE; ++s)
      if (s < n) fill(s, kt0 + s);
    // B^T side output (NT forward GEMMs of the wide MLP): the tiles_m workgroups of one column panel
    // each write a k-slice of its transpose, rows [bt_lo, bt_hi), from the B image of the k-stage that
    // holds them - 16 B per thread (8 columns of one k row), no extra global reads
    int bt_lo = 0, bt_hi = 0;
    if constexpr (TB && !SPLIT) {
      if (g.bt_out) {
        const int tiles_m = (g.M + BM - 1) / BM;
        const int rows_per = (((g.K + tiles_m - 1) / tiles_m) + 31) & ~31;
        bt_lo = min(g.K, tm * rows_per);
        bt_hi = min(g.K, bt_lo + rows_per);
      }
    }
    for (int it = 0; it < n; ++it) {
      wait_stage<FILL_OPS, S>(min(S - 2, n - 1 - it));  // this wave's part of stage `it` has landed
      raw_barrier();  // every wave's part has; every wave finished reading stage it - 1
      if (it + S - 1 < n && it + S - 1 >= PRE) fill((it + S - 1) & (S - 1), kt0 + it + S - 1);  // refill stage it - 1
      const int cur = it & (S - 1);
      const char* ai = img(cur, 0);
      const char* bi = img(cur, 1);
      if constexpr (TB && !SPLIT) {
        const int k0 = (kt0 + it) * KT;
        const int lo = max(bt_lo, k0), hi = min(bt_hi, k0 + KT);
        constexpr int RPP = NT / 16;  // k rows per pass (16 threads of 8 columns = one 128-wide row)
        for (int kb = lo; kb < hi; kb += RPP) {
          const int kl = kb + (tid >> 4), ng = tid & 15;
          const int col = n0 + ng * 8;
          if (kl < hi && col + 8 <= g.N) {
            const int kk = kl - k0;
            uint32_t w[4];
#pragma unroll
            for (int e = 0; e < 8; e += 2) {
              const int r0 = ng * 8 + e, r1 = r0 + 1;
              const uint16_t lo16 = *reinterpret_cast<const uint16_t*>(
                  bi + r0 * (2 * KT) + (((kk >> 3) ^ (r0 & (KT / 8 - 1))) << 4) + (kk & 7) * 2);
              const uint16_t hi16 = *reinterpret_cast<const uint16_t*>(
                  bi + r1 * (2 * KT) + (((kk >> 3) ^ (r1 & (KT / 8 - 1))) << 4) + (kk & 7) * 2);
              w[e >> 1] = (uint32_t)lo16 | ((uint32_t)hi16 << 16);
            }
            *reinterpret_cast<uint4*>(g.bt_out + (size_t)kl * g.bt_ld + col) = make_uint4(w[0], w[1], w[2], w[3]);
          }
        }
      }
      if constexpr (GA) {
        // the gathered rows for the dW GEMM, from the A image of this k stage: the tiles_n workgroups
        // of a row panel each write a band of its rows, 16 B per thread
        if (ga->a_out) {
          constexpr int CPR = KT / 8, RPP = NT / CPR;
          const int k0 = (kt0 + it) * KT;
          const int band = (BM + tiles_n - 1) / tiles_n;
          const int lo = min(BM, tn * band), hi = min(BM, lo + band);
          for (int rb = lo; rb < hi; rb += RPP) {
            const int rr = rb + tid / CPR, cc = tid % CPR;
            if (rr < hi && m0 + rr < g.M)
              *reinterpret_cast<uint4*>(ga->a_out + (size_t)(m0 + rr) * g.K + k0 + cc * 8) =
                  *reinterpret_cast<const uint4*>(ai + rr * (2 * KT) + ((cc ^ (rr & (CPR - 1))) << 4));
          }
        }
      }
#pragma unroll
      for (int ks = 0; ks < KT / 32; ++ks) {
        bf16x8 af[IM], bfr[4];
#pragma unroll
        for (int i = 0; i < IM; ++i) af[i] = g2_frag<AMC, KT>(ai, wr * (BM / WM) + i * 16, ks, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) bfr[j] = g2_frag<BMC, KT>(bi, wc * 64 + j * 16, ks, lane);
        if (do_cs) {  // fused bias gradient: row sums of the A fragments (lane: 8 k of row l&15)
#pragma unroll
          for (int i = 0; i < IM; ++i)
#pragma unroll
            for (int e = 0; e < 8; ++e) cs[i] += bf16_to_f32((uint16_t)af[i][e]);
        }
#pragma unroll
        for (int i = 0; i < IM; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = SPLIT ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0)
                              : __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
      }
    }
  }
  if constexpr (GA) {
    // the rest of the step prologue, after the k loop (its loads drained, so these waits cover only
    // themselves), spread over the grid: labels, the Adam step counter, the gradient ranges to clear
    const int nwg = ((g.M + BM - 1) / BM) * tiles_n;
    const int t = wgid * NT + tid, nt = nwg * NT;
    if (t == 0 && ga->step_counter) ga->step_counter[0] += 1;
    if (glab_r >= 0) ga->ydst[glab_r] = glab;
    if (ga->ydst)
      for (int r = t + nt; r < g.M; r += nt) ga->ydst[r] = ga->Y[gather_row(*ga, gcur, r)];
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // (constant indices into the kernel argument)
      if (q >= ga->nz) break;
      float* z = ga->zero + ga->zoff[q];
      const int64_t n = ga->zcnt[q], n4 = n >> 2;
      for (int64_t i = t; i < n4; i += nt) reinterpret_cast<float4*>(z)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (t < n - (n4 << 2)) z[(n4 << 2) + t] = 0.f;
    }
  }
  if (do_cs) {  // lanes l, l+16, l+32, l+48 hold partial sums of the same row
#pragma unroll
    for (int i = 0; i < IM; ++i) {
      float v = cs[i];
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      const int row = m0 + wr * (BM / WM) + i * 16 + (lane & 15);
      if (lane < 16 && row < g.M) atomicAdd(g.colsum + row, v);
    }
  }
  // ---- epilogue.  The MFMAs ran with swapped operands (B fragment first), so each 16x16
  // accumulator is the TRANSPOSED tile: lane (c = lane&15, g = lane>>4) holds row 16i + c and the
  // 4 CONSECUTIVE columns 16j + 4g .. +3 -> 8-byte bf16 / 16-byte fp32 row stores instead of
  // 2-byte scattered ones (and 4-wide bias / aux loads).
  if (SPLIT && g.split_part) {  // two-pass split-K: this slice's partial tile, plain stores
    float* part = g.split_part + (size_t)split * g.M * g.N;
    const int col_l = lane & 15, row_l = (lane >> 4) * 4;
#pragma unroll
    for (int i = 0; i < IM; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = n0 + wc * 64 + j * 16 + col_l;
        if (col >= g.N) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = m0 + wr * (BM / WM) + i * 16 + row_l + r;
          if (row < g.M) part[(size_t)row * g.N + col] = acc[i][j][r];
        }
      }
    return;
  }
  if (SPLIT) {  // natural layout: col = lane&15, rows 4*(lane>>4) + r
    const int col_l = lane & 15, row_l = (lane >> 4) * 4;
#pragma unroll
    for (int i = 0; i < IM; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = n0 + wc * 64 + j * 16 + col_l;
        if (col >= g.N) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = m0 + wr * (BM / WM) + i * 16 + row_l + r;
          if (row < g.M) {
            float* dst = reinterpret_cast<float*>(g.C) + (size_t)row * g.ldc + col;
            atomicAdd(dst, acc[i][j][r] * g.alpha);
          }
        }
      }
    return;
  }
  const int c16 = lane & 15;
  const int g4 = (lane >> 4) * 4;
  const bool bias_epi = g.bias && g.epilogue >= EPI_BIAS && g.epilogue <= EPI_BIAS_GELU;
  const bool vec_ok = (g.ldc % 4 == 0) && ((((uintptr_t)g.C) & 15) == 0) &&
                      (!g.aux || (((uintptr_t)g.aux) & 7) == 0);
#pragma unroll
  for (int i = 0; i < IM; ++i) {
    const int row = m0 + wr * (BM / WM) + i * 16 + c16;
    if (row >= g.M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col0 = n0 + wc * 64 + j * 16 + g4;
      if (col0 >= g.N) continue;
      const size_t o0 = (size_t)row * g.ldc + col0;
      const bool full = vec_ok && col0 + 4 <= g.N;
      float z[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) z[r] = acc[i][j][r] * g.alpha;
      if (bias_epi) {
        if (full) {
          const float4 bv = *reinterpret_cast<const float4*>(g.bias + col0);
          z[0] += bv.x; z[1] += bv.y; z[2] += bv.z; z[3] += bv.w;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) z[r] += (col0 + r < g.N) ? g.bias[col0 + r] : 0.f;
        }
      }
      if (g.residual) {
        const float* R = g.residual + o0;
        if (full) {
          const float4 rv = *reinterpret_cast<const float4*>(R);
          z[0] += rv.x; z[1] += rv.y; z[2] += rv.z; z[3] += rv.w;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) z[r] += (col0 + r < g.N) ? R[r] : 0.f;
        }
      }
      uint16_t* aux16 = reinterpret_cast<uint16_t*>(g.aux);
      if (g.epilogue == EPI_BIAS_GELU && aux16) {  // keep the pre-activation for GELU'
        if (full) {
          uint2 pk;
          pk.x = f32_to_bf16(z[0]) | ((uint32_t)f32_to_bf16(z[1]) << 16);
          pk.y = f32_to_bf16(z[2]) | ((uint32_t)f32_to_bf16(z[3]) << 16);
          *reinterpret_cast<uint2*>(aux16 + o0) = pk;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (col0 + r < g.N) aux16[o0 + r] = f32_to_bf16(z[r]);
        }
      }
      if (g.epilogue == EPI_RELU_MASK || g.epilogue == EPI_GELU_GRAD) {
        float a[4];
        if (full) {
          const uint2 pk = *reinterpret_cast<const uint2*>(aux16 + o0);
          a[0] = bf16_to_f32(pk.x & 0xffff); a[1] = bf16_to_f32(pk.x >> 16);
          a[2] = bf16_to_f32(pk.y & 0xffff); a[3] = bf16_to_f32(pk.y >> 16);
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) a[r] = (col0 + r < g.N) ? bf16_to_f32(aux16[o0 + r]) : 0.f;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r)
          z[r] = g.epilogue == EPI_RELU_MASK ? (a[r] > 0.f ? z[r] : 0.f) : z[r] * gelu_grad_f(a[r]);
      } else if (g.epilogue == EPI_BIAS_RELU) {
#pragma unroll
        for (int r = 0; r < 4; ++r) z[r] = fmaxf(z[r], 0.f);
      } else if (g.epilogue == EPI_BIAS_GELU) {
#pragma unroll
        for (int r = 0; r < 4; ++r) z[r] = gelu_f(z[r]);
      }
      if (g.out_f32) {
        float* C = reinterpret_cast<float*>(g.C) + o0;
        if (full) {
          float4 v = make_float4(z[0], z[1], z[2], z[3]);
          if (g.accumulate) {
            const float4 c0 = *reinterpret_cast<const float4*>(C);
            v.x += c0.x; v.y += c0.y; v.z += c0.z; v.w += c0.w;
          }
          *reinterpret_cast<float4*>(C) = v;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (col0 + r < g.N) C[r] = g.accumulate ? C[r] + z[r] : z[r];
        }
      } else {
        uint16_t* C = reinterpret_cast<uint16_t*>(g.C) + o0;
        if (full) {
          if (g.accumulate) {
            const uint2 c0 = *reinterpret_cast<const uint2*>(C);
            z[0] += bf16_to_f32(c0.x & 0xffff); z[1] += bf16_to_f32(c0.x >> 16);
            z[2] += bf16_to_f32(c0.y & 0xffff); z[3] += bf16_to_f32(c0.y >> 16);
          }
          uint2 pk;
          pk.x = f32_to_bf16(z[0]) | ((uint32_t)f32_to_bf16(z[1]) << 16);
          pk.y = f32_to_bf16(z[2]) | ((uint32_t)f32_to_bf16(z[3]) << 16);
          *reinterpret_cast<uint2*>(C) = pk;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (col0 + r < g.N) C[r] = f32_to_bf16((g.accumulate ? bf16_to_f32(C[r]) : 0.f) + z[r]);
        }
      }
    }
  }
}

template <bool TA, bool TB, bool SPLIT, int BM = 128, int S = 2, int WM = 2, int KT = 64>
__global__ __launch_bounds__(128 * WM, WM == 4 ? 2 : (BM == 64 ? 4 : 2)) void gemm2_kernel(GemmArgs g, int splits) {
  gemm2_body<TA, TB, SPLIT, BM, S, WM, KT>(g, splits, xcd_wgid());
}

// the wide-MLP step's first forward GEMM with the batch gather folded in (GatherFwd, kernels.h)
template <int BM, int S, int WM, int KT>
__global__ __launch_bounds__(128 * WM, WM == 4 ? 2 : 2) void gemm2_gather_kernel(GemmArgs g, GatherFwd ga) {
  gemm2_body<false, true, false, BM, S, WM, KT, true>(g, 1, xcd_wgid(), &ga);
}

// Grouped split-K launch: up to DW_GROUP independent problems (the dW GEMMs of one transformer
// block, or of every block when the backward defers them to its end) in ONE grid, so the
// per-launch fixed cost (ramp, first-load latency, tail) is paid once.
constexpr int DW_GROUP = 16;
// Optional work riding in a grouped dW launch: the TabTransformer feature-token embedding's parameter
// gradients (csrc/tt_io.hip embed_bwd_kernel) - batch sums over the first block's dh, which the
// autograd order puts right before this launch.  One extra workgroup per feature (F of them fit the
// slots the GEMM grid leaves free: 448 of 512 at the bench shape), 8 sample slots x 64 dimensions,
// one writer per gradient element (no atomics): the separate kernel and its boundary go away.
struct EmbedRide {
  const float* x;   // [B][F] features (null: no ride)
  const float* dh;  // [B][F][64]
  float* dE; float* dc;  // [F][64], accumulated
  int B, F;
};
struct GemmGroup {
  GemmArgs g[DW_GROUP];
  int splits[DW_GROUP];
  int start[DW_GROUP + 1];  // first work id of each problem; start[n] = total
  int n;
  EmbedRide er;
};

__device__ __forceinline__ void embed_ride(const EmbedRide& e, int f, float* sm) {
  const int s = threadIdx.x >> 6, d = threadIdx.x & 63, ns = blockDim.x >> 6;
  float aw = 0.f, ab = 0.f;
  for (int b = s; b < e.B; b += ns) {
    const size_t tok = (size_t)b * e.F + f;
    const float g = e.dh[tok * 64 + d];
    aw = fmaf(e.x[tok], g, aw);
    ab += g;
  }
  sm[s * 64 + d] = aw;
  sm[(ns + s) * 64 + d] = ab;
  __syncthreads();
  if (threadIdx.x < 128) {
    const int which = threadIdx.x >> 6;
    float v = 0.f;
    for (int q = 0; q < ns; ++q) v += sm[(which * ns + q) * 64 + d];
    float* dst = (which ? e.dc : e.dE) + (size_t)f * 64 + d;
    *dst += v;
  }
}

template <bool TA, bool TB, int S, int WM = 2>
__global__ __launch_bounds__(128 * WM, 2) void gemm2_grouped_kernel(GemmGroup gg) {
  const int w = xcd_wgid();
  if (gg.er.x && w >= gg.start[gg.n]) {  // riding embedding-gradient workgroup
    extern __shared__ __attribute__((aligned(16))) char smem_er[];
    embed_ride(gg.er, w - gg.start[gg.n], reinterpret_cast<float*>(smem_er));
    return;
  }
  int p = 0;
#pragma unroll
  for (int i = 1; i < DW_GROUP; ++i) p += (i < gg.n && w >= gg.start[i]) ? 1 : 0;
  gemm2_body<TA, TB, true, 128, S, WM>(gg.g[p], gg.splits[p], w - gg.start[p]);
}

// zero the fp32 C[M, ldc] panel that split-K slices accumulate into (a kernel node, not a
// hipMemset2DAsync node: see gather_batch_kernel on memset nodes in replayed graphs)
__global__ __launch_bounds__(256) void zero_panel_kernel(float* __restrict__ C, int ldc, int M, int N) {
  const int64_t total = (int64_t)M * N;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / N;
    C[r * ldc + (e - r * N)] = 0.f;
  }
}

// Second pass of the two-pass split-K: C[r][c] (+)= alpha * sum_s part[s][r][c], slices summed in
// order (bit-reproducible), 4 columns per thread when N % 4 == 0.  Replaces `splits` fp32 atomics per
// output element: on the 1024 x 1024 x 4096 dW each slice's 1 M atomics cost ~3.4 us
// (profiles/gemm_splitk_sweep_*), the partials one streaming read.
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ part, int splits, float* C,
                                                           int ldc, int M, int N, int accumulate, float alpha) {
  const size_t MN = (size_t)M * N;
  if ((N & 3) == 0) {
    const int64_t total = (int64_t)(MN >> 2);
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
      float4 s = reinterpret_cast<const float4*>(part)[e];
      for (int q = 1; q < splits; ++q) {
        const float4 v = reinterpret_cast<const float4*>(part + (size_t)q * MN)[e];
        s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
      }
      const int64_t f = e * 4;
      const int64_t r = f / N;
      float* dst = C + r * ldc + (f - r * N);
      if (accumulate) {
        dst[0] += alpha * s.x; dst[1] += alpha * s.y; dst[2] += alpha * s.z; dst[3] += alpha * s.w;
      } else {
        dst[0] = alpha * s.x; dst[1] = alpha * s.y; dst[2] = alpha * s.z; dst[3] = alpha * s.w;
      }
    }
    return;
  }
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < (int64_t)MN; e += (int64_t)gridDim.x * blockDim.x) {
    float s = part[e];
    for (int q = 1; q < splits; ++q) s += part[(size_t)q * MN + e];
    const int64_t r = e / N;
    float* dst = C + r * ldc + (e - r * N);
    *dst = accumulate ? *dst + alpha * s : alpha * s;
  }
}

// the same second pass for a grouped launch: problem p owns float4 elements [start[p], start[p+1])
struct SplitRedGroup {
  const float* part[DW_GROUP];
  float* C[DW_GROUP];
  int N[DW_GROUP], splits[DW_GROUP];
  int64_t MN[DW_GROUP];
  int64_t start[DW_GROUP + 1];
  int n, accumulate;
};

__global__ __launch_bounds__(256) void splitk_reduce_grouped_kernel(SplitRedGroup r) {
  const int64_t total = r.start[r.n];
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    int p = 0;
#pragma unroll
    for (int i = 1; i < DW_GROUP; ++i) p += (i < r.n && e >= r.start[i]) ? 1 : 0;
    const int64_t q4 = e - r.start[p];
    const float* part = r.part[p];
    float4 s = reinterpret_cast<const float4*>(part)[q4];
    for (int q = 1; q < r.splits[p]; ++q) {
      const float4 v = reinterpret_cast<const float4*>(part + (size_t)q * r.MN[p])[q4];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    float4* dst = reinterpret_cast<float4*>(r.C[p]) + q4;  // C_i is [M_i][N_i] contiguous (ldc = N_i)
    if (r.accumulate) {
      const float4 c = *dst;
      s.x += c.x; s.y += c.y; s.z += c.z; s.w += c.w;
    }
    *dst = s;
  }
}

}  // namespace dct

template <bool TA, bool TB>
static hipError_t launch_gemm(const dct::GemmArgs& g, hipStream_t st) {
  const size_t lds = (size_t)(2 * dct::GBM * dct::GLD + 2 * dct::GBN * dct::GLD) * sizeof(uint16_t);
  auto fn = dct::gemm_bf16_kernel<TA, TB>;
  hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  const int tiles = ((g.M + dct::GBM - 1) / dct::GBM) * ((g.N + dct::GBN - 1) / dct::GBN);
  hipLaunchKernelGGL(fn, dim3(tiles), dim3(dct::GNT), lds, st, g);
  return hipGetLastError();
}

static bool gemm_v2_ok(const dct::GemmArgs& g, int ta, int tb) {
  if (g.K % dct::GBK) return false;
  auto aligned = [](const void* p) { return (((uintptr_t)p) & 15) == 0; };
  if (!aligned(g.A) || !aligned(g.B) || g.lda % 8 || g.ldb % 8) return false;
  if (ta && g.M % 8) return false;    // MC image of A: 8-row chunks inside [0, M)
  if (!tb && g.N % 8) return false;   // MC image of B
  return true;
}

// Two-pass split-K partials.  Auto mode takes it for <= 4 slices per tile: 1024 x 1024 x 4096 dW
// (4 slices) 30.0 -> 23.3 us, tabular step 0.186 -> 0.1835 ms; with 16-64 slices (1024 x 256 x
// 4096, the 32k-row transformer dW) the reduce pass costs more than the atomics it removes (15.9 ->
// 16.7 us, 13-15 -> 28-29 us; profiles/gemm_splitk_two_pass_ab_r2.log).
// One buffer per process, allocated outside stream capture and only ever superseded, never freed (a
// captured graph keeps the pointer it recorded); the split GEMMs and their reduce run in stream
// order on one compute stream, so one buffer serves them in turn.  (An in-launch reduction by the
// last-arriving slice measured slower than this reduce launch, profiles/gemm_splitk_inlaunch_ab_r4.log.)
static float* g_part = nullptr;
static size_t g_part_bytes = 0;
static int g_part_dev = -1;
static float* split_partials(size_t bytes, int max_splits, hipStream_t st) {
  if (max_splits > 4) return nullptr;
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  if (g_part && g_part_dev == dev && g_part_bytes >= bytes) return g_part;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
  if (g_part_dev != -1 && g_part_dev != dev) return nullptr;  // one device per process
  const size_t want = std::max<size_t>(bytes, (size_t)32 << 20);
  float* w = nullptr;
  if (hipMalloc(&w, want) != hipSuccess) { (void)hipGetLastError(); return nullptr; }
  g_part = w; g_part_bytes = want; g_part_dev = dev;
  return g_part;
}

static int device_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
      cus = v;
    else
      cus = 256;
  }
  return cus;
}

// LDS pipeline depth: 2.  Measured on the MLP / transformer shapes (tools/bench_gemm_mlp.py,
// profiles/gemm_pipeline_ab_r1.log, profiles/gemm_probe_r4.log): 3 or 4 stages never beat 2 - with
// 32 KB of operands per k-step a CU's global -> LDS rate, not the round-trip latency, bounds these
// one-tile-per-CU grids.

template <bool TA, bool TB>
static hipError_t launch_gemm2(dct::GemmArgs g, hipStream_t st) {
  hipError_t e;
  const int tiles_n = (g.N + dct::GBN - 1) / dct::GBN;
  const int tiles = ((g.M + dct::GBM - 1) / dct::GBM) * tiles_n;
  const int nk = g.K / dct::GBK;
  int splits = 1;
  if (g.out_f32 && g.epilogue == dct::EPI_NONE && !g.residual && g.alpha == 1.0f && tiles < 256 && nk >= 8) {
    // >= 8 k-tiles per slice: fewer fp32 atomics (measured: 64 slices of 8 beat 128 of 4 by 20-30 %
    // on the 32k-row transformer dW shapes - tools/bench_dw.py)
    // workgroups to aim for: one per CU.  512 (two slices per CU) doubled the fp32 atomic traffic
    // for no extra bandwidth: 1024x1024x4096 dW 38 -> 28 us at 256 (profiles/gemm_pipeline_ab_r1.log)
    const int target = device_cus();
    splits = std::min(nk / 8, (target + tiles - 1) / tiles);
    if (splits < 1) splits = 1;
  }
  if (splits > 1) {
    g.split_part = split_partials((size_t)splits * g.M * g.N * sizeof(float), splits, st);
  }
  if (splits > 1 && !g.accumulate && !g.split_part) {  // slices accumulate atomically into a zeroed C
    const int64_t total = (int64_t)g.M * g.N;
    const int zgrid = (int)std::min<int64_t>(2048, (total + 255) / 256);
    hipLaunchKernelGGL(dct::zero_panel_kernel, dim3(zgrid), dim3(256), 0, st, reinterpret_cast<float*>(g.C), g.ldc,
                       g.M, g.N);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  const int nk_slice = (nk + splits - 1) / splits;
  auto launch = [&](auto fn, int grid, int stages, int threads = dct::GNT) -> hipError_t {
    // one k-tile -> one LDS stage; otherwise `stages` stages of A + B images
    const size_t lds = (size_t)(nk_slice > 1 ? 2 * stages : 2) * dct::G2_BYTES;
    hipError_t err = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (err != hipSuccess) return err;
    hipLaunchKernelGGL(fn, dim3(grid), dim3(threads), lds, st, g, splits);
    return hipGetLastError();
  };
  // between one half and one 128 x 128 tile per CU (the 4096 x 1024 MLP layers: 256 tiles): 8 waves (two per SIMD)
  // and 128-deep k stages.  Such grids are bound by each CU's global -> LDS rate, and 256-byte row
  // segments per stage raise it: 4096 x 1024 x 1024 fwd / dX 15.1 / 17.2 -> 13.4 / 14.8 us
  // (half-height tiles, two per CU, below), tabular step 176.2 -> 175.7 us; from K = 256 on (the
  // 256-feature input layer: two k stages) 166.7 -> 163.7 us (profiles/gemm_k128_ab_r4.log,
  // tools/probes/gemm_probe.hip).
  if (splits == 1 && tiles <= device_cus() && 2 * tiles > device_cus() && g.K % 128 == 0 &&
      g.K >= 256) {
    auto fn = dct::gemm2_kernel<TA, TB, false, 128, 2, 4, 128>;
    const size_t lds = (size_t)2 * 2 * (128 * 2 * 128);  // 2 stages x (A + B) images of 128 x 128 bf16
    e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(fn, dim3(tiles), dim3(512), lds, st, g, 1);
    return hipGetLastError();
  }
  if constexpr (!TA) {
    // small K (<= 4 k-tiles) and too few 128-row tiles to fill 256 CUs several times over: half-height tiles
    // ... and whenever 128-row tiles would give at most one workgroup per CU (the 4096 x 1024 MLP
    // layers: 256 tiles): two half-height tiles per CU overlap one's loads with the other's MFMAs,
    // 16.7 -> 14.5 us fwd / 17.4 -> 15.5 us dX at 4096x1024x1024, ahead of hipBLASLt (17.8 / 17.2;
    // profiles/gemm_bm64_ab_r1.log)
    if (splits == 1 && (nk <= 4 || tiles <= device_cus()) && tiles < 1024)
      return launch(dct::gemm2_kernel<TA, TB, false, 64, 2>, ((g.M + 63) / 64) * tiles_n, 2);
  }
  if (splits > 1) {
    const int grid = tiles * splits;
    // 8 waves (two per SIMD) on the split-K dW tiles: more loads in flight per CU on these
    // load-path-bound one-tile-per-CU grids - tabular step 170.9 -> 165.9 us, the TabTransformer's
    // grouped dW launch unchanged (profiles/gemm_split_8w_ab_r4.log)
    e = launch(dct::gemm2_kernel<TA, TB, true, 128, 2, 4>, grid, 2, 512);
    if (e != hipSuccess || !g.split_part) return e;
    const int64_t n4 = ((int64_t)g.M * g.N + 3) / 4;
    hipLaunchKernelGGL(dct::splitk_reduce_kernel, dim3((int)std::min<int64_t>(2048, (n4 + 255) / 256)), dim3(256), 0,
                       st, g.split_part, splits, reinterpret_cast<float*>(g.C), g.ldc, g.M, g.N, g.accumulate,
                       g.alpha);
    return hipGetLastError();
  }
  return launch(dct::gemm2_kernel<TA, TB, false, 128, 2>, tiles, 2);
}

// dW = dZ^T X as `splits` split-K slices stored to part[splits][M][N] (no reduce: the consumer -
// the executor's Adam - sums them in slice order); colsum (+)= column sums of dZ by atomics.
// dZ [K][M], X [K][N] bf16 row-major.  Returns hipErrorInvalidValue when the shape does not take the
// LDS-DMA kernel or the slices would not each hold >= 1 k-tile.
extern "C" int dct_gemm_bf16_dw_partials(const uint16_t* dZ, const uint16_t* X, float* part, float* colsum, int M,
                                         int N, int K, int splits, void* stream) {
  dct::GemmArgs g{};
  g.A = dZ; g.B = X; g.C = part; g.M = M; g.N = N; g.K = K; g.lda = M; g.ldb = N; g.ldc = N;
  g.epilogue = dct::EPI_NONE; g.out_f32 = 1; g.accumulate = 0; g.alpha = 1.0f;
  g.vec_a = ((((uintptr_t)dZ) & 15) == 0) && (M % 8 == 0);
  g.vec_b = ((((uintptr_t)X) & 15) == 0) && (N % 8 == 0);
  g.colsum = colsum;
  g.split_part = part;
  const int nk = K / dct::GBK;
  if (!part || M <= 0 || N <= 0 || !gemm_v2_ok(g, 1, 0) || splits < 1 || splits > nk) return (int)hipErrorInvalidValue;
  const int tiles = ((M + dct::GBM - 1) / dct::GBM) * ((N + dct::GBN - 1) / dct::GBN);
  const int nk_slice = (nk + splits - 1) / splits;
  if ((splits - 1) * nk_slice >= nk) return (int)hipErrorInvalidValue;  // an empty slice would store zeros: fine, but keep it tight
  auto fn = dct::gemm2_kernel<true, false, true, 128, 2, 4>;
  const size_t lds = (size_t)(nk_slice > 1 ? 4 : 2) * dct::G2_BYTES;
  hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(fn, dim3(tiles * splits), dim3(512), lds, reinterpret_cast<hipStream_t>(stream),
                     g, splits);
  return (int)hipGetLastError();
}

// dW split-K partials with an Adam range riding along: workgroups [0, gemm_wgs) are the GEMM's
// (XCD-aware remap over that count), the rest run Adam over the range.  The Adam
// workgroups need no LDS but inherit the launch's dynamic LDS (64 KB), so one sits beside each
// GEMM tile on a CU (2 x 64 KB <= 160 KB): the HBM-bound optimizer streams under the GEMM, which is
// bound by each CU's global -> LDS rate (tabular step: the separate Adam launch was 17 us).
// F4: the float4 body (adam_flat_range) instead of one element per thread (adam_scalar_range, the
// executor's choice: 155.4-157.1 vs 158.0-158.6 us per tabular step, profiles/packed_fp32_lds_dma_r6.log).
// Both are exact here because this file is compiled without packed fp32 (_build.py FILE_FLAGS):
// compiled WITH v_pk_* the float4 body went wrong beside the GEMM tiles' LDS-DMA (same log).
template <int S_ADAM, bool F4 = false>
__global__ __launch_bounds__(512, 2) void gemm2_dw_adam_kernel(dct::GemmArgs g, int splits, int gemm_wgs,
                                                               dct::AdamArgs a, int64_t lo, int64_t hi) {
  if ((int)blockIdx.x < gemm_wgs) {
    const int orig = blockIdx.x, xcd = orig & 7;
    const int q8 = gemm_wgs >> 3, r8 = gemm_wgs & 7;
    const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
    dct::gemm2_body<true, false, true, 128, 2, 4>(g, splits, wgid);
  } else if constexpr (F4) {
    dct::adam_flat_range<true, S_ADAM>(a, lo, hi, blockIdx.x - gemm_wgs, gridDim.x - gemm_wgs);
  } else {
    dct::adam_scalar_range<true, S_ADAM>(a, lo, hi, blockIdx.x - gemm_wgs, gridDim.x - gemm_wgs);
  }
}

extern "C" int dct_gemm_bf16_dw_partials_adam(const uint16_t* dZ, const uint16_t* X, float* part, float* colsum, int M,
                                              int N, int K, int splits, const dct::AdamRange* r, void* stream) {
  return dct_gemm_bf16_dw_partials_adam_ex(dZ, X, part, colsum, M, N, K, splits, r, 0, stream);
}

extern "C" int dct_gemm_bf16_dw_partials_adam_ex(const uint16_t* dZ, const uint16_t* X, float* part, float* colsum,
                                                 int M, int N, int K, int splits, const dct::AdamRange* r, int f4,
                                                 void* stream) {
  if (!r) return dct_gemm_bf16_dw_partials(dZ, X, part, colsum, M, N, K, splits, stream);
  dct::GemmArgs g{};
  g.A = dZ; g.B = X; g.C = part; g.M = M; g.N = N; g.K = K; g.lda = M; g.ldb = N; g.ldc = N;
  g.epilogue = dct::EPI_NONE; g.out_f32 = 1; g.accumulate = 0; g.alpha = 1.0f;
  g.vec_a = ((((uintptr_t)dZ) & 15) == 0) && (M % 8 == 0);
  g.vec_b = ((((uintptr_t)X) & 15) == 0) && (N % 8 == 0);
  g.colsum = colsum;
  g.split_part = part;
  const int nk = K / dct::GBK;
  if (!part || M <= 0 || N <= 0 || !gemm_v2_ok(g, 1, 0) || splits < 1 || splits > nk) return (int)hipErrorInvalidValue;
  const int tiles = ((M + dct::GBM - 1) / dct::GBM) * ((N + dct::GBN - 1) / dct::GBN);
  const int nk_slice = (nk + splits - 1) / splits;
  if ((splits - 1) * nk_slice >= nk) return (int)hipErrorInvalidValue;
  dct::AdamArgs a{};
  int max_sp = 1;
  const int e0 = dct::adam_args_from_range(*r, a, &max_sp);
  if (e0) return e0;
  const int gemm_wgs = tiles * splits;
  // one Adam workgroup (512 threads) per CU beside the GEMM tiles, fewer for a short range
  const int64_t work = r->hi - r->lo;  // elements, one per thread and iteration
  int adam_wgs = (int)std::min<int64_t>((work + 511) / 512, device_cus());
  if (adam_wgs < 1) adam_wgs = 1;
  const size_t lds = (size_t)(nk_slice > 1 ? 4 : 2) * dct::G2_BYTES;
  auto fn = f4 ? (max_sp > 4 ? gemm2_dw_adam_kernel<8, true> : gemm2_dw_adam_kernel<4, true>)
              : (max_sp > 4 ? gemm2_dw_adam_kernel<8> : gemm2_dw_adam_kernel<4>);
  hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(fn, dim3(gemm_wgs + adam_wgs), dim3(512), lds, reinterpret_cast<hipStream_t>(stream), g, splits,
                     gemm_wgs, a, r->lo, r->hi);
  return (int)hipGetLastError();
}

// the split count launch_gemm2 picks for an fp32-out dW of this shape (1 = not split)
extern "C" int dct_gemm_dw_auto_splits(int M, int N, int K) {
  const int tiles = ((M + dct::GBM - 1) / dct::GBM) * ((N + dct::GBN - 1) / dct::GBN);
  const int nk = K / dct::GBK;
  if (tiles >= 256 || nk < 8 || K % dct::GBK) return 1;
  const int splits = std::min(nk / 8, (device_cus() + tiles - 1) / tiles);
  return splits < 1 ? 1 : splits;
}

extern "C" int dct_bias_act_bwd(const void* dY, const void* act_aux, uint16_t* dZ, float* dbias, int M, int N,
                                int ldy, int act, int accumulate_bias, void* stream);

extern "C" int dct_gemm_bf16_ex(const uint16_t* A, const uint16_t* B, void* C, const float* bias, int M, int N, int K,
                                int lda, int ldb, int ldc, int trans_a, int trans_b, int epilogue, int out_f32,
                                int accumulate, void* aux, float* colsum, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  dct::GemmArgs g{};
  g.A = A; g.B = B; g.C = C; g.bias = bias; g.aux = aux;
  g.M = M; g.N = N; g.K = K; g.lda = lda; g.ldb = ldb; g.ldc = ldc;
  g.epilogue = epilogue; g.out_f32 = out_f32; g.accumulate = accumulate; g.alpha = 1.0f;
  g.vec_a = ((((uintptr_t)A) & 15) == 0) && (lda % 8 == 0);
  g.vec_b = ((((uintptr_t)B) & 15) == 0) && (ldb % 8 == 0);
  g.colsum = colsum;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (gemm_v2_ok(g, trans_a, trans_b)) {
    if (!trans_a && trans_b) return (int)launch_gemm2<false, true>(g, st);
    if (!trans_a && !trans_b) return (int)launch_gemm2<false, false>(g, st);
    if (trans_a && !trans_b) return (int)launch_gemm2<true, false>(g, st);
    return (int)launch_gemm2<true, true>(g, st);
  }
  g.colsum = nullptr;
  int e = dct_gemm_bf16(A, B, C, bias, M, N, K, lda, ldb, ldc, trans_a, trans_b, epilogue, out_f32, accumulate, aux,
                        stream);
  if (e || !colsum) return e;
  // generic path: the A rows' sums by the column-sum kernel (op(A) = A^T when trans_a: A is [K][M])
  if (trans_a) return dct_bias_act_bwd(A, nullptr, nullptr, colsum, K, M, lda, 0, 1, stream);
  return (int)hipErrorNotSupported;
}

// Grouped dW: C_i (+)= dZ_i^T X_i (+ colsum_i += column sums of dZ_i) for i < n (n <= 4), one
// launch.  dZ_i [K][M_i] and X_i [K][N_i] bf16 row-major (K = rows of the batch), C_i fp32 [M_i][N_i].
// Falls back to one launch per problem when a problem does not fit the grouped split-K kernel.
static int dw_grouped_impl(int n, const uint16_t* const* dZ, const uint16_t* const* X, float* const* C,
                           const int* M, const int* N, int K, float* const* colsum, int accumulate,
                           const dct::EmbedRide& er, void* stream);

extern "C" int dct_gemm_bf16_dw_grouped(int n, const uint16_t* const* dZ, const uint16_t* const* X, float* const* C,
                                        const int* M, const int* N, int K, float* const* colsum, int accumulate,
                                        void* stream) {
  return dw_grouped_impl(n, dZ, X, C, M, N, K, colsum, accumulate, dct::EmbedRide{}, stream);
}

// the same launch with the TabTransformer embedding gradients riding (dct::EmbedRide; ex null: none).
// Returns 1 when the ride did NOT run (the problems took the per-problem fallback): the caller then
// launches dct_tt_embed_bwd itself.
extern "C" int dct_gemm_bf16_dw_grouped_embed(int n, const uint16_t* const* dZ, const uint16_t* const* X,
                                              float* const* C, const int* M, const int* N, int K,
                                              float* const* colsum, int accumulate, const float* ex,
                                              const float* edh, float* edE, float* edc, int eB, int eF,
                                              void* stream) {
  return dw_grouped_impl(n, dZ, X, C, M, N, K, colsum, accumulate, dct::EmbedRide{ex, edh, edE, edc, eB, eF}, stream);
}

static int dw_grouped_impl(int n, const uint16_t* const* dZ, const uint16_t* const* X, float* const* C,
                           const int* M, const int* N, int K, float* const* colsum, int accumulate,
                           const dct::EmbedRide& er, void* stream) {
  if (n <= 0 || n > dct::DW_GROUP || K <= 0) return n == 0 ? 0 : (int)hipErrorInvalidValue;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  dct::GemmGroup gg{};
  gg.n = n;
  bool grouped = true;
  int total = 0, max_slice = 1;
  for (int i = 0; i < n; ++i) {
    dct::GemmArgs& g = gg.g[i];
    g.A = dZ[i]; g.B = X[i]; g.C = C[i]; g.bias = nullptr; g.aux = nullptr;
    g.M = M[i]; g.N = N[i]; g.K = K; g.lda = M[i]; g.ldb = N[i]; g.ldc = N[i];
    g.epilogue = dct::EPI_NONE; g.out_f32 = 1; g.accumulate = accumulate; g.alpha = 1.0f;
    g.vec_a = ((((uintptr_t)dZ[i]) & 15) == 0) && (M[i] % 8 == 0);
    g.vec_b = ((((uintptr_t)X[i]) & 15) == 0) && (N[i] % 8 == 0);
    g.colsum = colsum ? colsum[i] : nullptr;
    g.residual = nullptr;
    const int tiles = ((g.M + dct::GBM - 1) / dct::GBM) * ((g.N + dct::GBN - 1) / dct::GBN);
    const int nk = g.K / dct::GBK;
    if (!gemm_v2_ok(g, 1, 0) || tiles >= 256 || nk < 8) { grouped = false; break; }
  }
  // k-tiles per split slice: 8, doubled (up to 64) while the whole group would exceed two
  // workgroups per CU.  One transformer block's four dW GEMMs (448 workgroups at 8) keep 8; the
  // four blocks' sixteen deferred to one launch go to 32 (448 workgroups instead of 1792: a quarter
  // of the fp32 atomics, four times the k-loop per slice): TabTransformer step 0.411 -> 0.368 ms
  // (profiles/tt_dw_mink_ab_r2.log).
  const int target = device_cus();
  int min_kt = 8;
  for (;;) {
    total = 0;
    max_slice = 1;
    for (int i = 0; grouped && i < n; ++i) {
      const dct::GemmArgs& g = gg.g[i];
      const int tiles = ((g.M + dct::GBM - 1) / dct::GBM) * ((g.N + dct::GBN - 1) / dct::GBN);
      const int nk = g.K / dct::GBK;
      int splits = std::min(nk / min_kt, (target + tiles - 1) / tiles);
      if (splits < 1) splits = 1;
      gg.splits[i] = splits;
      gg.start[i] = total;
      total += tiles * splits;
      max_slice = std::max(max_slice, (nk + splits - 1) / splits);
    }
    if (!grouped || total <= 2 * device_cus() || min_kt >= 64) break;
    min_kt *= 2;
  }
  if (!grouped) {
    for (int i = 0; i < n; ++i) {
      const int e = dct_gemm_bf16_ex(dZ[i], X[i], C[i], nullptr, M[i], N[i], K, M[i], N[i], N[i], 1, 0, dct::EPI_NONE, 1,
                                     accumulate, nullptr, colsum ? colsum[i] : nullptr, stream);
      if (e) return e;
    }
    return er.x ? 1 : 0;  // the ride did not run
  }
  gg.start[n] = total;
  gg.er = er;
  const int ride = er.x ? er.F : 0;
  hipError_t e;
  // two-pass split-K (see split_partials): partial regions back to back, one grouped reduce after
  dct::SplitRedGroup rg{};
  size_t part_floats = 0;
  bool two_pass = true;
  int max_splits = 1;
  for (int i = 0; i < n; ++i) two_pass = two_pass && N[i] % 4 == 0 && ((((uintptr_t)C[i]) & 15) == 0);
  for (int i = 0; i < n; ++i) part_floats += (size_t)gg.splits[i] * M[i] * N[i];
  for (int i = 0; i < n; ++i) max_splits = std::max(max_splits, gg.splits[i]);
  float* part = two_pass ? split_partials(part_floats * sizeof(float), max_splits, st) : nullptr;
  if (part) {
    rg.n = n; rg.accumulate = accumulate;
    size_t off = 0;
    int64_t s4 = 0;
    for (int i = 0; i < n; ++i) {
      gg.g[i].split_part = part + off;
      rg.part[i] = part + off; rg.C[i] = C[i]; rg.N[i] = N[i]; rg.splits[i] = gg.splits[i];
      rg.MN[i] = (int64_t)M[i] * N[i];
      rg.start[i] = s4;
      s4 += rg.MN[i] / 4;
      off += (size_t)gg.splits[i] * M[i] * N[i];
    }
    rg.start[n] = s4;
  }
  if (!accumulate && !part) {
    for (int i = 0; i < n; ++i) {
      const int64_t tot = (int64_t)M[i] * N[i];
      hipLaunchKernelGGL(dct::zero_panel_kernel, dim3((int)std::min<int64_t>(2048, (tot + 255) / 256)), dim3(256), 0,
                         st, C[i], N[i], M[i], N[i]);
    }
  }
  const size_t lds = (size_t)(max_slice > 1 ? 4 : 2) * dct::G2_BYTES;
  auto fn = dct::gemm2_grouped_kernel<true, false, 2, 4>;
  e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(fn, dim3(total + ride), dim3(512), lds, st, gg);
  e = hipGetLastError();
  if (e != hipSuccess || !part) return (int)e;
  hipLaunchKernelGGL(dct::splitk_reduce_grouped_kernel,
                     dim3((int)std::min<int64_t>(2048, (rg.start[n] + 255) / 256)), dim3(256), 0, st, rg);
  return (int)hipGetLastError();
}

extern "C" int dct_gemm_bf16_residual(const uint16_t* A, const uint16_t* W, float* C, const float* bias,
                                      const float* residual, int M, int N, int K, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  dct::GemmArgs g{};
  g.A = A; g.B = W; g.C = C; g.bias = bias; g.residual = residual;
  g.M = M; g.N = N; g.K = K; g.lda = K; g.ldb = K; g.ldc = N;
  g.epilogue = bias ? dct::EPI_BIAS : dct::EPI_NONE; g.out_f32 = 1; g.accumulate = 0; g.alpha = 1.0f;
  g.vec_a = ((((uintptr_t)A) & 15) == 0) && (K % 8 == 0);
  g.vec_b = ((((uintptr_t)W) & 15) == 0) && (K % 8 == 0);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (gemm_v2_ok(g, 0, 1)) return (int)launch_gemm2<false, true>(g, st);  // never split-K with a residual
  return (int)launch_gemm<false, true>(g, st);
}

// dct_gemm_bf16 (below) that also writes op(B)^T = B^T [K][N] (row stride bt_ld) to bt_out: NT only, on
// the LDS-DMA kernels without split-K (hipErrorInvalidValue otherwise, nothing launched)
extern "C" int dct_gemm_bf16_bt(const uint16_t* A, const uint16_t* B, void* C, const float* bias, int M, int N, int K,
                                int lda, int ldb, int ldc, int epilogue, int out_f32, void* aux, uint16_t* bt_out,
                                int bt_ld, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  dct::GemmArgs g{};
  g.A = A; g.B = B; g.C = C; g.bias = bias; g.aux = aux;
  g.M = M; g.N = N; g.K = K; g.lda = lda; g.ldb = ldb; g.ldc = ldc;
  g.epilogue = epilogue; g.out_f32 = out_f32; g.accumulate = 0; g.alpha = 1.0f;
  g.vec_a = ((((uintptr_t)A) & 15) == 0) && (lda % 8 == 0);
  g.vec_b = ((((uintptr_t)B) & 15) == 0) && (ldb % 8 == 0);
  g.bt_out = bt_out; g.bt_ld = bt_ld;
  const bool split_k = out_f32 && epilogue == dct::EPI_NONE;  // (launch_gemm2 splits only fp32 EPI_NONE outputs)
  if (!gemm_v2_ok(g, 0, 1) || split_k || (((uintptr_t)bt_out) & 15) || (bt_ld % 8) || (N % 8))
    return (int)hipErrorInvalidValue;
  return (int)launch_gemm2<false, true>(g, reinterpret_cast<hipStream_t>(stream));
}

// The wide-MLP step's batch gather (csrc/step_kernels.hip gather_batch_kernel) folded into its first
// forward GEMM: the A chunks are LDS-DMA loads from the dataset rows themselves, one workgroup per row band
// writes the gathered rows out for the dW GEMM, and labels / step counter / gradient clearing ride along -
// one launch and one kernel boundary fewer per step.  The same two kernel shapes launch_gemm2 picks for an
// NT bf16 forward: 8-wave 128-deep stages for a grid of 1/2..1 tile per CU, else 4 waves, 64-deep stages.
extern "C" int dct_gemm_bf16_gather_fwd(const uint16_t* X, int ldx, const uint16_t* W, uint16_t* C, const float* bias,
                                        int M, int N, int K, int epilogue, void* aux, const dct::GatherFwd* ga,
                                        void* stream) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  if (!ga || !ga->idx || !ga->cursor || ga->n_items <= 0 || ga->stride < 0 || ga->nz < 0 || ga->nz > 4 ||
      (ga->ydst && !ga->Y) || (((uintptr_t)ga->a_out) & 15))
    return (int)hipErrorInvalidValue;
  for (int q = 0; q < ga->nz; ++q)
    if (!ga->zero || (((uintptr_t)ga->zero) & 15) || ga->zoff[q] % 4 || ga->zcnt[q] < 0) return (int)hipErrorInvalidValue;
  if (epilogue == dct::EPI_RELU_MASK || epilogue == dct::EPI_GELU_GRAD) return (int)hipErrorInvalidValue;
  dct::GemmArgs g{};
  g.A = X; g.B = W; g.C = C; g.bias = bias; g.aux = aux;
  g.M = M; g.N = N; g.K = K; g.lda = ldx; g.ldb = K; g.ldc = N;
  g.epilogue = epilogue; g.out_f32 = 0; g.accumulate = 0; g.alpha = 1.0f;
  g.vec_a = ((((uintptr_t)X) & 15) == 0) && (ldx % 8 == 0);
  g.vec_b = ((((uintptr_t)W) & 15) == 0) && (K % 8 == 0);
  if (!gemm_v2_ok(g, 0, 1) || N % 8) return (int)hipErrorInvalidValue;
  const int tiles = ((M + dct::GBM - 1) / dct::GBM) * ((N + dct::GBN - 1) / dct::GBN);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (tiles <= device_cus() && 2 * tiles > device_cus() && K % 128 == 0 && K >= 256) {
    auto fn = dct::gemm2_gather_kernel<128, 2, 4, 128>;
    const size_t lds = (size_t)2 * 2 * (128 * 2 * 128);
    hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(fn, dim3(tiles), dim3(512), lds, st, g, *ga);
    return (int)hipGetLastError();
  }
  auto fn = dct::gemm2_gather_kernel<128, 2, 2, 64>;
  const size_t lds = (size_t)(K / dct::GBK > 1 ? 4 : 2) * dct::G2_BYTES;
  hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(fn, dim3(tiles), dim3(256), lds, st, g, *ga);
  return (int)hipGetLastError();
}

extern "C" int dct_gemm_bf16(const uint16_t* A, const uint16_t* B, void* C, const float* bias, int M, int N, int K,
                             int lda, int ldb, int ldc, int trans_a, int trans_b, int epilogue, int out_f32,
                             int accumulate, void* aux, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  dct::GemmArgs g{};
  g.A = A; g.B = B; g.C = C; g.bias = bias; g.aux = aux;
  g.M = M; g.N = N; g.K = K; g.lda = lda; g.ldb = ldb; g.ldc = ldc;
  g.epilogue = epilogue; g.out_f32 = out_f32; g.accumulate = accumulate; g.alpha = 1.0f;
  // 16-B vector staging needs 16-B aligned rows along the contiguous dimension
  g.vec_a = ((((uintptr_t)A) & 15) == 0) && (lda % 8 == 0);
  g.vec_b = ((((uintptr_t)B) & 15) == 0) && (ldb % 8 == 0);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipError_t e;
  if (gemm_v2_ok(g, trans_a, trans_b)) {
    if (!trans_a && trans_b) return (int)launch_gemm2<false, true>(g, st);
    if (!trans_a && !trans_b) return (int)launch_gemm2<false, false>(g, st);
    if (trans_a && !trans_b) return (int)launch_gemm2<true, false>(g, st);
    return (int)launch_gemm2<true, true>(g, st);
  }
  if (!trans_a && trans_b) e = launch_gemm<false, true>(g, st);
  else if (!trans_a && !trans_b) e = launch_gemm<false, false>(g, st);
  else if (trans_a && !trans_b) e = launch_gemm<true, false>(g, st);
  else e = launch_gemm<true, true>(g, st);
  return (int)e;
}
