// Weight gradients of the TabTransformer block kernels (csrc/tt_block.hip) as whole-problem tiles:
//
//   C[Mi][Ni] += A^T B,  colsum[Mi] += column sums of A     A [K][Mi], B [K][Ni] bf16 row-major, K = rows
//
// for the four products of a block: dW2 = dout^T f (64 x 256), dW1 = dpre^T a2 (256 x 64),
// dWo = dh1^T o (64 x 64), dWqkv = dqkv^T a1 (192 x 64), every block of the model in one launch.
// The generic split-K GEMM (gemm_bf16.hip gemm2_grouped_kernel) tiles them 128 x 128: every problem
// has a 64-wide operand, whose 128-wide image then holds each 16-byte chunk twice, and the two 128-
// column tiles of dW2 / dW1 each load the narrow operand again - 448 MB of global -> LDS traffic for
// 268 MB of operands, on a kernel bound by the CU's load rate.  Here a workgroup owns a problem's
// whole output for a slice of the rows, so every operand byte is loaded once per slice.
//
// Per 64-row chunk both operands go to LDS as k-row-major images (register-staged, the next chunk's
// loads in flight under this chunk's MFMAs) and reach v_mfma_f32_16x16x32_bf16 through
// ds_read_b64_tr_b16 (both are "k down the rows": A^T's rows and B's columns are image columns).
// Rows are XOR-swizzled per 16-byte chunk so the 8 rows a 32-lane half reads land on 16 distinct
// 4-bank slots.  Wave w owns a quarter of the output tiles (mt-major), so each m-tile - and its
// bias column sums - has one owner.  Slices per problem follow its bytes per row (about one
// workgroup per CU in all); outputs and bias sums leave as fp32 atomics.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dct_common.h"
#include "kernels.h"

namespace dct {
namespace ttdw {

constexpr int KC = 64;        // rows per chunk
constexpr int MAXQ = 16;      // problems per launch
constexpr int MAXW = 320;     // max Mi + Ni
constexpr int LDS_BYTES = 2 * KC * MAXW * 2;  // two stages of A | B images (80 KB)

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));  // staging (HIP's uint4 struct array went to scratch)
typedef __attribute__((address_space(3))) bf16x4 lds4;

struct Prob {
  const uint16_t* A;  // [K][Mi]
  const uint16_t* B;  // [K][Ni]
  float* C;           // [Mi][Ni]
  float* colsum;      // [Mi] or null
  int kind;           // 0: 64 x 256, 1: 256 x 64, 2: 64 x 64, 3: 192 x 64
  int slices, chunks_per_slice, wg0;  // first workgroup id of the problem
};
struct Args {
  Prob p[MAXQ];
  int n, K;
};

// physical 16-byte chunk of chunk c in row r of an image with W-byte rows
template <int W>
__device__ __forceinline__ int swz(int r, int c) {
  if constexpr ((W / 4) % 64 == 0) return c ^ (((r & 3) | (((r >> 3) & 1) << 2)) << 1);
  else return c ^ ((r & 2) | ((r >> 1) & 4));
}

// fragment of columns 16 t .. 16 t + 15 (lane c), k = 32 ks + 8 g + e (element e), natural order
template <int W>
__device__ __forceinline__ bf16x8 tr_frag(const char* img, int t, int ks, int c, int g) {
  const int q = c >> 2, p = c & 3, ch = 2 * t + (p >> 1);
  const int r0 = 32 * ks + 8 * g + q, r1 = r0 + 4;
  const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4*)(img + r0 * W + (swz<W>(r0, ch) << 4) + (p & 1) * 8));
  const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4*)(img + r1 * W + (swz<W>(r1, ch) << 4) + (p & 1) * 8));
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

template <int MI, int NI, int NW>
__device__ __forceinline__ void dw_body(const Prob& P, int slice, int K, char* smem) {
  constexpr int WA = MI * 2, WB = NI * 2;           // image row bytes
  constexpr int MT = MI / 16, NT = NI / 16;          // 16 x 16 tiles
  // NW waves as a WR x WC grid over the 16 x 16 output tiles
  constexpr int WR = (MT % NW == 0) ? NW : 4, WC = NW / WR;
  constexpr int WMT = MT / WR, WNT = NT / WC;        // tiles per wave
  static_assert(WR * WC == NW && WMT * WR == MT && WNT * WC == NT, "whole tiles per wave");
  constexpr int NTH = 64 * NW;
  constexpr int CA = KC * WA / 16, CB = KC * WB / 16;  // 16-byte chunks per image
  constexpr int PER = (CA + CB) / NTH;                // per thread
  static_assert(CA % NTH == 0 && CB % NTH == 0, "whole chunk rounds per image");
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int mt0 = (wv / WC) * WMT, nt0 = (wv % WC) * WNT;  // first tile of the wave
  const int k0 = slice * P.chunks_per_slice * KC;
  const int nch = min(P.chunks_per_slice, (K - k0) / KC);

  auto stage = [&](int s) -> char* { return smem + s * KC * (WA + WB); };
  u32x4 stg[2][PER];  // two chunks' loads in flight (the kernel is bound by bytes in flight per CU)
  constexpr int QA = CA / NTH;  // rounds of the A image, then the B image
#define TTDW_LOAD(SET, CH)                                                                                  \
  {                                                                                                    \
    const int r0_ = k0 + (CH) * KC;                                                                    \
    _Pragma("unroll") for (int q = 0; q < QA; ++q) {                                                   \
      const int L = q * NTH + tid, r = L / (WA / 16), cc = L - r * (WA / 16);                          \
      stg[SET][q] = *reinterpret_cast<const u32x4*>(P.A + (size_t)(r0_ + r) * MI + cc * 8);                 \
    }                                                                                                  \
    _Pragma("unroll") for (int q = QA; q < PER; ++q) {                                                 \
      const int L = (q - QA) * NTH + tid, r = L / (WB / 16), cc = L - r * (WB / 16);                   \
      stg[SET][q] = *reinterpret_cast<const u32x4*>(P.B + (size_t)(r0_ + r) * NI + cc * 8);                 \
    }                                                                                                  \
  }
#define TTDW_STORE(SET, S)                                                                                  \
  {                                                                                                    \
    char* base_ = stage(S);                                                                            \
    _Pragma("unroll") for (int q = 0; q < QA; ++q) {                                                   \
      const int L = q * NTH + tid, r = L / (WA / 16), cc = L - r * (WA / 16);                          \
      *reinterpret_cast<u32x4*>(base_ + r * WA + (swz<WA>(r, cc) << 4)) = stg[SET][q];                      \
    }                                                                                                  \
    _Pragma("unroll") for (int q = QA; q < PER; ++q) {                                                 \
      const int L = (q - QA) * NTH + tid, r = L / (WB / 16), cc = L - r * (WB / 16);                   \
      *reinterpret_cast<u32x4*>(base_ + KC * WA + r * WB + (swz<WB>(r, cc) << 4)) = stg[SET][q];            \
    }                                                                                                  \
  }

  f32x4 acc[WMT][WNT];
#pragma unroll
  for (int i = 0; i < WMT; ++i)
#pragma unroll
    for (int j = 0; j < WNT; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float cs[WMT];
#pragma unroll
  for (int i = 0; i < WMT; ++i) cs[i] = 0.f;
  const bool do_cs = P.colsum != nullptr && nt0 == 0;  // the wave that owns these m-tiles' first n-tile

#define TTDW_COMPUTE(CH)                                                                                \
  {                                                                                                     \
    const char* IA = stage((CH) & 1);                                                                   \
    const char* IB = IA + KC * WA;                                                                      \
    _Pragma("unroll") for (int ks = 0; ks < KC / 32; ++ks) {                                            \
      bf16x8 af[WMT], bfr[WNT];                                                                         \
      _Pragma("unroll") for (int i = 0; i < WMT; ++i) af[i] = tr_frag<WA>(IA, mt0 + i, ks, c, g);       \
      _Pragma("unroll") for (int j = 0; j < WNT; ++j) bfr[j] = tr_frag<WB>(IB, nt0 + j, ks, c, g);      \
      if (do_cs) {                                                                                      \
        _Pragma("unroll") for (int i = 0; i < WMT; ++i)                                                 \
          _Pragma("unroll") for (int e = 0; e < 8; ++e) cs[i] += bf16_to_f32((uint16_t)af[i][e]);       \
      }                                                                                                 \
      _Pragma("unroll") for (int i = 0; i < WMT; ++i)                                                   \
        _Pragma("unroll") for (int j = 0; j < WNT; ++j)                                                 \
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);       \
    }                                                                                                   \
  }
  // chunk ch computes from LDS stage ch & 1 while chunk ch + 1 waits in one register set and chunk
  // ch + 2's loads fly into the other; the loop body covers two chunks so the sets are static
  if (nch > 0) {
    TTDW_LOAD(0, 0);
    TTDW_STORE(0, 0);
  }
  if (nch > 1) TTDW_LOAD(1, 1);
  __syncthreads();
  for (int ch = 0; ch < nch; ch += 2) {
    if (ch + 2 < nch) TTDW_LOAD(0, ch + 2);
    TTDW_COMPUTE(ch);
    if (ch + 1 < nch) TTDW_STORE(1, (ch + 1) & 1);
    __syncthreads();
    if (ch + 1 >= nch) break;
    if (ch + 3 < nch) TTDW_LOAD(1, ch + 3);
    TTDW_COMPUTE(ch + 1);
    if (ch + 2 < nch) TTDW_STORE(0, (ch + 2) & 1);
    __syncthreads();
  }
  // C layout: acc[i][j][r] = C[16 (mt0 + i) + 4 g + r][16 (nt0 + j) + c]
#pragma unroll
  for (int i = 0; i < WMT; ++i)
#pragma unroll
    for (int j = 0; j < WNT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        atomicAdd(P.C + (size_t)(16 * (mt0 + i) + 4 * g + r) * NI + 16 * (nt0 + j) + c, acc[i][j][r]);
  if (do_cs) {
#pragma unroll
    for (int i = 0; i < WMT; ++i) {
      float v = cs[i];
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      if (g == 0) atomicAdd(P.colsum + 16 * (mt0 + i) + c, v);
    }
  }
}

// bijective XCD-aware remap (consecutive ids on one XCD)
__device__ __forceinline__ int xcd_id() {
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
}

template <int NW>
__global__ __launch_bounds__(64 * NW, 1) void tt_dw_kernel(Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int w = xcd_id();
  // the problem by a select chain (a dynamic index into the kernel argument array put it in scratch)
  Prob P = a.p[0];
#pragma unroll
  for (int i = 1; i < MAXQ; ++i)
    if (i < a.n && w >= a.p[i].wg0) P = a.p[i];
  const int slice = w - P.wg0;
  switch (P.kind) {
    case 0: dw_body<64, 256, NW>(P, slice, a.K, smem); break;
    case 1: dw_body<256, 64, NW>(P, slice, a.K, smem); break;
    case 2: dw_body<64, 64, NW>(P, slice, a.K, smem); break;
    default: dw_body<192, 64, NW>(P, slice, a.K, smem); break;
  }
}

static int device_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0, v = 0;
    cus = (hipGetDevice(&dev) == hipSuccess &&
           hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
              ? v
              : 256;
  }
  return cus;
}

}  // namespace ttdw
}  // namespace dct

extern "C" {

// n (<= 16) problems C_i[M_i][N_i] += A_i^T B_i (+ colsum_i += column sums of A_i) over the same K rows
// (K % 64 == 0); (M_i, N_i) one of (64, 256), (256, 64), (64, 64), (192, 64); A / B 16-byte aligned
int dct_tt_dw(int n, const uint16_t* const* A, const uint16_t* const* B, float* const* C, float* const* colsum,
              const int* M, const int* N, int K, int waves, int wg_per_cu, void* stream) {
  using namespace dct::ttdw;
  if (n <= 0 || n > MAXQ || K <= 0 || K % KC) return (int)hipErrorInvalidValue;
  Args a{};
  a.n = n;
  a.K = K;
  double total_bytes = 0;
  for (int i = 0; i < n; ++i) total_bytes += M[i] + N[i];
  const int nw = waves == 4 ? 4 : 8;
  const int target = device_cus() * (wg_per_cu == 2 ? 2 : 1);
  const int chunks = K / KC;
  int wg = 0;
  for (int i = 0; i < n; ++i) {
    int kind;
    if (M[i] == 64 && N[i] == 256) kind = 0;
    else if (M[i] == 256 && N[i] == 64) kind = 1;
    else if (M[i] == 64 && N[i] == 64) kind = 2;
    else if (M[i] == 192 && N[i] == 64) kind = 3;
    else return (int)hipErrorInvalidValue;
    if (!A[i] || !B[i] || !C[i] || ((((uintptr_t)A[i]) | ((uintptr_t)B[i])) & 15)) return (int)hipErrorInvalidValue;
    // slices in proportion to the problem's bytes per row: about one workgroup per CU overall
    int s = (int)(target * (M[i] + N[i]) / total_bytes + 0.5);
    s = s < 1 ? 1 : (s > chunks ? chunks : s);
    const int per = (chunks + s - 1) / s;
    s = (chunks + per - 1) / per;  // no empty slice
    a.p[i] = Prob{A[i], B[i], C[i], colsum ? colsum[i] : nullptr, kind, s, per, wg};
    wg += s;
  }
  static bool attr = false;
  if (!attr) {
    for (const void* k : {(const void*)tt_dw_kernel<4>, (const void*)tt_dw_kernel<8>}) {
      const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
      if (e != hipSuccess) return (int)e;
    }
    attr = true;
  }
  if (nw == 4)
    hipLaunchKernelGGL(tt_dw_kernel<4>, dim3(wg), dim3(256), LDS_BYTES, reinterpret_cast<hipStream_t>(stream), a);
  else
    hipLaunchKernelGGL(tt_dw_kernel<8>, dim3(wg), dim3(512), LDS_BYTES, reinterpret_cast<hipStream_t>(stream), a);
  return (int)hipGetLastError();
}

}  // extern "C"
