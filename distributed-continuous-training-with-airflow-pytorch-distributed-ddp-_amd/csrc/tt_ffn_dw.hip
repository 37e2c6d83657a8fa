// Weight gradients of the TabTransformer block's FFN (csrc/tt_block.hip) from its two narrow inputs:
//
//   pre  = a2 W1^T + b1            f   = bf16(gelu(pre))              (recomputed, as the forward)
//   dF   = bf16(dout) W2           dp  = bf16(dF * gelu'(bf16(pre)))  (recomputed, as the backward)
//   dW2 += bf16(dout)^T f          db2 += colsum(bf16(dout))
//   dW1 += dp^T a2                 db1 += colsum(dp)
//
// The block kernels used to write f ([B*64][256] bf16, forward) and dp ([B*64][256] bf16, backward)
// for the split-K dW GEMMs to read back: 64 MB per block through HBM at the benchmark batch, for
// products whose only other inputs are a2 and dout16 ([B*64][64] bf16 each, 8 MB).  Here the
// [64 x 256] hidden tiles are rebuilt from those two by MFMAs (the extra 2 x 2 x 64 x 256 flops per
// row are ~3 us of the chip's bf16 rate over all four blocks) and consumed where they are produced:
// the accumulator tiles of the first two products feed the last two as MFMA operands without
// leaving the registers (cdna_hip_programming.md 'An accumulator tile as the next MFMA's operand').
//
// Work: problem (block) p x FF column group J (64 columns) x row slice s; 4 waves = 2 sets of 2.
// Each set streams 64-row chunks of a2 and dout16 through LDS (register-staged, double-buffered);
// a wave owns 32 of the group's 64 columns (two 16-column tiles) and all 64 rows of its set's chunk:
//   (1) P[token][j]  = a2 . W1^T   A = a2 rows (ds_read_b128), B = W1 rows (registers)
//   (2) D[token][j]  = do . W2     A = dout rows,               B = W2 columns (registers)
//   (4) dW2[dm][j]  += do^T . f    A = dout^T (ds_read_b64_tr_b16), B = f (P's accumulator layout)
//   (5) dW1[j][dm]  += dp^T . a2   A = dp (D's accumulator layout), B = a2 (ds_read_b64_tr_b16)
// With P / D in the C layout (lane: 4 consecutive tokens 4g..4g+3 of column c), two token tiles
// give an operand's 8 k-elements: element e of lane group g is token 16 (2s + e/4) + 4g + e%4 -
// the transposed reads of the other operand fetch exactly those tokens.  At the end the two sets'
// partials meet in LDS and the group's 2 x 64 x 64 dW tiles + biases go out as fp32 atomics (one
// set of atomics per slice: the launcher sizes slices for ~one workgroup per CU).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dct_common.h"
#include "kernels.h"

namespace dct {
namespace ttf {

constexpr int DM = 64, FF = 256, JW = 64, NJ = FF / JW, NSET = 2, WPS = 2, CH = 64;
constexpr int IMG = CH * DM * 2;                   // one 64 x 64 bf16 operand image (8 KB)
constexpr int LDS_BYTES = 2 * NSET * 2 * IMG;      // [stage][set][a2 | dout] = 64 KB
constexpr int MAXP = 4;

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

struct Prob {
  const uint16_t* a2;    // [M][64] bf16
  const uint16_t* dout;  // [M][64] bf16 (the block output's gradient, bf16-rounded)
  const uint16_t* w1;    // [256][64] bf16
  const uint16_t* w2;    // [64][256] bf16
  const float* b1;       // [256]
  float* dw1;            // [256][64] fp32, accumulated
  float* dw2;            // [64][256]
  float* db1;            // [256]
  float* db2;            // [64]
};
struct Args {
  Prob p[MAXP];
  int n, M, slices, steps;  // steps: chunk pairs per slice (rows per slice = steps * NSET * CH)
};

__device__ __forceinline__ f32x4 mfma32(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// byte offset of 16-byte chunk ch (0..7) of row r in a 128-byte-row image, XOR-swizzled by r & 7
__device__ __forceinline__ int img_off(int r, int ch) { return r * 128 + ((ch ^ (r & 7)) << 4); }

// A/B fragment of rows 16 i .. 16 i + 15, k = 32 ks + 8 g .. + 7 (row-major operand)
__device__ __forceinline__ bf16x8 row_frag(const char* img, int i, int ks, int c, int g) {
  return *reinterpret_cast<const bf16x8*>(img + img_off(16 * i + c, 4 * ks + g));
}

// transposed fragment: column 16 m + c of tokens 16 (2 s + e / 4) + 4 g + e % 4, e = 0..7
__device__ __forceinline__ bf16x8 tr_frag(const char* img, int m, int s, int c, int g) {
  const int q = c >> 2, p = c & 3, ch = 2 * m + (p >> 1);
  const int r0 = 32 * s + 4 * g + q, r1 = r0 + 16;
  typedef __attribute__((address_space(3))) bf16x4 lds4;
  const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4*)(img + img_off(r0, ch) + (p & 1) * 8));
  const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4*)(img + img_off(r1, ch) + (p & 1) * 8));
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

// bijective XCD-aware remap: consecutive work ids (the NJ column groups of one row slice, which
// read the same a2 / dout rows) land on one XCD and share its L2
__device__ __forceinline__ int xcd_id() {
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
}

__global__ __launch_bounds__(256, 1) void tt_ffn_dw_kernel(Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int w = xcd_id();
  const int per_p = NJ * a.slices;
  const int pi = w / per_p, rem = w - pi * per_p;
  const int slice = rem / NJ, J = rem - slice * NJ;
  const Prob& P = a.p[pi];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int set = wv / WPS, ws = wv % WPS, ts = ws * 64 + lane;  // thread index within the set
  const int c = lane & 15, g = lane >> 4;
  const int jb = J * JW + 32 * ws;  // this wave's first column
  const int rows_slice = a.steps * NSET * CH;
  const int row_s = slice * rows_slice;

  // weights of the wave's two column tiles, as B fragments: W1 rows / W2 columns (k = dm)
  bf16x8 w1f[2][2], w2f[2][2];
  float b1v[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int j = jb + 16 * t + c;
    b1v[t] = P.b1[j];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      w1f[t][ks] = *reinterpret_cast<const bf16x8*>(P.w1 + (size_t)j * DM + 32 * ks + 8 * g);
#pragma unroll
      for (int e = 0; e < 8; ++e) w2f[t][ks][e] = (short)P.w2[(size_t)(32 * ks + 8 * g + e) * FF + j];
    }
  }

  f32x4 dw2[4][2], dw1[2][4];  // [dm tile][j tile], [j tile][dm tile]
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int t = 0; t < 2; ++t) { dw2[i][t] = (f32x4){0.f, 0.f, 0.f, 0.f}; dw1[t][i] = (f32x4){0.f, 0.f, 0.f, 0.f}; }
  float db1p[2] = {0.f, 0.f}, db2p[4] = {0.f, 0.f, 0.f, 0.f};
  const bool do_db2 = J == 0 && ws == 0;  // one wave per set sums dout's columns

  auto img = [&](int stage, int op) -> char* { return smem + ((stage * NSET + set) * 2 + op) * IMG; };
  // a set's chunk: 2 images x 512 16-byte granules over its 128 threads = 8 per thread
  uint4 stg[8];
  auto load = [&](int step) {
    const int r0 = row_s + (step * NSET + set) * CH;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int gi = q * 128 + ts, op = gi >> 9, loc = gi & 511, r = loc >> 3, ch = loc & 7;
      const uint16_t* src = (op ? P.dout : P.a2) + (size_t)(r0 + r) * DM + ch * 8;
      stg[q] = *reinterpret_cast<const uint4*>(src);
    }
  };
  auto store = [&](int stage) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int gi = q * 128 + ts, op = gi >> 9, loc = gi & 511, r = loc >> 3, ch = loc & 7;
      *reinterpret_cast<uint4*>(img(stage, op) + img_off(r, ch)) = stg[q];
    }
  };

  load(0);
  store(0);
  __syncthreads();
  for (int st = 0; st < a.steps; ++st) {
    const int cur = st & 1;
    if (st + 1 < a.steps) load(st + 1);  // in flight under this chunk's MFMAs
    const char* A2 = img(cur, 0);
    const char* DO = img(cur, 1);
    // (1), (2): P / D tiles [token tile i][column tile t]
    f32x4 pa[4][2], da[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int t = 0; t < 2; ++t) { pa[i][t] = (f32x4){0.f, 0.f, 0.f, 0.f}; da[i][t] = pa[i][t]; }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bf16x8 af = row_frag(A2, i, ks, c, g), df = row_frag(DO, i, ks, c, g);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          pa[i][t] = mfma32(af, w1f[t][ks], pa[i][t]);
          da[i][t] = mfma32(df, w2f[t][ks], da[i][t]);
        }
      }
    // f and dp as operands: k-step s takes token tiles 2s (elements 0..3) and 2s + 1 (4..7)
    bf16x8 ff[2][2], dp[2][2];  // [s][t]
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float z = pa[2 * s + (e >> 2)][t][e & 3] + b1v[t];
          const uint16_t fb = f32_to_bf16(gelu_f(z));
          const uint16_t pb = f32_to_bf16(da[2 * s + (e >> 2)][t][e & 3] * gelu_grad_f(bf16_to_f32(f32_to_bf16(z))));
          ff[s][t][e] = (short)fb;
          dp[s][t][e] = (short)pb;
          db1p[t] += bf16_to_f32(pb);
        }
    // (4) dW2 += dout^T f ; (5) dW1 += dp^T a2
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 dt = tr_frag(DO, m, s, c, g), at = tr_frag(A2, m, s, c, g);
        if (do_db2) {
#pragma unroll
          for (int e = 0; e < 8; ++e) db2p[m] += bf16_to_f32((uint16_t)dt[e]);
        }
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          dw2[m][t] = mfma32(dt, ff[s][t], dw2[m][t]);
          dw1[t][m] = mfma32(dp[s][t], at, dw1[t][m]);
        }
      }
    if (st + 1 < a.steps) store(cur ^ 1);  // the other stage: last read before the previous barrier
    __syncthreads();
  }

  // the two sets' partials meet in LDS (set 1 writes, set 0 adds and issues the atomics)
  float* red = reinterpret_cast<float*>(smem) + ws * (64 * 70);  // per wave: 70 floats per lane
  if (set == 1) {
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          red[((m * 2 + t) * 4 + r) * 64 + lane] = dw2[m][t][r];
          red[(32 + (t * 4 + m) * 4 + r) * 64 + lane] = dw1[t][m][r];
        }
    red[64 * 64 + lane] = db1p[0];
    red[65 * 64 + lane] = db1p[1];
#pragma unroll
    for (int m = 0; m < 4; ++m) red[(66 + m) * 64 + lane] = db2p[m];
  }
  __syncthreads();
  if (set != 0) return;
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        dw2[m][t][r] += red[((m * 2 + t) * 4 + r) * 64 + lane];
        dw1[t][m][r] += red[(32 + (t * 4 + m) * 4 + r) * 64 + lane];
      }
  db1p[0] += red[64 * 64 + lane];
  db1p[1] += red[65 * 64 + lane];
#pragma unroll
  for (int m = 0; m < 4; ++m) db2p[m] += red[(66 + m) * 64 + lane];
  // C layouts: dw2[m][t][r] = dW2[dm 16m + 4g + r][j jb + 16t + c]; dw1[t][m][r] = dW1[j jb + 16t + 4g + r][dm 16m + c]
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        atomicAdd(P.dw2 + (size_t)(16 * m + 4 * g + r) * FF + jb + 16 * t + c, dw2[m][t][r]);
        atomicAdd(P.dw1 + (size_t)(jb + 16 * t + 4 * g + r) * DM + 16 * m + c, dw1[t][m][r]);
      }
  // biases: lanes c, c+16, c+32, c+48 hold partial sums of the same column
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    float v = db1p[t];
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    if (g == 0) atomicAdd(P.db1 + jb + 16 * t + c, v);
  }
  if (do_db2) {
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      float v = db2p[m];
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      if (g == 0) atomicAdd(P.db2 + 16 * m + c, v);
    }
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

}  // namespace ttf
}  // namespace dct

extern "C" {

// n (<= 4) blocks' FFN weight gradients over the same M rows (M % 128 == 0), accumulated into
// dw1 [256][64], dw2 [64][256], db1 [256], db2 [64] (fp32).  a2 / dout / w1: 16-byte aligned.
int dct_tt_ffn_dw(int n, const uint16_t* const* a2, const uint16_t* const* dout, const uint16_t* const* w1,
                  const uint16_t* const* w2, const float* const* b1, float* const* dw1, float* const* dw2,
                  float* const* db1, float* const* db2, int M, void* stream) {
  using namespace dct::ttf;
  if (n <= 0 || n > MAXP || M <= 0 || M % (NSET * CH)) return (int)hipErrorInvalidValue;
  Args a{};
  a.n = n;
  a.M = M;
  for (int i = 0; i < n; ++i) {
    if (!a2[i] || !dout[i] || !w1[i] || !w2[i] || !b1[i] || !dw1[i] || !dw2[i] || !db1[i] || !db2[i])
      return (int)hipErrorInvalidValue;
    if ((((uintptr_t)a2[i]) | ((uintptr_t)dout[i]) | ((uintptr_t)w1[i])) & 15) return (int)hipErrorInvalidValue;
    a.p[i] = Prob{a2[i], dout[i], w1[i], w2[i], b1[i], dw1[i], dw2[i], db1[i], db2[i]};
  }
  // row slices: about one workgroup per CU over all problems and column groups, each slice a
  // whole number of chunk pairs
  const int pairs = M / (NSET * CH);
  int slices = device_cus() / (n * NJ);
  slices = slices < 1 ? 1 : (slices > pairs ? pairs : slices);
  while (pairs % slices) --slices;
  a.slices = slices;
  a.steps = pairs / slices;
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)tt_ffn_dw_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                             LDS_BYTES);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  hipLaunchKernelGGL(tt_ffn_dw_kernel, dim3(n * NJ * slices), dim3(256), LDS_BYTES,
                     reinterpret_cast<hipStream_t>(stream), a);
  return (int)hipGetLastError();
}

}  // extern "C"
