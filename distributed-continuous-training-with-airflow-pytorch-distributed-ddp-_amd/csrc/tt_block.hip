// Whole-block fused forward of the TabTransformer layer (BASELINE.json config 5: 64 feature
// tokens, d_model 64, 4 heads of 16, FFN 256) - one workgroup per sample, every intermediate in LDS.
//
//   h1  = h  + Wo  Attn(Wqkv LN1(h) + bqkv) + bo
//   out = h1 + W2 gelu(W1 LN2(h1) + b1) + b2
//
// The unfused path is 7 kernels per layer (LN, QKV GEMM, attention, proj GEMM, LN, fc1, fc2), each
// a full HBM round trip of a [B*64, <=256] activation plus a launch: ~65 us per layer at batch 512
// on MI355X, of which the math is < 2 us.  Here a sample's 64 x 64 residual rows are read once,
// all seven stages run out of 68 KB of LDS (2 workgroups per CU), weights come from L2 (96 KB
// shared by every workgroup), and only the tensors the backward consumes are written - staged
// through LDS so every global store is a 16-byte coalesced chunk.  Same saved-tensor contract as
// the two unfused autograd nodes (ops/nn.py _PreNormAttnFn / _PreNormFFNFn), so the backward is
// unchanged.
//
// Work split (4 waves): LayerNorms and row-parallel GEMMs (proj, fc1, fc2) - wave w owns token
// rows 16w..16w+15; QKV GEMM + attention - wave w owns head w (its Q/K/V columns for all 64
// tokens), so attention never leaves the wave's registers and LDS rows.
// MFMA layouts: v_mfma_f32_16x16x32_bf16 (A: row = lane&15, k = 8*(lane>>4)+j; B likewise with
// col; C: col = lane&15, row = 4*(lane>>4)+r); attention uses the 16x16x16 form (head dim 16).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dct_common.h"

namespace dct {
namespace ttb {

constexpr int T = 64, DM = 64, NH = 4, DH = 16, FF = 256;
constexpr int HS_LD = DM + 4;       // fp32 residual rows (272 B)
constexpr int AS_LD = DM + 8;       // bf16 LN output / attention output rows (144 B)
constexpr int QKV_LD = 3 * DM + 8;  // bf16 (400 B)
constexpr int F_LD = FF + 8;        // bf16 (528 B)
constexpr int HS_BYTES = T * HS_LD * 4;
constexpr int AS_BYTES = T * AS_LD * 2;
constexpr int R_BYTES = T * F_LD * 2;  // QKV (25.6 KB) then FFN hidden (33.8 KB)
constexpr int LDS_BYTES = HS_BYTES + 2 * AS_BYTES + R_BYTES;

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma32(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16(bf16x4 a, bf16x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float sum4g(float v) {  // over lanes l, l^16, l^32, l^48
  v += __shfl_xor(v, 16);
  v += __shfl_xor(v, 32);
  return v;
}
__device__ __forceinline__ float max4g(float v) {
  v = fmaxf(v, __shfl_xor(v, 16));
  v = fmaxf(v, __shfl_xor(v, 32));
  return v;
}
__device__ __forceinline__ bf16x4 pack4(f32x4 v) {
  bf16x4 r;
  r[0] = (short)f32_to_bf16(v[0]); r[1] = (short)f32_to_bf16(v[1]);
  r[2] = (short)f32_to_bf16(v[2]); r[3] = (short)f32_to_bf16(v[3]);
  return r;
}

struct Args {
  const float* h;
  const float *ln1_w, *ln1_b;
  const uint16_t* wqkv; const float* bqkv;
  const uint16_t* wo; const float* bo;
  const float *ln2_w, *ln2_b;
  const uint16_t* w1; const float* b1;
  const uint16_t* w2; const float* b2;
  uint16_t* a1; float* mean1; float* rstd1;
  uint16_t* qkv; uint16_t* o; float* lse;
  float* h1;
  uint16_t* a2; float* mean2; float* rstd2;
  uint16_t* f; uint16_t* pre;
  float* out;
  int B;
  float eps, scale;
};

// 64-row LDS tile -> contiguous global rows, 16-byte chunks over the whole workgroup
template <int ROW_BYTES, int LD_BYTES>
__device__ __forceinline__ void store_tile(void* g, const void* s) {
  constexpr int CPR = ROW_BYTES / 16;
  for (int idx = threadIdx.x; idx < T * CPR; idx += 256) {
    const int r = idx / CPR, c = idx - r * CPR;
    *reinterpret_cast<uint4*>(reinterpret_cast<char*>(g) + r * ROW_BYTES + c * 16) =
        *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(s) + r * LD_BYTES + c * 16);
  }
}

// LayerNorm of the wave's 16 rows: lane -> row 16w + (lane&15), columns 16g..16g+15.
// Input fp32 from `src` (global when from_global, else the LDS residual tile); the fp32 row is
// (re)written to HS, the bf16 normalised row to AS.
__device__ __forceinline__ void layer_norm_rows(const float* src, bool from_global, float* HS, uint16_t* AS,
                                                const float* w, const float* b, float* mean_out, float* rstd_out,
                                                int row0, float eps) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r = 16 * wv + (lane & 15), g = lane >> 4;
  float v[16];
  const float* p = from_global ? src + (size_t)(row0 + r) * DM + 16 * g : HS + r * HS_LD + 16 * g;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 t = reinterpret_cast<const float4*>(p)[q];
    v[4 * q] = t.x; v[4 * q + 1] = t.y; v[4 * q + 2] = t.z; v[4 * q + 3] = t.w;
  }
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < 16; ++e) s += v[e];
  const float mean = sum4g(s) * (1.f / DM);
  float qv = 0.f;
#pragma unroll
  for (int e = 0; e < 16; ++e) { const float d = v[e] - mean; qv += d * d; }
  const float rstd = rsqrtf(sum4g(qv) * (1.f / DM) + eps);
  if (from_global) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      reinterpret_cast<float4*>(HS + r * HS_LD + 16 * g)[q] = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
  }
  float wv4[16], bv4[16];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 tw = reinterpret_cast<const float4*>(w + 16 * g)[q];
    const float4 tb = reinterpret_cast<const float4*>(b + 16 * g)[q];
    wv4[4 * q] = tw.x; wv4[4 * q + 1] = tw.y; wv4[4 * q + 2] = tw.z; wv4[4 * q + 3] = tw.w;
    bv4[4 * q] = tb.x; bv4[4 * q + 1] = tb.y; bv4[4 * q + 2] = tb.z; bv4[4 * q + 3] = tb.w;
  }
  bf16x8 o0, o1;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    o0[e] = (short)f32_to_bf16((v[e] - mean) * rstd * wv4[e] + bv4[e]);
    o1[e] = (short)f32_to_bf16((v[e + 8] - mean) * rstd * wv4[e + 8] + bv4[e + 8]);
  }
  *reinterpret_cast<bf16x8*>(AS + r * AS_LD + 16 * g) = o0;
  *reinterpret_cast<bf16x8*>(AS + r * AS_LD + 16 * g + 8) = o1;
  if (g == 0) {
    mean_out[row0 + r] = mean;
    rstd_out[row0 + r] = rstd;
  }
}

__global__ __launch_bounds__(256, 2) void tt_block_fwd_kernel(Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* HS = reinterpret_cast<float*>(smem);
  uint16_t* AS = reinterpret_cast<uint16_t*>(smem + HS_BYTES);
  uint16_t* OS = reinterpret_cast<uint16_t*>(smem + HS_BYTES + AS_BYTES);
  uint16_t* RS = reinterpret_cast<uint16_t*>(smem + HS_BYTES + 2 * AS_BYTES);
  const int bidx = blockIdx.x;
  const int row0 = bidx * T;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = lane & 15, g = lane >> 4;

  // ---- P1: LN1 (rows of this wave)
  layer_norm_rows(a.h, true, HS, AS, a.ln1_w, a.ln1_b, a.mean1, a.rstd1, row0, a.eps);
  __syncthreads();

  // ---- P2: a1 out; QKV = a1 Wqkv^T + bqkv for head wv (Q, K, V column tiles wv, 4+wv, 8+wv)
  store_tile<DM * 2, AS_LD * 2>(a.a1 + (size_t)row0 * DM, AS);
  {
    f32x4 acc[3][4];
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[t][i] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < DM / 32; ++ks) {
      bf16x8 bw[3], af[4];
#pragma unroll
      for (int t = 0; t < 3; ++t)
        bw[t] = *reinterpret_cast<const bf16x8*>(a.wqkv + (size_t)(t * DM + DH * wv + c) * DM + 32 * ks + 8 * g);
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const bf16x8*>(AS + (16 * i + c) * AS_LD + 32 * ks + 8 * g);
#pragma unroll
      for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[t][i] = mfma32(af[i], bw[t], acc[t][i]);
    }
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const int col = t * DM + DH * wv + c;
      const float bv = a.bqkv[col];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) RS[(16 * i + 4 * g + r) * QKV_LD + col] = f32_to_bf16(acc[t][i][r] + bv);
    }
  }
  __syncthreads();

  // ---- P3: qkv out; attention of head wv over the 64 tokens (S^T = K Q^T; P V)
  store_tile<3 * DM * 2, QKV_LD * 2>(a.qkv + (size_t)row0 * 3 * DM, RS);
  {
    const uint16_t* Qs = RS + DH * wv;
    const uint16_t* Ks = RS + DM + DH * wv;
    const uint16_t* Vs = RS + 2 * DM + DH * wv;
    f32x4 st[4][4];
    bf16x4 kf[4], qf[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      kf[i] = *reinterpret_cast<const bf16x4*>(Ks + (16 * i + c) * QKV_LD + 4 * g);
      qf[i] = *reinterpret_cast<const bf16x4*>(Qs + (16 * i + c) * QKV_LD + 4 * g);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) st[i][j] = mfma16(kf[i], qf[j], (f32x4){0.f, 0.f, 0.f, 0.f});
    bf16x4 pf[4][4];
    float lsev[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float m = -3.402823466e+38f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) m = fmaxf(m, st[i][j][r]);
      m = max4g(m) * a.scale;
      float l = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = __expf(st[i][j][r] * a.scale - m);
          st[i][j][r] = e;
          l += e;
        }
      l = sum4g(l);
      const float inv = 1.f / l;
#pragma unroll
      for (int i = 0; i < 4; ++i) pf[j][i] = pack4(st[i][j] * inv);
      lsev[j] = m + __logf(l);
    }
    bf16x4 vf[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint16_t* vp = Vs + (16 * i + 4 * g) * QKV_LD + c;
      vf[i][0] = (short)vp[0]; vf[i][1] = (short)vp[QKV_LD];
      vf[i][2] = (short)vp[2 * QKV_LD]; vf[i][3] = (short)vp[3 * QKV_LD];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 4; ++i) acc = mfma16(pf[j][i], vf[i], acc);
#pragma unroll
      for (int r = 0; r < 4; ++r) OS[(16 * j + 4 * g + r) * AS_LD + DH * wv + c] = f32_to_bf16(acc[r]);
    }
    if (g == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) a.lse[((size_t)bidx * NH + wv) * T + 16 * j + c] = lsev[j];
    }
  }
  __syncthreads();

  // ---- P4: o out; h1 = h + o Wo^T + bo (rows of this wave); LN2 of the same rows
  store_tile<DM * 2, AS_LD * 2>(a.o + (size_t)row0 * DM, OS);
  {
    f32x4 acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < DM / 32; ++ks) {
      const bf16x8 af = *reinterpret_cast<const bf16x8*>(OS + (16 * wv + c) * AS_LD + 32 * ks + 8 * g);
#pragma unroll
      for (int t = 0; t < 4; ++t)
        acc[t] = mfma32(af, *reinterpret_cast<const bf16x8*>(a.wo + (size_t)(16 * t + c) * DM + 32 * ks + 8 * g), acc[t]);
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int col = 16 * t + c;
      const float bv = a.bo[col];
#pragma unroll
      for (int r = 0; r < 4; ++r) HS[(16 * wv + 4 * g + r) * HS_LD + col] += acc[t][r] + bv;
    }
  }
  layer_norm_rows(nullptr, false, HS, AS, a.ln2_w, a.ln2_b, a.mean2, a.rstd2, row0, a.eps);
  __syncthreads();

  // ---- P5: h1, a2 out; F = gelu(a2 W1^T + b1) (rows of this wave), pre-activation out
  store_tile<DM * 4, HS_LD * 4>(a.h1 + (size_t)row0 * DM, HS);
  store_tile<DM * 2, AS_LD * 2>(a.a2 + (size_t)row0 * DM, AS);
  {
    f32x4 acc[FF / 16];
#pragma unroll
    for (int t = 0; t < FF / 16; ++t) acc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < DM / 32; ++ks) {
      const bf16x8 af = *reinterpret_cast<const bf16x8*>(AS + (16 * wv + c) * AS_LD + 32 * ks + 8 * g);
#pragma unroll
      for (int t = 0; t < FF / 16; ++t)
        acc[t] = mfma32(af, *reinterpret_cast<const bf16x8*>(a.w1 + (size_t)(16 * t + c) * DM + 32 * ks + 8 * g), acc[t]);
    }
    uint16_t* pre = a.pre + (size_t)(row0 + 16 * wv + 4 * g) * FF;
#pragma unroll
    for (int t = 0; t < FF / 16; ++t) {
      const int col = 16 * t + c;
      const float bv = a.b1[col];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float z = acc[t][r] + bv;
        pre[r * FF + col] = f32_to_bf16(z);
        RS[(16 * wv + 4 * g + r) * F_LD + col] = f32_to_bf16(gelu_f(z));
      }
    }
  }
  __syncthreads();

  // ---- P6: f out; out = h1 + F W2^T + b2 (rows of this wave)
  store_tile<FF * 2, F_LD * 2>(a.f + (size_t)row0 * FF, RS);
  {
    f32x4 acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < FF / 32; ++ks) {
      const bf16x8 af = *reinterpret_cast<const bf16x8*>(RS + (16 * wv + c) * F_LD + 32 * ks + 8 * g);
#pragma unroll
      for (int t = 0; t < 4; ++t)
        acc[t] = mfma32(af, *reinterpret_cast<const bf16x8*>(a.w2 + (size_t)(16 * t + c) * FF + 32 * ks + 8 * g), acc[t]);
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int col = 16 * t + c;
      const float bv = a.b2[col];
#pragma unroll
      for (int r = 0; r < 4; ++r) HS[(16 * wv + 4 * g + r) * HS_LD + col] += acc[t][r] + bv;
    }
  }
  __syncthreads();
  store_tile<DM * 4, HS_LD * 4>(a.out + (size_t)row0 * DM, HS);
}

}  // namespace ttb
}  // namespace dct

extern "C" {

// ptrs (26, in order): h, ln1_w, ln1_b, wqkv, bqkv, wo, bo, ln2_w, ln2_b, w1, b1, w2, b2,
//   a1, mean1, rstd1, qkv, o, lse, h1, a2, mean2, rstd2, f, pre, out
int dct_tt_block_fwd(const uintptr_t* p, int n_ptrs, int Bsz, int T, int DM, int H, int FF, float eps, float scale,
                     void* stream) {
  using namespace dct::ttb;
  if (n_ptrs != 26 || T != dct::ttb::T || DM != dct::ttb::DM || H != NH || FF != dct::ttb::FF || Bsz <= 0)
    return (int)hipErrorInvalidValue;
  uintptr_t any = 0;
  for (int i = 0; i < n_ptrs; ++i) {
    if (!p[i]) return (int)hipErrorInvalidValue;
    any |= p[i];
  }
  if (any & 15) return (int)hipErrorInvalidValue;  // 16-byte vector loads / stores everywhere
  Args a;
  a.h = (const float*)p[0]; a.ln1_w = (const float*)p[1]; a.ln1_b = (const float*)p[2];
  a.wqkv = (const uint16_t*)p[3]; a.bqkv = (const float*)p[4];
  a.wo = (const uint16_t*)p[5]; a.bo = (const float*)p[6];
  a.ln2_w = (const float*)p[7]; a.ln2_b = (const float*)p[8];
  a.w1 = (const uint16_t*)p[9]; a.b1 = (const float*)p[10];
  a.w2 = (const uint16_t*)p[11]; a.b2 = (const float*)p[12];
  a.a1 = (uint16_t*)p[13]; a.mean1 = (float*)p[14]; a.rstd1 = (float*)p[15];
  a.qkv = (uint16_t*)p[16]; a.o = (uint16_t*)p[17]; a.lse = (float*)p[18];
  a.h1 = (float*)p[19]; a.a2 = (uint16_t*)p[20]; a.mean2 = (float*)p[21]; a.rstd2 = (float*)p[22];
  a.f = (uint16_t*)p[23]; a.pre = (uint16_t*)p[24]; a.out = (float*)p[25];
  a.B = Bsz; a.eps = eps; a.scale = scale;
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)tt_block_fwd_kernel,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  hipLaunchKernelGGL(tt_block_fwd_kernel, dim3(Bsz), dim3(256), LDS_BYTES, reinterpret_cast<hipStream_t>(stream), a);
  return (int)hipGetLastError();
}

}  // extern "C"
