// Adam riding in the dW GEMM launch (gemm2_dw_adam_kernel, csrc/gemm_bf16.hip): why did the float4
// Adam path (adam_flat_range, the compiler's packed v_pk_* fp32 math) update the LOW component of 16
// consecutive lanes with denom = eps while the GEMM's MFMA workgroups shared the CUs
// (profiles/adam_ride_debug_r5.log)?  This probe runs the production riding kernel's shape - the
// tabular 1024 x 1024 x 4096 split-K dW GEMM tiles plus 256 Adam workgroups over a 1 M-element range
// - with each Adam body, repeated from the same initial state, and compares every element of p / m / v
// against the one-launch scalar Adam (adam_scalar_range alone), bit for bit:
//   mode 0: float4 path (adam_flat_range) beside the GEMM tiles       (the r5 failure)
//   mode 1: scalar path (adam_scalar_range) beside the GEMM tiles     (the r5 fix)
//   mode 2: float4 path alone (no GEMM workgroups in the launch)
//   mode 3: float4 path, GEMM workgroups exit at once (same kernel, same code object, no MFMA work)
//   mode 4..7: float4 path beside SYNTHETIC tiles (MFMA chains; +1 LDS-DMA refills, +2 ds_read operands)
//   mode 8: the float4 Adam as its own launch on a second stream beside GEMM-only launches (cross-kernel)
//   mode 16 + SCAL: a copy of the float4 body with the sites in SCAL kept out of packing (adam4_probe);
//                   SCAL 16 / 32: the denominator paired by hand with / without op_sel on src1
// Build (tools/probes/build_adam_ride_probe.sh): once as is, once with -fno-slp-vectorize (no v_pk_*
// in the Adam body); run: adam_ride_probe <mode> <iterations>.
#include "gemm_bf16.hip"

// (gemm_bf16.hip's dct_gemm_bf16_ex references the bias / activation backward of nn_kernels.hip; never
// called here)
extern "C" int dct_bias_act_bwd(const void*, const void*, uint16_t*, float*, int, int, int, int, int, void*) {
  return (int)hipErrorNotSupported;
}

#include <cstdio>
#include <cstring>
#include <vector>

// A copy of adam_flat_range's float4 Adam (PARTS, no slices) whose per-element steps can be taken out of
// the compiler's packing one site at a time: each bit of SCAL computes that step for all four
// components with scalar v_fma_f32 / v_mul_f32 in inline asm (nothing left to pair):
//   1: m = b1 m + (1 - b1) g   2: v = b2 v + (1 - b2) g^2   4: denom = sqrt(v) rbc2 + eps   8: step_size * m
__device__ __forceinline__ float asm_fma(float a, float b, float c) {
  float r;
  asm volatile("v_fma_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float asm_mul(float a, float b) {
  float r;
  asm volatile("v_mul_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
template <int SCAL>
__device__ __forceinline__ void adam4_probe(float4& P, float4 G, float4& Mm, float4& V, const dct::AdamArgs& a) {
  float p[4] = {P.x, P.y, P.z, P.w}, g[4] = {G.x, G.y, G.z, G.w}, m[4] = {Mm.x, Mm.y, Mm.z, Mm.w},
        v[4] = {V.x, V.y, V.z, V.w}, d[4], u[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    g[i] *= a.grad_scale;
    g[i] += a.wd * p[i];
    m[i] = (SCAL & 1) ? asm_fma(a.b1, m[i], asm_mul(1.f - a.b1, g[i])) : a.b1 * m[i] + (1.f - a.b1) * g[i];
    v[i] = (SCAL & 2) ? asm_fma(a.b2, v[i], asm_mul(asm_mul(1.f - a.b2, g[i]), g[i]))
                      : a.b2 * v[i] + (1.f - a.b2) * g[i] * g[i];
  }
  float sq[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) sq[i] = sqrtf(v[i]);
  if constexpr (SCAL & 48) {
    // the denominator pairs by hand: 16 = the compiler's first-pass form (src1 = {step_size, rbc2},
    // op_sel picks rbc2 for the LOW half), 32 = src1 = {rbc2, rbc2}, no op_sel
    typedef float f2 __attribute__((ext_vector_type(2)));
    const f2 e2 = (f2){a.eps, a.eps};
    const f2 s1 = (SCAL & 16) ? (f2){a.step_size, a.rbc2} : (f2){a.rbc2, a.rbc2};
#pragma unroll
    for (int i = 0; i < 4; i += 2) {
      const f2 q = (f2){sq[i], sq[i + 1]};
      f2 r;
      if constexpr (SCAL & 16)
        asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[1,1,1]" : "=v"(r) : "v"(q), "v"(s1), "v"(e2));
      else
        asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(r) : "v"(q), "v"(s1), "v"(e2));
      d[i] = r.x;
      d[i + 1] = r.y;
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if constexpr (!(SCAL & 48)) d[i] = (SCAL & 4) ? asm_fma(sq[i], a.rbc2, a.eps) : sq[i] * a.rbc2 + a.eps;
    u[i] = (SCAL & 8) ? asm_mul(a.step_size, m[i]) : a.step_size * m[i];
    p[i] -= u[i] / d[i];
  }
  P = make_float4(p[0], p[1], p[2], p[3]);
  Mm = make_float4(m[0], m[1], m[2], m[3]);
  V = make_float4(v[0], v[1], v[2], v[3]);
}
template <int SCAL>
__device__ __forceinline__ void adam_probe_range(dct::AdamArgs a, int64_t lo, int64_t hi, int blk, int nblk) {
  bool pending = a.step_counter != nullptr;
  const int64_t n4 = (hi < a.n ? hi : a.n) >> 2;
  const int64_t stride = (int64_t)nblk * blockDim.x;
  float4* p4 = reinterpret_cast<float4*>(a.p);
  const float4* g4 = reinterpret_cast<const float4*>(a.g);
  float4* m4 = reinterpret_cast<float4*>(a.m);
  float4* v4 = reinterpret_cast<float4*>(a.v);
  for (int64_t i = (lo >> 2) + (int64_t)blk * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 p = p4[i], m = m4[i], v = v4[i], g = g4[i];
    if (pending) {
      dct::adam_bias_correction(a);
      pending = false;
    }
    adam4_probe<SCAL>(p, g, m, v, a);
    p4[i] = p;
    m4[i] = m;
    v4[i] = v;
  }
}

// synthetic stand-ins for the GEMM tiles (modes 4..7): 8 waves of back-to-back 16x16x32 bf16 MFMAs whose
// operands come from LDS (ds_read_b128), refilled by 16-B LDS-DMA (global_load_lds_dwordx4, M0 set in
// asm as the GEMM does) - ROLE bit 1: LDS-DMA refills, bit 2: ds_read operands (else registers)
template <int ROLE>
__device__ __forceinline__ void synth_tile(const uint16_t* src, float* sink) {
  extern __shared__ __attribute__((aligned(16))) char dyn[];
  typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
  typedef float f4 __attribute__((ext_vector_type(4)));
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  f4 acc[4];
  for (int j = 0; j < 4; ++j) acc[j] = (f4){0.f, 0.f, 0.f, 0.f};
  bf8 x = *reinterpret_cast<const bf8*>(src + (t & 1023) * 8), y = *reinterpret_cast<const bf8*>(src + ((t * 7) & 1023) * 8);
  for (int it = 0; it < 256; ++it) {
    if constexpr (ROLE & 1) {
      const uint16_t* g = src + (((it * 512 + t) * 8) & ((1 << 22) - 1));
      const uint32_t dst = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(dyn + ((it & 3) * 512 + wave * 64) * 16));
      uint32_t keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(g), "s"(dst) : "memory");
    }
    if constexpr (ROLE & 2) {
      x = *reinterpret_cast<const bf8*>(dyn + (((it + 1) & 3) * 512 + ((t * 5) & 511)) * 16);
      y = *reinterpret_cast<const bf8*>(dyn + (((it + 2) & 3) * 512 + ((t * 3) & 511)) * 16);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k & 3] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, y, acc[k & 3], 0, 0, 0);
    if constexpr (ROLE & 1) {
      if ((it & 3) == 3) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
    }
  }
  float r = 0.f;
  for (int j = 0; j < 4; ++j) r += acc[j][0] + acc[j][2];
  if (r == 1234.5f) sink[t] = r;
}

template <int MODE>
__global__ __launch_bounds__(512, 2) void ride_probe_kernel(dct::GemmArgs g, int splits, int gemm_wgs, dct::AdamArgs a,
                                                            int64_t lo, int64_t hi) {
  if ((int)blockIdx.x < gemm_wgs) {
    if constexpr (MODE == 3) return;
    if constexpr (MODE >= 4 && MODE <= 7) {  // synthetic tile role (MODE - 4 = ROLE bits)
      synth_tile<MODE - 4>(g.A, reinterpret_cast<float*>(g.C));
      return;
    }
    const int orig = blockIdx.x, xcd = orig & 7;
    const int q8 = gemm_wgs >> 3, r8 = gemm_wgs & 7;
    const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
    dct::gemm2_body<true, false, true, 128, 2, 4>(g, splits, wgid);
  } else if constexpr (MODE == 1) {
    dct::adam_scalar_range<true, 8>(a, lo, hi, blockIdx.x - gemm_wgs, gridDim.x - gemm_wgs);
  } else if constexpr (MODE >= 4 && MODE <= 7) {
    dct::adam_flat_range<true, 8>(a, lo, hi, blockIdx.x - gemm_wgs, gridDim.x - gemm_wgs);
  } else if constexpr (MODE >= 16) {  // the probe copy, sites (MODE - 16) scalarised
    adam_probe_range<MODE - 16>(a, lo, hi, blockIdx.x - gemm_wgs, gridDim.x - gemm_wgs);
  } else {
    dct::adam_flat_range<true, 8>(a, lo, hi, blockIdx.x - gemm_wgs, gridDim.x - gemm_wgs);
  }
}

__global__ void ref_kernel(dct::AdamArgs a, int64_t lo, int64_t hi) {
  dct::adam_scalar_range<true, 8>(a, lo, hi, blockIdx.x, gridDim.x);
}

// mode 8: the float4 (packed) Adam as its OWN launch on a second stream, concurrent with GEMM-only
// launches of the same tiles on the first stream - another kernel's packed fp32 beside the GEMM's
// LDS-DMA (what an RCCL reduce kernel on a DDP comm stream would be: RCCL's fp32 sum kernels use
// v_pk_add_f32)
__global__ __launch_bounds__(512) void flat4_kernel(dct::AdamArgs a, int64_t lo, int64_t hi) {
  dct::adam_flat_range<true, 8>(a, lo, hi, blockIdx.x, gridDim.x);
}

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                      \
    }                                                                                    \
  } while (0)

static uint32_t rng = 12345u;
static float frand() {
  rng = rng * 1664525u + 1013904223u;
  return ((rng >> 8) & 0xFFFFFF) / 16777216.0f - 0.5f;
}

int main(int argc, char** argv) {
  const int mode = argc > 1 ? std::atoi(argv[1]) : 0;
  const int iters = argc > 2 ? std::atoi(argv[2]) : 50;
  // the tabular step's middle dW: M = N = 1024 (dZ^T X over K = 4096 rows), 4 split-K slices
  const int M = 1024, N = 1024, K = 4096, splits = 4;
  const int64_t n = 1 << 20;  // Adam range: one 1024 x 1024 layer (W2 of the tabular model)
  std::vector<uint16_t> hz((size_t)K * M), hx((size_t)K * N);
  for (auto& h : hz) { float f = frand(); uint32_t u; std::memcpy(&u, &f, 4); h = (uint16_t)(u >> 16); }
  for (auto& h : hx) { float f = frand(); uint32_t u; std::memcpy(&u, &f, 4); h = (uint16_t)(u >> 16); }
  std::vector<float> hp(n), hg(n), hm(n), hv(n);
  for (int64_t i = 0; i < n; ++i) {
    hp[i] = 0.05f * frand();
    hg[i] = 1e-4f * frand();  // gradients of the tabular scale: v ~ 1e-13 .. 1e-15, below 2^-32 (sqrt rescaling path)
    hm[i] = 1e-5f * frand();
    hv[i] = 1e-12f * (frand() + 0.5f);
  }
  uint16_t *dz, *dx;
  float *part, *colsum, *p, *g, *m, *v, *rp, *rm, *rv;
  int* step;
  CK(hipMalloc(&dz, hz.size() * 2));
  CK(hipMalloc(&dx, hx.size() * 2));
  CK(hipMalloc(&part, (size_t)splits * M * N * 4));
  CK(hipMalloc(&colsum, (size_t)M * 4));
  for (float** b : {&p, &g, &m, &v, &rp, &rm, &rv}) CK(hipMalloc(b, n * 4));
  CK(hipMalloc(&step, 4));
  const int t = 3;
  CK(hipMemcpy(step, &t, 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dz, hz.data(), hz.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dx, hx.data(), hx.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(g, hg.data(), n * 4, hipMemcpyHostToDevice));
  auto reset = [&](float* P, float* Mm, float* V) {
    CK(hipMemcpy(P, hp.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(Mm, hm.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(V, hv.data(), n * 4, hipMemcpyHostToDevice));
  };
  dct::AdamRange r{};
  r.g = g; r.n = n; r.lr = 1e-3f; r.b1 = 0.9f; r.b2 = 0.999f; r.eps = 1e-8f; r.wd = 0.f; r.grad_scale = 1.f;
  r.step_counter = step; r.nparts = 0; r.lo = 0; r.hi = n;
  dct::AdamArgs a{};
  int max_sp = 1;
  // reference: the scalar Adam as its own launch
  reset(rp, rm, rv);
  r.p = rp; r.m = rm; r.v = rv;
  if (dct::adam_args_from_range(r, a, &max_sp)) return 3;
  hipLaunchKernelGGL(ref_kernel, dim3(256), dim3(512), 0, 0, a, (int64_t)0, n);
  CK(hipDeviceSynchronize());
  std::vector<float> ref_p(n), ref_m(n), ref_v(n), op(n), om(n), ov(n);
  CK(hipMemcpy(ref_p.data(), rp, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(ref_m.data(), rm, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(ref_v.data(), rv, n * 4, hipMemcpyDeviceToHost));

  dct::GemmArgs gg{};
  gg.A = dz; gg.B = dx; gg.C = part; gg.M = M; gg.N = N; gg.K = K; gg.lda = M; gg.ldb = N; gg.ldc = N;
  gg.epilogue = dct::EPI_NONE; gg.out_f32 = 1; gg.accumulate = 0; gg.alpha = 1.0f;
  gg.vec_a = 1; gg.vec_b = 1; gg.colsum = colsum; gg.split_part = part;
  const int tiles = (M / dct::GBM) * (N / dct::GBN);
  const int gemm_wgs = mode == 2 ? 0 : tiles * splits;
  const int adam_wgs = 256;
  r.p = p; r.m = m; r.v = v;
  if (dct::adam_args_from_range(r, a, &max_sp)) return 3;
  const size_t lds = 4 * dct::G2_BYTES;
  void (*fn)(dct::GemmArgs, int, int, dct::AdamArgs, int64_t, int64_t) =
      mode == 0 || mode == 2 ? ride_probe_kernel<0> : (mode == 1 ? ride_probe_kernel<1> : ride_probe_kernel<3>);
  switch (mode) {  // 16 + SCAL: the probe copy of the float4 body beside the GEMM tiles
    case 4: fn = ride_probe_kernel<4>; break;   // float4 Adam beside synthetic MFMA tiles (register operands)
    case 5: fn = ride_probe_kernel<5>; break;   // ... + LDS-DMA refills
    case 6: fn = ride_probe_kernel<6>; break;   // ... operands by ds_read_b128, no LDS-DMA
    case 7: fn = ride_probe_kernel<7>; break;   // ... LDS-DMA + ds_read_b128 (the GEMM's traffic)
    case 16: fn = ride_probe_kernel<16>; break;
    case 17: fn = ride_probe_kernel<17>; break;
    case 18: fn = ride_probe_kernel<18>; break;
    case 20: fn = ride_probe_kernel<20>; break;
    case 24: fn = ride_probe_kernel<24>; break;
    case 31: fn = ride_probe_kernel<31>; break;
    case 32: fn = ride_probe_kernel<32>; break;   // 16 + 16: hand-paired denominator with op_sel
    case 48: fn = ride_probe_kernel<48>; break;   // 16 + 32: hand-paired denominator, no op_sel
    default: break;
  }
  CK(hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  CK(hipFuncSetAttribute((const void*)ride_probe_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  long long bad_total = 0, bad_iters = 0;
  hipStream_t sa = 0, sb = 0;
  if (mode == 8) {
    CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
  }
  for (int it = 0; it < iters; ++it) {
    reset(p, m, v);
    if (mode == 8) {
      // GEMM tiles alone (no Adam workgroups) back to back on stream A; the packed Adam on stream B
      // starts once the first GEMM launch is running
      for (int k = 0; k < 4; ++k)
        hipLaunchKernelGGL(ride_probe_kernel<1>, dim3(gemm_wgs), dim3(512), lds, sa, gg, splits, gemm_wgs, a, (int64_t)0,
                           (int64_t)0);
      hipLaunchKernelGGL(flat4_kernel, dim3(256), dim3(512), 0, sb, a, (int64_t)0, n);
      CK(hipGetLastError());
      CK(hipDeviceSynchronize());
    } else
    hipLaunchKernelGGL(fn, dim3(gemm_wgs + adam_wgs), dim3(512), lds, 0, gg, splits, gemm_wgs, a, (int64_t)0, n);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(op.data(), p, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(om.data(), m, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(ov.data(), v, n * 4, hipMemcpyDeviceToHost));
    long long bp = 0, bm = 0, bv = 0;
    int64_t first = -1;
    int comp_hist[4] = {0, 0, 0, 0}, pass_hist[2] = {0, 0};
    for (int64_t i = 0; i < n; ++i) {
      if (std::memcmp(&op[i], &ref_p[i], 4)) {
        ++bp;
        ++pass_hist[(i >> 2) >= 256 * 512 ? 1 : 0];
        ++comp_hist[i & 3];
        if (first < 0) first = i;
      }
      bm += std::memcmp(&om[i], &ref_m[i], 4) != 0;
      bv += std::memcmp(&ov[i], &ref_v[i], 4) != 0;
    }
    if (bp || bm || bv) {
      ++bad_iters;
      bad_total += bp;
      double ratio = 0.0;
      if (first >= 0) ratio = (op[first] - hp[first]) / (double)(ref_p[first] - hp[first]);
      std::printf("iter %d: p %lld m %lld v %lld differ; p by component x/y/z/w %d/%d/%d/%d; first %lld "
                  "(update ratio %.1f, v %.3e); first / later loop pass %d / %d\n",
                  it, bp, bm, bv, comp_hist[0], comp_hist[1], comp_hist[2], comp_hist[3], (long long)first, ratio,
                  first >= 0 ? ref_v[first] : 0.f, pass_hist[0], pass_hist[1]);
    }
  }
  std::printf("mode %d: %lld of %d launches differ from the scalar one-launch Adam, %lld p elements in all\n", mode,
              bad_iters, iters, bad_total);
  return 0;
}
