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

template <int MODE>
__global__ __launch_bounds__(512, 2) void ride_probe_kernel(dct::GemmArgs g, int splits, int gemm_wgs, dct::AdamArgs a,
                                                            int64_t lo, int64_t hi) {
  if ((int)blockIdx.x < gemm_wgs) {
    if constexpr (MODE == 3) return;
    const int orig = blockIdx.x, xcd = orig & 7;
    const int q8 = gemm_wgs >> 3, r8 = gemm_wgs & 7;
    const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
    dct::gemm2_body<true, false, true, 128, 2, 4>(g, splits, wgid);
  } else if constexpr (MODE == 1) {
    dct::adam_scalar_range<true, 8>(a, lo, hi, blockIdx.x - gemm_wgs, gridDim.x - gemm_wgs);
  } else {
    dct::adam_flat_range<true, 8>(a, lo, hi, blockIdx.x - gemm_wgs, gridDim.x - gemm_wgs);
  }
}

__global__ void ref_kernel(dct::AdamArgs a, int64_t lo, int64_t hi) {
  dct::adam_scalar_range<true, 8>(a, lo, hi, blockIdx.x, gridDim.x);
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
  CK(hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  long long bad_total = 0, bad_iters = 0;
  for (int it = 0; it < iters; ++it) {
    reset(p, m, v);
    hipLaunchKernelGGL(fn, dim3(gemm_wgs + adam_wgs), dim3(512), lds, 0, gg, splits, gemm_wgs, a, (int64_t)0, n);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(op.data(), p, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(om.data(), m, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(ov.data(), v, n * 4, hipMemcpyDeviceToHost));
    long long bp = 0, bm = 0, bv = 0;
    int64_t first = -1;
    int comp_hist[4] = {0, 0, 0, 0};
    for (int64_t i = 0; i < n; ++i) {
      if (std::memcmp(&op[i], &ref_p[i], 4)) {
        ++bp;
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
                  "(update ratio %.1f, v %.3e)\n",
                  it, bp, bm, bv, comp_hist[0], comp_hist[1], comp_hist[2], comp_hist[3], (long long)first, ratio,
                  first >= 0 ? ref_v[first] : 0.f);
    }
  }
  std::printf("mode %d: %lld of %d launches differ from the scalar one-launch Adam, %lld p elements in all\n", mode,
              bad_iters, iters, bad_total);
  return 0;
}
