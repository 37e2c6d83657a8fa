// Main-loop probe for the tabular MLP's bf16 GEMM shape (4096 x 1024 x 1024, A [M][K], B [N][K]):
// where does a k-step of the LDS-DMA pipeline spend its time when the grid holds ONE 128 x 128
// tile per CU (profiles/gemm_probe_r4.log)?
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/gemm_probe.hip -o build/gemm_probe
//   ./build/gemm_probe [M N K]
//
// Variants (tile BM x BN, WM x WN waves, S LDS stages = S - 1 k-tiles in flight):
//   MODE 0  the full loop;  MODE 1  no MFMA (global -> LDS -> fragments only);
//   MODE 2  no global loads in the loop (MFMAs on the prologue's stages).
// PROF instantiations add s_memtime stamps per wave: cycles waiting for the stage (vmcnt),
// at the barrier, and issuing fills + fragment reads + MFMAs.
// Standalone: no framework code; the production kernel is csrc/gemm_bf16.hip.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__);         \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

// KB: k per stage (64 or 128); an image row is 2 KB bytes = KB / 8 chunks of 16 B

__host__ __device__ inline uint16_t f2bf(float f) {
  uint32_t u = __builtin_bit_cast(uint32_t, f);
  u += 0x7fff + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}
__host__ __device__ inline float bf2f(uint16_t h) {
  return __builtin_bit_cast(float, (uint32_t)h << 16);
}

// ROWS x KB bf16 image, row r's 16-B chunk c stored at physical chunk c ^ (r & (CPR - 1)) (conflict-free
// ds_read_b128 fragments); the DMA writes lane-linear LDS, so the swizzle is on the source address
template <int ROWS, int NT, int KB>
__device__ __forceinline__ void fill(const uint16_t* __restrict__ G, int ld, int r0, int k0, char* img, int tid) {
  constexpr int CPR = KB / 8;
  constexpr int CH = ROWS * CPR / NT;
  static_assert(CH >= 1 && CH * NT == ROWS * CPR, "whole chunks per thread");
  const int wave = tid >> 6, lane = tid & 63;
#pragma unroll
  for (int q = 0; q < CH; ++q) {
    const int L = q * NT + wave * 64 + lane;
    const int r = L / CPR, c = (L % CPR) ^ (r & (CPR - 1));
    const uint16_t* src = G + (size_t)(r0 + r) * ld + k0 + c * 8;
    const uint32_t dst =
        __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void*)(img + (q * NT + wave * 64) * 16));
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(dst)
                 : "memory");
  }
}

template <int KB>
__device__ __forceinline__ bf16x8 frag(const char* img, int rb, int ks, int lane) {
  constexpr int CPR = KB / 8;
  const int row = rb + (lane & 15);
  const int c = ks * 4 + (lane >> 4);
  return *reinterpret_cast<const bf16x8*>(img + row * (2 * KB) + ((c ^ (row & (CPR - 1))) << 4));
}

template <int F>
__device__ __forceinline__ void wait_newer(int newer) {  // stage landed: <= newer * F loads pending
  if (newer <= 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if (newer == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(F) : "memory");
  else if (newer == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * F) : "memory");
  else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * F) : "memory");
}

__device__ __forceinline__ unsigned long long stamp() { return __builtin_amdgcn_s_memtime(); }

// LW > 0: producer / consumer - WM x WN compute waves never issue a load, LW loader waves only
// fill stages (they wait for their own DMA before the shared barrier)
template <int BM, int BN, int WM, int WN, int S, int MODE, bool PROF, int LW = 0, int KB = 64>
__global__ __launch_bounds__(64 * (WM * WN + LW)) void probe_gemm(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B,
                                                         uint16_t* __restrict__ C, int M, int N, int K,
                                                         unsigned long long* __restrict__ prof, int ld) {
  constexpr int NC = 64 * WM * WN;          // compute threads
  constexpr int LNT = LW > 0 ? 64 * LW : NC;  // loading threads
  constexpr int IM = BM / WM / 16, JN = BN / WN / 16;
  constexpr int IMG_A = BM * 2 * KB, STAGE = (BM + BN) * 2 * KB;
  constexpr int F = (BM + BN) * (KB / 8) / LNT;  // LDS-DMA instructions per loading thread per stage
  static_assert(S >= 2 && S <= 4 && 3 * F <= 63, "vmcnt range");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int tiles_n = N / BN;
  const int m0 = (wg / tiles_n) * BM, n0 = (wg % tiles_n) * BN;
  const int nk = K / KB;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const bool is_loader = LW > 0 && wave >= WM * WN;
  const bool does_load = LW == 0 || is_loader, does_mma = LW == 0 || !is_loader;
  const int ltid = LW > 0 ? (int)threadIdx.x - NC : (int)threadIdx.x;
  const int wr = (wave % (WM * WN)) / WN, wc = wave % WN;
  f32x4 acc[IM][JN];
#pragma unroll
  for (int i = 0; i < IM; ++i)
#pragma unroll
    for (int j = 0; j < JN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  auto fill_stage = [&](int s, int kt) {
    char* base = smem + s * STAGE;
    fill<BM, LNT, KB>(A, ld, m0, kt * KB, base, ltid);
    fill<BN, LNT, KB>(B, ld, n0, kt * KB, base + IMG_A, ltid);
  };
  unsigned long long t_wait = 0, t_bar = 0, t_comp = 0;
  const unsigned long long t_start = PROF ? stamp() : 0ull;
#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < nk && does_load) fill_stage(s, s);
  for (int it = 0; it < nk; ++it) {
    const unsigned long long t0 = PROF ? stamp() : 0ull;
    if (does_load) {
      if (MODE != 2) wait_newer<F>(min(S - 2, nk - 1 - it));
      else if (it == 0) wait_newer<F>(0);
    }
    const unsigned long long t1 = PROF ? stamp() : 0ull;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const unsigned long long t2 = PROF ? stamp() : 0ull;
    if (MODE != 2 && does_load && it + S - 1 < nk) fill_stage((it + S - 1) % S, it + S - 1);
    const int cur = MODE == 2 ? it % (S - 1) : it % S;
    const char* ai = smem + cur * STAGE;
    const char* bi = ai + IMG_A;
#pragma unroll
    for (int ks = 0; ks < KB / 32; ++ks) {
      if (!does_mma) break;
      bf16x8 af[IM], bfr[JN];
#pragma unroll
      for (int i = 0; i < IM; ++i) af[i] = frag<KB>(ai, wr * (BM / WM) + i * 16, ks, lane);
#pragma unroll
      for (int j = 0; j < JN; ++j) bfr[j] = frag<KB>(bi, wc * (BN / WN) + j * 16, ks, lane);
#pragma unroll
      for (int i = 0; i < IM; ++i)
#pragma unroll
        for (int j = 0; j < JN; ++j) {
          if (MODE == 1) acc[i][j][0] += (float)(af[i][ks] ^ bfr[j][ks + 1]);
          else acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
        }
    }
    if (PROF) {
      const unsigned long long t3 = stamp();
      t_wait += t1 - t0;
      t_bar += t2 - t1;
      t_comp += t3 - t2;
    }
  }
  // swapped operands: lane holds row 16i + (lane & 15), columns 16j + 4 (lane >> 4) .. + 3
#pragma unroll
  for (int i = 0; i < IM; ++i) {
    if (!does_mma) break;
    const int row = m0 + wr * (BM / WM) + i * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < JN; ++j) {
      const int col = n0 + wc * (BN / WN) + j * 16 + 4 * (lane >> 4);
      uint2 pk;
      pk.x = f2bf(acc[i][j][0]) | ((uint32_t)f2bf(acc[i][j][1]) << 16);
      pk.y = f2bf(acc[i][j][2]) | ((uint32_t)f2bf(acc[i][j][3]) << 16);
      *reinterpret_cast<uint2*>(C + (size_t)row * N + col) = pk;
    }
  }
  if (PROF) {
    const unsigned long long t_end = stamp();
    if (lane == 0 && does_mma) {  // compute waves only
      unsigned long long* p = prof + ((size_t)wg * (WM * WN) + wave) * 4;
      p[0] = t_end - t_start;
      p[1] = t_wait;
      p[2] = t_bar;
      p[3] = t_comp;
    }
  }
}

// fp32 reference of sampled entries
__global__ void ref_entries(const uint16_t* A, const uint16_t* B, const int* rows, const int* cols, float* out, int n,
                            int K, int ld) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const uint16_t* a = A + (size_t)rows[e] * ld;
  const uint16_t* b = B + (size_t)cols[e] * ld;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += bf2f(a[k]) * bf2f(b[k]);
  out[e] = s;
}

struct Ctx {
  int M, N, K;
  uint16_t *A, *B, *C, *Ap, *Bp;  // Ap / Bp: the same operands with padded rows (ld = K + 64)
  unsigned long long* prof;
  int *rows, *cols;
  float* ref;
  std::vector<int> hr, hc;
  std::vector<float> href;
  hipStream_t st;
};

template <int BM, int BN, int WM, int WN, int S, int MODE, int LW = 0, int KB = 64>
void run(Ctx& c, const char* name, int iters, bool padded = false) {
  const uint16_t* A = padded ? c.Ap : c.A;
  const uint16_t* B = padded ? c.Bp : c.B;
  const int ld = padded ? c.K + 64 : c.K;
  if (c.M % BM || c.N % BN || c.K % KB) {
    printf("{\"variant\": \"%s\", \"skipped\": \"shape\"}\n", name);
    return;
  }
  constexpr int NT = 64 * (WM * WN + LW);
  const int grid = (c.M / BM) * (c.N / BN);
  const size_t lds = (size_t)S * (BM + BN) * 2 * KB;
  auto k = probe_gemm<BM, BN, WM, WN, S, MODE, false, LW, KB>;
  auto kp = probe_gemm<BM, BN, WM, WN, S, MODE, true, LW, KB>;
  CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  CK(hipFuncSetAttribute((const void*)kp, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(k, dim3(grid), dim3(NT), lds, c.st, A, B, c.C, c.M, c.N, c.K, c.prof, ld);
  CK(hipGetLastError());
  CK(hipStreamSynchronize(c.st));
  double err = 0.0;
  if (MODE == 0) {  // numerics of the sampled entries vs the fp32 reference
    std::vector<uint16_t> hC((size_t)c.M * c.N);
    CK(hipMemcpy(hC.data(), c.C, hC.size() * 2, hipMemcpyDeviceToHost));
    for (size_t e = 0; e < c.hr.size(); ++e) {
      const float got = bf2f(hC[(size_t)c.hr[e] * c.N + c.hc[e]]);
      err = std::max(err, (double)std::fabs(got - c.href[e]) / (1.0 + std::fabs(c.href[e])));
    }
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> per;
  for (int r = 0; r < 5; ++r) {
    CK(hipEventRecord(e0, c.st));
    for (int i = 0; i < iters; ++i)
      hipLaunchKernelGGL(k, dim3(grid), dim3(NT), lds, c.st, A, B, c.C, c.M, c.N, c.K, c.prof, ld);
    CK(hipEventRecord(e1, c.st));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    per.push_back(ms * 1e3f / iters);
  }
  std::sort(per.begin(), per.end());
  // one profiled launch: per-wave cycle split (compute waves)
  CK(hipMemsetAsync(c.prof, 0, (size_t)grid * WM * WN * 4 * 8, c.st));
  hipLaunchKernelGGL(kp, dim3(grid), dim3(NT), lds, c.st, A, B, c.C, c.M, c.N, c.K, c.prof, ld);
  CK(hipGetLastError());
  CK(hipStreamSynchronize(c.st));
  const int nw = grid * WM * WN;
  std::vector<unsigned long long> hp((size_t)nw * 4);
  CK(hipMemcpy(hp.data(), c.prof, hp.size() * 8, hipMemcpyDeviceToHost));
  double s[4] = {0, 0, 0, 0}, mx = 0;
  for (int w = 0; w < nw; ++w) {
    for (int q = 0; q < 4; ++q) s[q] += (double)hp[(size_t)w * 4 + q];
    mx = std::max(mx, (double)hp[(size_t)w * 4]);
  }
  const double flop = 2.0 * c.M * c.N * c.K;
  printf("{\"variant\": \"%s\", \"M\": %d, \"N\": %d, \"K\": %d, \"grid\": %d, \"threads\": %d, \"lds_kb\": %zu, "
         "\"us_med\": %.2f, \"us_min\": %.2f, \"tflops\": %.1f, \"max_rel_err\": %.2e, \"prof_cycles_per_wave\": "
         "{\"total\": %.0f, \"max_total\": %.0f, \"wait\": %.0f, \"barrier\": %.0f, \"issue\": %.0f}, "
         "\"per_kstep\": {\"wait\": %.0f, \"barrier\": %.0f, \"issue\": %.0f}}\n",
         name, c.M, c.N, c.K, grid, NT, lds / 1024, per[per.size() / 2], per[0], flop / per[per.size() / 2] / 1e6, err,
         s[0] / nw, mx, s[1] / nw, s[2] / nw, s[3] / nw, s[1] / nw / (c.K / KB), s[2] / nw / (c.K / KB),
         s[3] / nw / (c.K / KB));
  fflush(stdout);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

int main(int argc, char** argv) {
  Ctx c;
  c.M = argc > 1 ? atoi(argv[1]) : 4096;
  c.N = argc > 2 ? atoi(argv[2]) : 1024;
  c.K = argc > 3 ? atoi(argv[3]) : 1024;
  CK(hipStreamCreate(&c.st));
  std::vector<uint16_t> hA((size_t)c.M * c.K), hB((size_t)c.N * c.K);
  uint32_t x = 12345u;
  auto rnd = [&]() {
    x = x * 1664525u + 1013904223u;
    return (float)((x >> 8) & 0xffff) / 32768.0f - 1.0f;
  };
  for (auto& v : hA) v = f2bf(rnd());
  for (auto& v : hB) v = f2bf(rnd());
  CK(hipMalloc(&c.A, hA.size() * 2));
  CK(hipMalloc(&c.B, hB.size() * 2));
  CK(hipMalloc(&c.C, (size_t)c.M * c.N * 2));
  CK(hipMalloc(&c.prof, (size_t)(c.M / 64) * (c.N / 64) * 16 * 4 * 8));
  CK(hipMemcpy(c.A, hA.data(), hA.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(c.B, hB.data(), hB.size() * 2, hipMemcpyHostToDevice));
  {  // padded copies: row stride K + 64 elements (2,176 B for K = 1024 instead of a power of two)
    const int ldp = c.K + 64;
    std::vector<uint16_t> pA((size_t)c.M * ldp, 0), pB((size_t)c.N * ldp, 0);
    for (int r = 0; r < c.M; ++r) std::copy(hA.begin() + (size_t)r * c.K, hA.begin() + (size_t)(r + 1) * c.K, pA.begin() + (size_t)r * ldp);
    for (int r = 0; r < c.N; ++r) std::copy(hB.begin() + (size_t)r * c.K, hB.begin() + (size_t)(r + 1) * c.K, pB.begin() + (size_t)r * ldp);
    CK(hipMalloc(&c.Ap, pA.size() * 2));
    CK(hipMalloc(&c.Bp, pB.size() * 2));
    CK(hipMemcpy(c.Ap, pA.data(), pA.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(c.Bp, pB.data(), pB.size() * 2, hipMemcpyHostToDevice));
  }
  const int ns = 4096;
  for (int e = 0; e < ns; ++e) {
    x = x * 1664525u + 1013904223u;
    c.hr.push_back((int)(x % (uint32_t)c.M));
    x = x * 1664525u + 1013904223u;
    c.hc.push_back((int)(x % (uint32_t)c.N));
  }
  CK(hipMalloc(&c.rows, ns * 4));
  CK(hipMalloc(&c.cols, ns * 4));
  CK(hipMalloc(&c.ref, ns * 4));
  CK(hipMemcpy(c.rows, c.hr.data(), ns * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(c.cols, c.hc.data(), ns * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(ref_entries, dim3((ns + 255) / 256), dim3(256), 0, c.st, c.A, c.B, c.rows, c.cols, c.ref, ns, c.K, c.K);
  CK(hipGetLastError());
  c.href.resize(ns);
  CK(hipMemcpy(c.href.data(), c.ref, ns * 4, hipMemcpyDeviceToHost));
  const int it = 50;
  run<128, 128, 2, 2, 2, 0>(c, "t128x128_w2x2_s2", it);
  run<64, 128, 2, 2, 2, 0>(c, "t64x128_w2x2_s2", it);
  run<128, 128, 2, 2, 4, 0, 8>(c, "pc_t128x128_w2x2_l8_s4", it);
  run<128, 128, 2, 2, 2, 0, 0, 128>(c, "t128x128_w2x2_s2_bk128", it);
  run<64, 128, 2, 2, 2, 0, 0, 128>(c, "t64x128_w2x2_s2_bk128", it);
  run<128, 128, 2, 2, 2, 0, 8, 128>(c, "pc_t128x128_w2x2_l8_s2_bk128", it);
  run<128, 128, 2, 2, 2, 1, 8, 128>(c, "pc_t128x128_w2x2_l8_s2_bk128_nomfma", it);
  run<128, 128, 4, 2, 2, 0, 0, 128>(c, "t128x128_w4x2_s2_bk128", it);
  run<64, 64, 2, 2, 2, 0, 0, 128>(c, "t64x64_w2x2_s2_bk128", it);
  run<64, 64, 2, 2, 3, 0, 0, 128>(c, "t64x64_w2x2_s3_bk128", it);
  return 0;
}
