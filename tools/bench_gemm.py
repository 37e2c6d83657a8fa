"""bf16 GEMM throughput: our MFMA kernel (csrc/gemm_bf16.hip) vs torch.matmul (hipBLASLt).

    python tools/bench_gemm.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dct_amd  # noqa: E402,F401
from dct_amd.ops._native import native  # noqa: E402


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def main():
    nat = native()
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream().cuda_stream
    shapes = [(4096, 1024, 1024), (4096, 1024, 256), (16384, 1024, 1024), (8192, 8192, 8192), (4096, 4096, 4096)]
    for (M, N, K) in shapes:
        for ta, tb in ((0, 1), (0, 0), (1, 0)):
            A = torch.randn(K, M, device=dev).to(torch.bfloat16) if ta else torch.randn(M, K, device=dev).to(torch.bfloat16)
            B = torch.randn(N, K, device=dev).to(torch.bfloat16) if tb else torch.randn(K, N, device=dev).to(torch.bfloat16)
            C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            lda = A.shape[1]
            ldb = B.shape[1]

            def ours():
                nat.gemm_bf16(A.data_ptr(), B.data_ptr(), C.data_ptr(), 0, M, N, K, lda, ldb, N, ta, tb, 0, 0, 0, 0, st)

            At = A.t() if ta else A
            Bt = B.t() if tb else B

            def ref():
                torch.matmul(At, Bt, out=C)

            flops = 2.0 * M * N * K
            t_o = timeit(ours)
            t_r = timeit(ref)
            print(json.dumps({"M": M, "N": N, "K": K, "ta": ta, "tb": tb, "ours_tflops": round(flops / t_o / 1e12, 1),
                              "torch_tflops": round(flops / t_r / 1e12, 1), "ours_us": round(t_o * 1e6, 1),
                              "torch_us": round(t_r * 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
