#!/usr/bin/env python3
"""Kernel timing of the TabTransformer block weight gradients at the bench shape (4 blocks x the
four products dW2 64x256, dW1 256x64, dWo 64x64, dWqkv 192x64 over 32768 rows): the generic grouped
split-K GEMM (gemm_bf16_dw_grouped) against csrc/tt_dw.hip with 4 / 8 waves per workgroup and one /
two workgroups per CU.  CUDA events, median of 50 launches after 10 warm-up."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

import dct_amd  # noqa: E402,F401
from dct_amd.ops._native import native  # noqa: E402


def timeit(fn, n=50, warm=10):
    for _ in range(warm):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return statistics.median(a.elapsed_time(b) * 1e3 for a, b in ev)


def main():
    dev = torch.device("cuda:0")
    nat = native()
    st = torch.cuda.current_stream().cuda_stream
    K = 32768
    shapes = [(64, 256), (256, 64), (64, 64), (192, 64)] * 4
    A = [torch.randn(K, m, device=dev).to(torch.bfloat16) for m, _ in shapes]
    B = [torch.randn(K, n, device=dev).to(torch.bfloat16) for _, n in shapes]
    C = [torch.zeros(m, n, device=dev) for m, n in shapes]
    S = [torch.zeros(m, device=dev) for m, _ in shapes]
    pa, pb, pc, ps = ([t.data_ptr() for t in L] for L in (A, B, C, S))
    Ms, Ns = [m for m, _ in shapes], [n for _, n in shapes]
    t = timeit(lambda: nat.gemm_bf16_dw_grouped(pa, pb, pc, Ms, Ns, K, ps, 1, st))
    print(f"grouped split-K GEMM (128x128 tiles): {t:.1f} us", flush=True)
    for w, f in ((4, 1), (8, 1), (8, 2)):
        t = timeit(lambda: nat.tt_dw(pa, pb, pc, ps, Ms, Ns, K, st, waves=w, wg_per_cu=f))
        print(f"tt_dw waves={w} workgroups/CU={f}: {t:.1f} us", flush=True)


if __name__ == "__main__":
    main()
