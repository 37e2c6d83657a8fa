#!/usr/bin/env python3
"""Why does a tabular-step GEMM take ~5 us longer inside the step than in isolation?

Times the 4096 x 1024 x 1024 forward GEMM (bias + ReLU epilogue, bf16 out) four ways, 60 launches
each on one stream, HIP events around the loop:
  iso        same operands every launch (A, W and C stay hot in every XCD's L2)
  chain      ping-pong: each launch reads the previous launch's output (the step's dependency:
             an activation written by the last kernel, dirty in the L2s of the XCDs that wrote it)
  chain3w    ping-pong through three different weight matrices (layers 1, 2, 3)
  rotate     independent operand sets larger than the L2s (cold, but not just-written)
and a step-shaped sequence (fwd GEMMs + dX + split-K dW) with and without a 1-thread kernel between
launches.  Prints one JSON line per variant (us per GEMM)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

import dct_amd  # noqa: E402,F401
from dct_amd.ops._native import native  # noqa: E402

M, N, K = 4096, 1024, 1024
EPI_BIAS_RELU = 2


def main():
    nat = native()
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream().cuda_stream
    torch.manual_seed(0)
    bf = torch.bfloat16
    X = [(torch.rand(M, K, device=dev) - 0.5).to(bf) for _ in range(2)]
    W = [((torch.rand(N, K, device=dev) - 0.5) / 16).to(bf) for _ in range(3)]
    bias = torch.zeros(N, device=dev)
    rot = [((torch.rand(M, K, device=dev) - 0.5).to(bf), torch.empty(M, N, device=dev, dtype=bf)) for _ in range(8)]
    C = torch.empty(M, N, device=dev, dtype=bf)

    def gemm(a, w, c, epi=EPI_BIAS_RELU):
        nat.gemm_bf16(a.data_ptr(), w.data_ptr(), c.data_ptr(), bias.data_ptr(), M, N, K, K, K, N, 0, 1, epi, 0, 0,
                      0, st)

    def timed(fn, n=60):
        for _ in range(5):
            fn(0)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(n):
            fn(i)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / n

    res = {}
    res["iso"] = timed(lambda i: gemm(X[0], W[0], C))
    res["chain"] = timed(lambda i: gemm(X[i & 1], W[0], X[(i + 1) & 1]))
    res["chain3w"] = timed(lambda i: gemm(X[i & 1], W[i % 3], X[(i + 1) & 1]))
    res["rotate"] = timed(lambda i: gemm(rot[i % 8][0], W[0], rot[i % 8][1]))
    zero = torch.zeros(4, device=dev)

    def chain_with_gap(i):
        gemm(X[i & 1], W[i % 3], X[(i + 1) & 1])
        nat.zero_f32(zero.data_ptr(), 4, st)  # a tiny kernel between GEMMs
    res["chain3w_plus_tiny_kernel"] = timed(chain_with_gap)
    for k, v in res.items():
        print(json.dumps({"variant": k, "us_per_gemm": round(v, 2)}), flush=True)


if __name__ == "__main__":
    main()
