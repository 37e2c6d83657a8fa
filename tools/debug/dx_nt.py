#!/usr/bin/env python3
"""Tabular dX GEMM (4096 x 1024 x 1024, ReLU-mask epilogue) as NN (B = W, transposed LDS reads - today)
vs NT (B = a transposed bf16 copy of W, the forward's operand layout), next to the forward GEMM;
rotating operand sets (L2-cold, as in the step).  Prints median us per launch."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import dct_amd  # noqa: E402,F401
from dct_amd.ops._native import native  # noqa: E402

nat = native()
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream().cuda_stream
M, N, K = 4096, 1024, 1024
S = 4
torch.manual_seed(0)
X = [(torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16) for _ in range(S)]
W = [(torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16) for _ in range(S)]
WT = [w.t().contiguous() for w in W]
act = [(torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16) for _ in range(S)]
bias = torch.zeros(N, device=dev)
Y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
D = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
D2 = torch.empty(M, K, device=dev, dtype=torch.bfloat16)


def fwd(i):  # Y = relu(X W^T + b)
    nat.gemm_bf16(X[i].data_ptr(), W[i].data_ptr(), Y.data_ptr(), bias.data_ptr(), M, N, K, K, K, N, 0, 1, 2, 0, 0, 0, st)


def dx_nn(i):  # dX = (dZ W) * relu'(act), dZ = X here [M][N=1024]
    nat.gemm_bf16(X[i].data_ptr(), W[i].data_ptr(), D.data_ptr(), 0, M, K, N, N, K, K, 0, 0, 4, 0, 0, act[i].data_ptr(), st)


def dx_nt(i):  # the same with B = W^T stored [K][N] (row k of W^T = column k of W)
    nat.gemm_bf16(X[i].data_ptr(), WT[i].data_ptr(), D2.data_ptr(), 0, M, K, N, N, N, K, 0, 1, 4, 0, 0,
                  act[i].data_ptr(), st)


res = {}
for rnd in range(5):
    for name, fn in (("fwd", fwd), ("dx_nn", dx_nn), ("dx_nt", dx_nt)):
        for i in range(3):
            fn(i % S)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for it in range(60):
            fn(it % S)
        e.record()
        torch.cuda.synchronize()
        res.setdefault(name, []).append(s.elapsed_time(e) / 60 * 1e3)
dx_nn(0)
dx_nt(0)
torch.cuda.synchronize()
print("dx_nt == dx_nn:", torch.equal(D, D2), float((D.float() - D2.float()).abs().max()))
for k, v in res.items():
    print(f"{k:6s} median {statistics.median(v):7.2f} us  min {min(v):7.2f}")
