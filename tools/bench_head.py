#!/usr/bin/env python3
"""Classifier head of the tabular step (B=4096 rows, K=1024, 2 classes): the fused skinny_head
kernel vs the four-kernel chain it replaces (skinny_fwd -> loss -> skinny_dw
-> skinny_dx).  Times 200 back-to-back launches with HIP events; prints one JSON line per variant."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import dct_amd  # noqa: F401
    from dct_amd.ops._native import native

    nat = native()
    dev = torch.device("cuda", 0)
    B, K, C = 4096, 1024, 2
    H = torch.relu(torch.randn(B, K, device=dev)).to(torch.bfloat16)
    W = (torch.randn(C, K, device=dev) * 0.03).to(torch.bfloat16)
    b = torch.zeros(C, device=dev)
    y = torch.randint(0, C, (B,), device=dev, dtype=torch.int32)
    dH = torch.empty(B, K, device=dev, dtype=torch.bfloat16)
    dW = torch.zeros(C, K, device=dev)
    db = torch.zeros(C, device=dev)
    ls = torch.zeros(1, device=dev)
    Z = torch.empty(B, C, device=dev, dtype=torch.bfloat16)
    dZ = torch.empty_like(Z)
    st = torch.cuda.current_stream().cuda_stream

    def fused():
        nat.skinny_head(H.data_ptr(), W.data_ptr(), b.data_ptr(), y.data_ptr(), dH.data_ptr(), dW.data_ptr(),
                        db.data_ptr(), ls.data_ptr(), B, K, C, 1.0 / B, 0, 1.0 / B, 1, st)

    def chain():
        nat.skinny_fwd(H.data_ptr(), W.data_ptr(), b.data_ptr(), Z.data_ptr(), B, K, C, st)
        nat.cross_entropy_fwd_bwd(Z.data_ptr(), 1, y.data_ptr(), dZ.data_ptr(), ls.data_ptr(), 0, B, C, 1.0 / B, 0, st)
        nat.skinny_dw(dZ.data_ptr(), H.data_ptr(), dW.data_ptr(), db.data_ptr(), B, K, C, st)
        nat.skinny_dx(dZ.data_ptr(), W.data_ptr(), H.data_ptr(), dH.data_ptr(), B, K, C, st)

    def timeit(fn, n=200):
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n * 1e3

    print(json.dumps({"variant": "chain(4 kernels)", "us": round(timeit(chain), 2)}), flush=True)
    print(json.dumps({"variant": "fused", "us": round(timeit(fused), 2)}), flush=True)

if __name__ == "__main__":
    main()
