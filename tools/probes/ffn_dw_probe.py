#!/usr/bin/env python3
"""Timing probe for the TabTransformer FFN weight gradients at the bench shape (4 blocks, batch 512
x 64 tokens = 32768 rows, d 64, FFN 256) on one MI355X:
  * gemm: the split-K grouped dW GEMMs over stored f / dpre (8 problems, one launch)
  * ffn:  csrc/tt_ffn_dw.hip rebuilding f / dpre from a2 / dout16 (4 problems, one launch)
  * one fused block's forward / backward with and without f / dpre stored (ops/nn.py _TT_FFN_DW)
CUDA-event times, median of 50 launches after 10 warm-up."""
import os
import sys
import statistics

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

import dct_amd  # noqa: E402,F401
from dct_amd.ops import nn as nnops  # noqa: E402
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
    M, bf = 32768, torch.bfloat16
    r = lambda *s: torch.randn(*s, device=dev).to(bf)  # noqa: E731
    blocks = []
    for _ in range(4):
        blocks.append(dict(a2=r(M, 64), do=r(M, 64), f=r(M, 256), dp=r(M, 256), w1=r(256, 64), w2=r(64, 256),
                           b1=torch.randn(256, device=dev), dw1=torch.zeros(256, 64, device=dev),
                           dw2=torch.zeros(64, 256, device=dev), db1=torch.zeros(256, device=dev),
                           db2=torch.zeros(64, device=dev)))
    zs, xs, cs, Ms, Ns, css = [], [], [], [], [], []
    for b in blocks:
        for dz, x, c, cb in ((b["do"], b["f"], b["dw2"], b["db2"]), (b["dp"], b["a2"], b["dw1"], b["db1"])):
            zs.append(dz.data_ptr()); xs.append(x.data_ptr()); cs.append(c.data_ptr())
            Ms.append(dz.shape[1]); Ns.append(x.shape[1]); css.append(cb.data_ptr())
    t_gemm = timeit(lambda: nat.gemm_bf16_dw_grouped(zs, xs, cs, Ms, Ns, M, css, 1, st))
    probs = [[b[k].data_ptr() for k in ("a2", "do", "w1", "w2", "b1", "dw1", "dw2", "db1", "db2")] for b in blocks]
    t_ffn = timeit(lambda: nat.tt_ffn_dw(probs, M, st))
    print(f"FFN dW of 4 blocks: grouped split-K GEMMs over stored f/dpre {t_gemm:.1f} us; "
          f"tt_ffn_dw from a2/dout16 {t_ffn:.1f} us", flush=True)
    # one fused block, forward and backward, with / without f and dpre stored
    B, T, H, d, n = 512, 64, 4, 64, 256
    g = torch.Generator(device="cpu").manual_seed(3)
    mk = lambda *s, scale=1.0: (scale * torch.randn(*s, generator=g)).to(dev).requires_grad_()  # noqa: E731
    t = dict(h=mk(M, d), ln1_w=(1 + 0.1 * torch.randn(d, generator=g)).to(dev).requires_grad_(),
             ln1_b=mk(d, scale=0.1), wqkv=mk(3 * d, d, scale=d ** -0.5), bqkv=mk(3 * d, scale=0.1),
             wo=mk(d, d, scale=d ** -0.5), bo=mk(d, scale=0.1),
             ln2_w=(1 + 0.1 * torch.randn(d, generator=g)).to(dev).requires_grad_(), ln2_b=mk(d, scale=0.1),
             w1=mk(n, d, scale=d ** -0.5), b1=mk(n, scale=0.1), w2=mk(d, n, scale=n ** -0.5), b2=mk(d, scale=0.1))
    keys = ["ln1_w", "ln1_b", "wqkv", "bqkv", "wo", "bo", "ln2_w", "ln2_b", "w1", "b1", "w2", "b2"]
    dout = torch.randn(M, d, device=dev)
    for flag in (False, True):
        nnops._TT_FFN_DW = flag
        holder = {}

        def fwd():
            holder["out"] = nnops.tt_block(t["h"], *[t[k] for k in keys], B, H, T)

        def step():
            out = nnops.tt_block(t["h"], *[t[k] for k in keys], B, H, T)
            out.backward(dout)

        tf = timeit(fwd)
        ts = timeit(step)
        print(f"_TT_FFN_DW={flag}: block forward {tf:.1f} us, forward+backward (incl. dW) {ts:.1f} us", flush=True)


if __name__ == "__main__":
    main()
