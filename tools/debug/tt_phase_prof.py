"""Per-phase timing of the fused TabTransformer block kernels (wall-clock marks, thread 0 of each
workgroup; csrc/tt_block.hip TT_MARK).  python tools/debug/tt_phase_prof.py [B]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

import dct_amd  # noqa: E402,F401
from dct_amd.ops import nn as nnops  # noqa: E402

FWD = ["LN1", "a1 out + QKV", "qkv out + attention", "o out + proj + LN2", "h1/a2 out + fc1 GELU",
       "f out + fc2", "out store + W^T"]
BWD = ["pre stage + dout", "dF W2 gelu' + dpre out", "da2 W1 + LN2 bwd + dh1 out", "do Wo",
       "qkv/o stage", "attention bwd", "dqkv out + da1 W", "LN1 bwd + dh out + LN grads"]


def report(name, bufs, labels, B):
    ts = torch.stack([b.view(B, 16)[:, : len(labels) + 1] for b in bufs[1:]]).double().cpu() * 10.0  # 100 MHz -> ns
    d = (ts[..., 1:] - ts[..., :-1]).mean(dim=(0, 1))
    start = ts[..., 0]
    spread = (start.max(1).values - start.min(1).values).mean()
    total = (ts[..., -1] - ts[..., 0]).mean()
    span = (ts[..., -1].max(1).values - ts[..., 0].min(1).values).mean()
    print(f"{name}: per-workgroup {total / 1e3:.2f} us, kernel span {span / 1e3:.2f} us, start spread {spread / 1e3:.2f} us")
    for lab, v in zip(labels, d.tolist()):
        print(f"   {lab:32s} {v / 1e3:7.2f} us")


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    dev = torch.device("cuda", 0)
    T, H, d, n = 64, 4, 64, 256
    g = torch.Generator(device="cpu").manual_seed(0)
    mk = lambda *s, scale=1.0: (scale * torch.randn(*s, generator=g)).to(dev).requires_grad_()  # noqa: E731
    h = mk(B * T, d)
    ps = [(1 + 0.1 * torch.randn(d, generator=g)).to(dev).requires_grad_(), mk(d, scale=0.1),
          mk(3 * d, d, scale=d ** -0.5), mk(3 * d, scale=0.1), mk(d, d, scale=d ** -0.5), mk(d, scale=0.1),
          (1 + 0.1 * torch.randn(d, generator=g)).to(dev).requires_grad_(), mk(d, scale=0.1),
          mk(n, d, scale=d ** -0.5), mk(n, scale=0.1), mk(d, n, scale=n ** -0.5), mk(d, scale=0.1)]
    dout = torch.randn(B * T, d, device=dev)
    nnops._TT_PROF = {}
    for _ in range(6):
        out = nnops.tt_block(h, *ps, B, H, T)
        out.backward(dout)
    torch.cuda.synchronize()
    report("forward", nnops._TT_PROF["fwd"], FWD, B)
    report("backward", nnops._TT_PROF["bwd"], BWD, B)


if __name__ == "__main__":
    main()
