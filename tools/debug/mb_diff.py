#!/usr/bin/env python3
"""mlp_block5's two-micro-batch kernels (DCT_MLP_BLOCK=8) vs the one-micro-batch kernels at batch 4,
per parameter segment: grad mode (one step), train mode (1 / 3 steps), and two in-process ranks with
the in-kernel exchange (1 / 3 steps).  Prints max |diff| per segment (0 = bit-identical)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import dct_amd  # noqa: E402,F401
from dct_amd.data.synthetic import weather_tensors  # noqa: E402
from dct_amd.ops._native import native  # noqa: E402
from dct_amd.ops.fused_mlp import FusedMLPKernel, mlp_num_params  # noqa: E402

DIMS = [5, 128, 128, 2]
SEG = [("W0", 640), ("b0", 128), ("W1", 16384), ("b1", 128), ("W2", 256), ("b2", 2)]
cuda = torch.device("cuda", 0)


def segs(a, b):
    out, o = [], 0
    for name, n in SEG:
        d = (a[o:o + n] - b[o:o + n]).abs().max().item()
        out.append(f"{name}:{d:.1e}")
        o += n
    return " ".join(out)


def kern(blk, B=4):
    os.environ["DCT_MLP_BLOCK"] = blk
    return FusedMLPKernel(DIMS, bmax=4 if B <= 4 else 16)


torch.manual_seed(0)
X, Y = weather_tensors(2000, seed=5)
Xd, Yd = X.to(cuda), Y.to(cuda, torch.int32)
P = mlp_num_params(DIMS)
p0 = (torch.randn(P) * 0.1).to(cuda)
idx = torch.randperm(2000)[:400].to(cuda, torch.int32)

# grad mode
g = {}
for blk in ("-1", "8"):
    k = kern(blk)
    gg = torch.zeros(P + 1, device=cuda)
    k.train(p0.clone(), None, None, Xd, Yd, idx, n_items=4, batch=4, steps=1, t0=0, lr=0.01, grad_out=gg)
    torch.cuda.synchronize()
    g[blk] = gg.cpu()
print("grad mode:", segs(g["-1"], g["8"]), "loss", (g["-1"][P] - g["8"][P]).abs().item())

for steps in (1, 3):
    r = {}
    for blk in ("-1", "8"):
        k = kern(blk)
        p, m, v = p0.clone(), torch.zeros_like(p0), torch.zeros_like(p0)
        loss = torch.zeros(steps, device=cuda)
        k.train(p, m, v, Xd, Yd, idx, n_items=400, batch=4, steps=steps, t0=0, lr=0.01, loss_out=loss)
        torch.cuda.synchronize()
        r[blk] = (p.cpu(), m.cpu(), v.cpu(), loss.cpu())
    print(f"train {steps}: p", segs(r["-1"][0], r["8"][0]), "| m", segs(r["-1"][1], r["8"][1]),
          "| loss", (r["-1"][3] - r["8"][3]).abs().max().item())

nat = native()
W = 2
for steps in (1, 1, 3):
    r = {}
    for blk in ("8", "-1"):
        k = kern(blk)
        xs = [nat.PeerExchange(W, q, k.xg_buffer_bytes(W, 4)) for q in range(W)]
        for x in xs:
            x.set_peers([y.recv for y in xs])
        ps = [p0.clone() for _ in range(W)]
        ms = [torch.zeros_like(p0) for _ in range(W)]
        vs = [torch.zeros_like(p0) for _ in range(W)]
        ls = [torch.zeros(steps, device=cuda) for _ in range(W)]
        scs = [torch.zeros(1, dtype=torch.int32, device=cuda) for _ in range(W)]
        strs = [torch.cuda.Stream(cuda) for _ in range(W)]
        torch.cuda.synchronize()
        for q in range(W):
            k.train(ps[q], ms[q], vs[q], Xd, Yd, idx[q * 200:], n_items=200, batch=4, steps=steps, t0=0, lr=0.01,
                    loss_out=ls[q], step_counter=scs[q], xg=xs[q], xg_timeout_s=5.0, stream=strs[q].cuda_stream)
        torch.cuda.synchronize()
        r[blk] = (ps[0].cpu(), ms[0].cpu(), ls[0].cpu(), [x.read_status() for x in xs])
    print(f"xg W=2 {steps}: status", r["-1"][3], r["8"][3], "p", segs(r["-1"][0], r["8"][0]), "| m",
          segs(r["-1"][1], r["8"][1]), "| loss", (r["-1"][2] - r["8"][2]).abs().max().item())
