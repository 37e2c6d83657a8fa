#!/usr/bin/env python3
"""Per-phase shader cycles of the row-parallel weather step (profiling build only:
DCT_PROF_BUILD=1 python -m dct_amd._build; csrc/mlp_wave_impl.h RSTAMP).  Prints each wave's cycles per
step in every phase; the stamps themselves cost cycles, so compare shares, not totals."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dct_amd  # noqa: E402,F401
from dct_amd.ops.fused_mlp import FusedMLPKernel, mlp_num_params  # noqa: E402

PHASES = ["x broadcast", "layer 0 + dropout", "out reduce", "loss", "backward + LDS write", "barrier 1",
          "row sum (+exchange)", "Adam", "publish + barrier 2 + read"]


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
    dev = torch.device("cuda", 0)
    dims = [5, 64, 2]
    P = mlp_num_params(dims)
    N = steps * 4 + 64
    X = torch.randn(N, 5, device=dev)
    Y = torch.randint(0, 2, (N,), device=dev, dtype=torch.int32)
    idx = torch.randperm(N, device=dev)[: steps * 4].to(torch.int32)
    p = torch.randn(P, device=dev) * 0.1
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    loss = torch.zeros(steps, device=dev)
    prof = torch.zeros(128, dtype=torch.int64, device=dev)
    k = FusedMLPKernel(dims, bmax=4)
    k.train(p, m, v, X, Y, idx, steps * 4, 4, steps, 0, 0.01, dropout=0.2, loss_out=loss, prof=prof)
    torch.cuda.synchronize()
    pr = prof.cpu().view(8, 16)[:4, :9].double() / steps
    print("cycles per step      " + "".join(f"wave{w:2d}  " for w in range(4)))
    for i, name in enumerate(PHASES):
        print(f"{name:26s}" + "".join(f"{pr[w, i].item():8.0f}" for w in range(4)))
    print(f"{'total':26s}" + "".join(f"{pr[w].sum().item():8.0f}" for w in range(4)))


if __name__ == "__main__":
    main()
