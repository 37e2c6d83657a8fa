#!/usr/bin/env python3
"""Per-phase shader cycles of the 3x128 weather step (csrc/mlp_block5.hip by default, mlp_block3.hip
with DCT_MLP_BLOCK=3, mlp_block2.hip with DCT_MLP_BLOCK=2, the 16-wave mlp_block4 with 4; PROF instantiation:
launched whenever a prof buffer is passed; no special build).  Prints each wave's cycles per step
in every phase; the stamps themselves cost cycles, so compare shares, not totals."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dct_amd  # noqa: E402,F401
from dct_amd.ops.fused_mlp import FusedMLPKernel, mlp_num_params  # noqa: E402

PHASES_B2 = ["F1 h1 + keep ballots", "F2 partials + prefetch", "barrier", "F2r h2 (8 partials)",
             "logits + loss", "dZ2, W2/b2/b1 Adam", "dX reduce-scatter", "dW0/db0 Adam", "dW1 + Adam"]
PHASES_B3 = ["F1 h1 + keep hash", "F2 partials + prefetch", "barrier A", "h2 own 16 + logit share",
             "barrier B", "logits + loss", "dZ2 + W2/b1/b2 Adam", "dX + dW0/db0 Adam", "dW1 + Adam"]
PHASES = PHASES_B2 if os.environ.get("DCT_MLP_BLOCK") == "2" else PHASES_B3  # block4: same phases
NWAVES = 16 if os.environ.get("DCT_MLP_BLOCK") == "4" else 8
_blk = os.environ.get("DCT_MLP_BLOCK", "")
ONCE = ["prologue (per launch)", "epilogue (per launch)"]


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
    dev = torch.device("cuda", 0)
    dims = [5, 128, 128, 2]
    P = mlp_num_params(dims)
    N = steps * 4 + 64
    X = torch.randn(N, 5, device=dev)
    Y = torch.randint(0, 2, (N,), device=dev, dtype=torch.int32)
    idx = torch.randperm(N, device=dev)[: steps * 4].to(torch.int32)
    p = torch.randn(P, device=dev) * 0.1
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    loss = torch.zeros(steps, device=dev)
    prof = torch.zeros(16 * 16, dtype=torch.int64, device=dev)
    k = FusedMLPKernel(dims, bmax=4)
    k.train(p, m, v, X, Y, idx, steps * 4, 4, steps, 0, 0.01, dropout=0.2, loss_out=loss, prof=prof)
    torch.cuda.synchronize()
    prof.zero_()
    t0 = time.perf_counter()
    k.train(p, m, v, X, Y, idx, steps * 4, 4, steps, 0, 0.01, dropout=0.2, loss_out=loss, prof=prof)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    raw = prof.cpu().view(16, 16)[:NWAVES].double()
    pr = raw[:, :len(PHASES)] / steps
    print(f"stamped launch: {dt / steps * 1e6:.3f} us/step (stamps included)")
    print("cycles per step        " + "".join(f" wave{w:<2d}" for w in range(NWAVES)))
    for i, name in enumerate(PHASES):
        print(f"{name:24s}" + "".join(f"{pr[w, i].item():7.0f}" for w in range(NWAVES)))
    print(f"{'total':24s}" + "".join(f"{pr[w].sum().item():7.0f}" for w in range(NWAVES)))
    for i, name in enumerate(ONCE):
        print(f"{name:24s}" + "".join(f"{raw[w, 9 + i].item():7.0f}" for w in range(NWAVES)))
    if _blk not in ("2", "3", "4"):  # mlp_block5: cumulative prologue marks (cycles since kernel start)
        for i, name in enumerate(["prologue: loads issued", "prologue: W1+m staged", "prologue: in registers",
                                  "prologue: LDS init done"]):
            print(f"{name:24s}" + "".join(f"{raw[w, 11 + i].item():7.0f}" for w in range(NWAVES)))


if __name__ == "__main__":
    main()
