#!/usr/bin/env python3
"""Per-phase shader cycles of the DATA-PARALLEL 3x128 weather step (csrc/mlp_block5_impl.h, XW = 2 /
4 / 8 ranks, the in-kernel reduce-scatter + sharded Adam + all-gather; profiling instantiations in
csrc/mlp_block5_xgprof.hip, launched whenever a prof buffer is passed).  W ranks of this script
share ONE GPU through the same IPC-mapped exchange buffers the multi-GPU run uses (a rehearsal: no
xGMI links, so the exchange latencies are HBM round trips, not the fabric's).

    python -m torch.distributed.run --nnodes=1 --nproc-per-node W --master-addr 127.0.0.1 \\
        --master-port 29620 tools/prof_b5x.py [steps]

Rank 0 prints, per phase, the cycles per step averaged over the 8 waves, min / max over ranks, and
the stamped launch's us/step (the stamps cost cycles: compare shares, not totals)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dct_amd  # noqa: E402,F401
from dct_amd.data.synthetic import weather_tensors  # noqa: E402
from dct_amd.ops.fused_mlp import FusedMLPKernel, mlp_num_params  # noqa: E402
from dct_amd.parallel import xgmi  # noqa: E402
from dct_amd.parallel.dist import init_distributed, shutdown  # noqa: E402

PHASES = {0: "F1 h1", 1: "F2 partials + prefetch", 2: "barrier A", 3: "h2 + logit shares", 4: "barrier B",
          5: "loss (+ loss push)", 6: "dZ2 + W2/b grads", 7: "dZ1 + dW0 + small push",
          15: "dW1 MFMA + RS push", 16: "RS poll wait", 17: "owned W1 Adam + AG push",
          18: "small: wait + Adam + AG push", 19: "AG poll wait", 20: "AG unpack + publish", 8: "tail"}
PS = 32


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
    ctx = init_distributed("gpu", backend="gloo")
    W, dev = ctx.world_size, ctx.device
    dims = [5, 128, 128, 2]
    B = 4
    kern = FusedMLPKernel(dims, bmax=4)
    xg = xgmi.setup_peer_exchange(kern, ctx, B)
    if xg is None:
        raise SystemExit("exchange unavailable")
    N = steps * B + 64
    X, Y = weather_tensors(N, seed=0)
    Xd, Yd = X.to(dev), Y.to(dev, torch.int32)
    idx = torch.randperm(N, generator=torch.Generator().manual_seed(ctx.rank))[: steps * B].to(dev, torch.int32)
    torch.manual_seed(0)
    P = mlp_num_params(dims)
    p = (torch.randn(P) * 0.1).to(dev)
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    loss = torch.zeros(steps, device=dev)
    prof = torch.zeros(8 * PS, dtype=torch.int64, device=dev)
    res = []
    for rep in range(2):  # the first launch warms the code object and the exchange
        prof.zero_()
        torch.cuda.synchronize()
        ctx.barrier()
        t0 = time.perf_counter()
        kern.train(p, m, v, Xd, Yd, idx, steps * B, B, steps, rep * steps, 0.01, dropout=0.2, step_base=rep * steps,
                   loss_out=loss, prof=prof, xg=xg, xg_timeout_s=10.0)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        res.append(dt)
    st = xgmi.check(xg, ctx)
    raw = prof.cpu().view(8, PS).double() / steps
    per_phase = {k: float(raw[:, k].mean()) for k in list(PHASES) + [9, 10]}
    allp = ctx.all_gather_object((per_phase, res[-1] / steps * 1e6))
    same = ctx.all_gather_object(p.cpu())
    if ctx.rank == 0:
        print(f"W={W} steps={steps} exchange_status={st} replicas_identical="
              f"{all(torch.equal(q, same[0]) for q in same)}")
        print(f"stamped launch us/step per rank: {[round(u, 3) for _, u in allp]}")
        print(f"{'phase (cycles/step, wave mean)':34s}{'rank-mean':>10s}{'min':>8s}{'max':>8s}")
        tot = 0.0
        for k in (0, 1, 2, 3, 4, 5, 6, 7, 15, 16, 17, 18, 19, 20, 8):
            vals = [pp[k] for pp, _ in allp]
            mean = sum(vals) / len(vals)
            tot += mean
            print(f"{PHASES[k]:34s}{mean:10.0f}{min(vals):8.0f}{max(vals):8.0f}")
        print(f"{'total':34s}{tot:10.0f}")
        # per launch (not per step): the prologue (kernel start -> first step) and the epilogue (last
        # step -> stores done, incl. the launch-end moment all-gather) - the fixed cost of every launch
        for k, name in ((9, "prologue (per launch)"), (10, "epilogue (per launch)")):
            vals = [pp[k] * steps for pp, _ in allp]
            print(f"{name:34s}{sum(vals) / len(vals):10.0f}{min(vals):8.0f}{max(vals):8.0f}")
    ctx.barrier()
    del xg
    shutdown(ctx)


if __name__ == "__main__":
    main()
