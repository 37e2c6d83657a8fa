#!/usr/bin/env python3
"""Host-side cost of a persistent weather-MLP launch: the driver's bench times 20 steps, where
the launch path (Python + pybind + hipLaunch + synchronize) is a large share of the window.
Times (a) torch.cuda.synchronize alone, (b) the keyword launch path (FusedMLPKernel.train),
(c) the bound launch (BoundTrain.run), each as enqueue-only and enqueue+sync."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dct_amd  # noqa: E402,F401
from dct_amd.ops.fused_mlp import FusedMLPKernel, mlp_num_params  # noqa: E402


def best(fn, n=200):
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2] * 1e6, ts[0] * 1e6


def main():
    dev = torch.device("cuda", 0)
    dims = [5, 64, 2]
    P = mlp_num_params(dims)
    k = FusedMLPKernel(dims, bmax=4)
    p = (torch.randn(P, device=dev) * 0.1)
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    N = 1 << 16
    X = torch.randn(N, 5, device=dev)
    Y = torch.randint(0, 2, (N,), device=dev, dtype=torch.int32)
    idx = torch.randint(0, N, (N,), device=dev, dtype=torch.int32)
    loss = torch.zeros(N // 4, device=dev)
    ctr = torch.zeros(1, dtype=torch.int32, device=dev)
    bl = k.prepare_train(p, m, v, X, Y, idx, n_items=N, batch=4, lr=1e-3, loss_out=loss, step_counter=ctr)

    def kw(steps):
        k.train(p, m, v, X, Y, idx, n_items=N, batch=4, steps=steps, t0=0, lr=1e-3, loss_out=loss[:steps],
                step_counter=ctr)

    torch.cuda.synchronize()
    out = {}
    out["sync_only"] = best(torch.cuda.synchronize)
    for steps in (1, 20):
        out[f"kw_enqueue_s{steps}"] = best(lambda: kw(steps))
        torch.cuda.synchronize()
        out[f"bound_enqueue_s{steps}"] = best(lambda: bl.run(0, steps))
        torch.cuda.synchronize()
        out[f"kw_launch_sync_s{steps}"] = best(lambda: (kw(steps), torch.cuda.synchronize()))
        out[f"bound_launch_sync_s{steps}"] = best(lambda: (bl.run(0, steps), torch.cuda.synchronize()))
    tiny = torch.zeros(1, device=dev)
    out["torch_tiny_launch_sync"] = best(lambda: (tiny.add_(1.0), torch.cuda.synchronize()))
    # GPU-side duration of the launch itself (prologue + steps), from events around it.
    for steps in (1, 20):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ts = []
        for _ in range(200):
            e0.record()
            bl.run(0, steps)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        ts.sort()
        out[f"bound_gpu_events_s{steps}"] = (ts[len(ts) // 2], ts[0])
    for name, (med, lo) in out.items():
        print(f"{name:24s} median {med:8.2f} us   min {lo:8.2f} us", flush=True)


if __name__ == "__main__":
    main()
