"""Per-step cost of the in-kernel all-reduce: W ranks as concurrent kernels on W streams of one
GPU (W <= 2 in-process; see tests/test_xgmi_gpu.py), s_memrealtime stamps of the exchange phase.

    python tools/prof_xg.py --steps 20000
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dct_amd  # noqa: E402,F401
from dct_amd.data.synthetic import weather_tensors  # noqa: E402
from dct_amd.ops._native import native  # noqa: E402
from dct_amd.ops.fused_mlp import FusedMLPKernel  # noqa: E402


def run(W, steps, B=4):
    nat = native()
    dev = torch.device("cuda", 0)
    kern = FusedMLPKernel([5, 64, 2], bmax=4)
    xs = [nat.PeerExchange(W, r, kern.xg_buffer_bytes(W)) for r in range(W)] if W > 1 else [None]
    if W > 1:
        for x in xs:
            x.set_peers([y.recv for y in xs])
    n = steps * B + 64
    X, Y = weather_tensors(n, seed=0)
    Xd, Yd = X.to(dev), Y.to(dev, torch.int32)
    idx = [torch.randperm(n, generator=torch.Generator().manual_seed(r)).to(dev, torch.int32) for r in range(W)]
    torch.manual_seed(0)
    p0 = torch.randn(5 * 64 + 64 + 64 * 2 + 2) * 0.1
    ps = [p0.clone().to(dev) for _ in range(W)]
    ms = [torch.zeros_like(ps[0]) for _ in range(W)]
    vs = [torch.zeros_like(ps[0]) for _ in range(W)]
    prof = [torch.zeros(32, dtype=torch.int64, device=dev) for _ in range(W)]
    streams = [torch.cuda.Stream(dev) for _ in range(W)]
    out = {}
    for rep in range(2):  # first pass warms code objects
        for t in prof:
            t.zero_()
        torch.cuda.synchronize()
        for r in range(W):
            kern.train(ps[r], ms[r], vs[r], Xd, Yd, idx[r], n_items=n, batch=B, steps=steps, t0=0, lr=0.01,
                       prof=prof[r], xg=xs[r], xg_timeout_s=5.0, stream=streams[r].cuda_stream)
        torch.cuda.synchronize()
    pr = prof[0].cpu().tolist()
    total_ticks = pr[31] - pr[30]
    out = {"W": W, "steps": steps, "us_per_step": total_ticks * 10e-3 / steps,
           "exchange_us_per_step": pr[29] * 10e-3 / steps if W > 1 else 0.0,
           "status": [x.read_status() for x in xs] if W > 1 else [0]}
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20000)
    a = ap.parse_args()
    print(json.dumps(run(1, a.steps)), flush=True)
    print(json.dumps(run(2, a.steps)), flush=True)
