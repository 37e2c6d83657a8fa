"""Diagnostic: per-phase cycle breakdown of the fused MLP step (in-kernel s_memtime stamps).

Only the *shares* are meaningful (stamps add their own cost); the effective shader clock is
Δs_memtime / Δs_memrealtime x 100 MHz.
    python tools/prof_fused.py [--dims 5,64,2] [--steps 5000]
"""
import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dct_amd  # noqa: E402,F401
from dct_amd.ops.fused_mlp import FusedMLPKernel, mlp_num_params  # noqa: E402

NAMES = {0: "gather", 1: "fwd0", 2: "fwd1", 3: "fwd2", 4: "fwd3", 5: "loss", 7: "dx1", 8: "dx2", 9: "dx3",
         11: "dW+adam"}
WAVE_NAMES = {0: "bcast+layer0", 1: "hidden+out-reduce", 2: "loss", 3: "backward", 4: "xg-exchange", 5: "adam"}


def run(dims, steps, B=4, dropout=0.2):
    dev = torch.device("cuda", 0)
    P = mlp_num_params(dims)
    N = steps * B + 64
    X = torch.randn(N, dims[0], device=dev)
    Y = torch.randint(0, dims[-1], (N,), device=dev, dtype=torch.int32)
    idx = torch.randperm(N, device=dev)[: steps * B].to(torch.int32)
    p = torch.randn(P, device=dev) * 0.1
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    loss = torch.zeros(steps, device=dev)
    k = FusedMLPKernel(dims, bmax=4 if B <= 4 else 16)
    prof = torch.zeros(32, dtype=torch.int64, device=dev)
    k.train(p, m, v, X, Y, idx, steps * B, B, steps, 0, 0.01, dropout=dropout, loss_out=loss)  # warm
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    k.train(p, m, v, X, Y, idx, steps * B, B, steps, 0, 0.01, dropout=dropout, loss_out=loss)
    ev1.record()
    torch.cuda.synchronize()
    plain_us = ev0.elapsed_time(ev1) * 1e3 / steps
    k.train(p, m, v, X, Y, idx, steps * B, B, steps, 0, 0.01, dropout=dropout, loss_out=loss, prof=prof)
    torch.cuda.synchronize()
    pr = prof.cpu().tolist()
    real_us = (pr[31] - pr[30]) / 100.0  # 100 MHz
    names = WAVE_NAMES if k.plan.use_wave else NAMES
    cyc = sum(pr[i] for i in names)
    clock_ghz = cyc / (real_us * 1e3) if real_us > 0 else float("nan")
    phases = {names[i]: round(pr[i] / steps, 1) for i in names if pr[i]}
    return {"dims": dims, "B": B, "us_per_step_plain": round(plain_us, 3),
            "us_per_step_stamped": round(real_us / steps, 3), "clock_ghz": round(clock_ghz, 3),
            "cycles_per_step": round(cyc / steps, 1), "phase_cycles_per_step": phases,
            "threads": k.plan.threads, "max_blocks_per_thread": k.plan.max_blocks_per_thread,
            "wave_kernel": bool(k.plan.use_wave)}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5000)
    a = ap.parse_args()
    for kern in ("auto", "lds"):
        os.environ["DCT_MLP_KERNEL"] = kern
        for dims in ([5, 64, 2], [5, 64, 64, 2], [5, 128, 128, 2]):
            r = run(dims, a.steps)
            r["kernel"] = kern
            print(json.dumps(r), flush=True)
