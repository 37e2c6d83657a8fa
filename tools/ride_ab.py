#!/usr/bin/env python3
"""A/B of the tabular 4x1024 step with Adam riding in the dW launches (default) vs one Adam launch
at the end (executor.adam_ride = False): alternating runs in one process, us/step over 200 steps."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dct_amd.models.mlp import build_mlp  # noqa: E402
from dct_amd.parallel.dist import init_distributed  # noqa: E402
from dct_amd.trainer.engines import adam_hparams_from  # noqa: E402
from dct_amd.trainer.graph_engine import GraphMLPEngine  # noqa: E402


def main():
    ctx = init_distributed("gpu")
    B, steps = 4096, 200
    n = B * (steps + 20)
    X = (torch.rand(n, 256, device=ctx.device) * 2 - 1).to(torch.bfloat16)
    Y = torch.randint(0, 2, (n,), device=ctx.device, dtype=torch.int32)
    torch.manual_seed(0)
    model = build_mlp("tabular-mlp-4x1024", 256)
    eng = GraphMLPEngine(model, ctx, B, seed=1, adam=adam_hparams_from(model.configure_optimizers()))
    rows = torch.arange(n)
    eng.attach_data(X, Y, rows, rows[:B])
    ni = eng.upload_epoch_indices(0)
    loss = torch.zeros(steps + 20, device=ctx.device)
    res = {True: [], False: []}
    for rnd in range(4):
        for ride in (True, False):
            eng.exe.adam_ride = ride
            eng.run_steps(ni, 10, loss, first_step=0)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.run_steps(ni, steps, loss, first_step=10)
            torch.cuda.synchronize()
            res[ride].append((time.perf_counter() - t0) / steps * 1e6)
    for ride in (True, False):
        print(f"adam_ride={ride}: us/step {[round(x, 1) for x in res[ride]]} min {min(res[ride]):.1f}", flush=True)


if __name__ == "__main__":
    main()
