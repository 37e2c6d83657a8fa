#!/usr/bin/env python3
"""Where does the driver-shaped bench window (20 steps) go?  Sets the weather engine up exactly
like bench.py, then times the same window several times in one process, and splits one window
into enqueue / wait parts with host timestamps."""
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dct_amd  # noqa: E402,F401
from dct_amd.data.synthetic import weather_tensors  # noqa: E402
from dct_amd.models.mlp import build_mlp  # noqa: E402
from dct_amd.parallel.dist import init_distributed  # noqa: E402
from dct_amd.trainer.engines import FusedMLPEngine, adam_hparams_from  # noqa: E402
from dct_amd.trainer.trainer import seed_everything  # noqa: E402


def main():
    steps, warmup, reps = 20, 5, 6
    ctx = init_distributed("gpu")
    seed_everything(42)
    total = warmup + steps * reps
    rows = int(math.ceil((total + 8) * 4 / 0.8)) + 1024
    X, Y = weather_tensors(rows, seed=0, dim=5)
    model = build_mlp(os.environ.get("PROBE_MODEL", "weather"), 5)  # e.g. weather-mlp-3x128
    eng = FusedMLPEngine(model, ctx, 4, seed=42, adam=adam_hparams_from(model.configure_optimizers()))
    n_train = int(0.8 * rows)
    perm = torch.randperm(rows, generator=torch.Generator().manual_seed(42))
    eng.attach_data(X, Y, perm[:n_train], perm[n_train:])
    n_items = eng.upload_epoch_indices(0, shuffle=True)
    loss = torch.zeros(total, dtype=torch.float32, device=ctx.device)
    split = int(os.environ.get("PROBE_WARMUP_CALLS", "1"))  # warmup steps spread over this many launches
    per = [warmup // split + (1 if i < warmup % split else 0) for i in range(split)]
    done = 0
    for k in per:
        eng.run_steps(n_items, k, loss, first_step=done)
        done += k
    first = warmup
    for r in range(reps):
        torch.cuda.synchronize()
        ctx.barrier()
        torch.cuda.synchronize()
        if r == reps - 1:
            time.sleep(0.05)  # an idle gap before the window
        t0 = time.perf_counter()
        eng.run_steps(n_items, steps, loss, first_step=first)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        ctx.barrier()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        if os.environ.get("PROBE_SAME_ROWS", "0") != "1":  # 1: every rep re-runs the same (L2-warm) batches
            first += steps
        print(f"rep {r:2d}: window {1e6 * (t3 - t0):7.1f} us  enqueue {1e6 * (t1 - t0):6.1f}  "
              f"wait {1e6 * (t2 - t1):6.1f}  tail {1e6 * (t3 - t2):5.1f}"
              + ("  (after 50 ms idle)" if r == reps - 1 else ""), flush=True)


if __name__ == "__main__":
    main()
