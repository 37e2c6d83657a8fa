#!/usr/bin/env python3
"""Which host calls issue the device copies (rocclr copyBuffer / fillBuffer dispatches) of the
TabTransformer training step (4.7 copyBuffer dispatches per step under counters)?

Runs the bench.py TabTransformer config (batch 512, 64 tokens, d 64, 4 heads, 4 layers) EAGERLY
(DCT_GRAPH=0, so every torch op is visible to the profiler; the captured graph replays the same
ops), warms up, then profiles 4 steps with torch.profiler (CPU + device activity, Python stacks)
and prints every host op that issued a memcpy / memset with its Python stack, plus the device
kernels per step.

    DCT_GRAPH=0 python tools/probes/tt_copy_attrib.py
"""
import os
import sys

os.environ.setdefault("DCT_GRAPH", "0")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import dct_amd  # noqa: E402,F401
from dct_amd.data.synthetic import make_tabular_device  # noqa: E402
from dct_amd.models import build_model  # noqa: E402
from dct_amd.parallel.dist import init_distributed, shutdown  # noqa: E402
from dct_amd.trainer.engines import AutogradEngine  # noqa: E402

STEPS = 4


def main():
    ctx = init_distributed("gpu")
    feats, rows, B = 64, 200_000, 512
    X, Y = make_tabular_device(rows, feats, num_classes=2, device=ctx.device, dtype=torch.float32, seed=0)
    model = build_model("tabtransformer", feats, d_model=64, heads=4, layers=4, lr=1e-3)
    eng = AutogradEngine(model, ctx, B, seed=42)
    perm = torch.randperm(rows, generator=torch.Generator().manual_seed(42))
    eng.attach_data(X, Y, perm[: int(0.8 * rows)], perm[int(0.8 * rows):])
    rd = eng.train_rows[: (STEPS + 8) * B].to(ctx.device)
    for s in range(8):
        eng.train_step(rd[s * B:(s + 1) * B], s)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        for s in range(8, 8 + STEPS):
            eng.train_step(rd[s * B:(s + 1) * B], s)
        torch.cuda.synchronize()
    ev = prof.events()
    # device activity per step
    dev = {}
    for e in ev:
        if e.device_type == torch.autograd.DeviceType.CUDA:
            dev.setdefault(e.name, [0, 0.0])
            dev[e.name][0] += 1
            dev[e.name][1] += e.device_time
    print("== device activity per step (count, us)")
    for k, (n, t) in sorted(dev.items(), key=lambda kv: -kv[1][1]):
        print(f"{n / STEPS:6.2f} {t / STEPS:9.1f}  {k[:110]}")
    print("== host calls issuing copies / fills (per step) with Python stacks")
    keys = ("Memcpy", "Memset", "memcpy", "memset", "copyBuffer", "fillBuffer")
    seen = {}
    for e in ev:
        if e.device_type != torch.autograd.DeviceType.CPU:
            continue
        if not any(k in e.name for k in ("hipMemcpy", "hipMemset", "cudaMemcpy", "cudaMemset")) and \
                not any(any(k in c.name for k in keys) for c in (e.cpu_children or [])):
            continue
        # climb to the outermost aten op with a Python stack
        p, stack = e, []
        while p is not None:
            if p.stack:
                stack = [s for s in p.stack if "dct_amd" in s or "tools/" in s][:6]
            p = p.cpu_parent
        key = (e.name, tuple(stack))
        seen[key] = seen.get(key, 0) + 1
    for (name, stack), n in sorted(seen.items(), key=lambda kv: -kv[1]):
        print(f"{n / STEPS:5.2f}/step  {name}")
        for s in stack:
            print(f"           {s}")
    # aten::copy_ / clone / contiguous callers (the usual source of device-to-device memcpys)
    print("== aten copy-type ops per step")
    agg = {}
    for e in ev:
        if e.device_type == torch.autograd.DeviceType.CPU and e.name in ("aten::copy_", "aten::clone",
                                                                          "aten::contiguous", "aten::zero_",
                                                                          "aten::fill_", "aten::zeros"):
            p, stack = e, []
            while p is not None:
                if p.stack:
                    stack = [s for s in p.stack if "dct_amd" in s][:4]
                p = p.cpu_parent
            key = (e.name, tuple(stack))
            agg[key] = agg.get(key, 0) + 1
    for (name, stack), n in sorted(agg.items(), key=lambda kv: -kv[1]):
        print(f"{n / STEPS:5.2f}/step  {name}  <- {' | '.join(stack)}")
    shutdown(ctx)


if __name__ == "__main__":
    main()
