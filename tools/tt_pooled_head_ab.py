#!/usr/bin/env python3
"""A/B of the TabTransformer step (bench.py's config: batch 512, 64 tokens, d 64, 4 heads, 4 layers)
with the last block handing the classifier head its token mean (models/tabtransformer.py POOLED_HEAD,
default) against the head pooling the last block's full [B*64, 64] output itself.  Two engines, each
graph-captured with its setting, timed alternately on one GPU: ms/step over 200 device-loop steps.

    python tools/tt_pooled_head_ab.py [FLAG]   # FLAG: a models/tabtransformer.py switch, default POOLED_HEAD
                                               # (FUSED_EMBED: the first block embeds the features itself)"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dct_amd  # noqa: E402,F401
from dct_amd.data.synthetic import make_tabular_device  # noqa: E402
from dct_amd.models import build_model  # noqa: E402
from dct_amd.models import tabtransformer as ttm  # noqa: E402
from dct_amd.parallel.dist import init_distributed  # noqa: E402
from dct_amd.trainer.engines import AutogradEngine  # noqa: E402


FLAG = sys.argv[1] if len(sys.argv) > 1 else "POOLED_HEAD"


def make(ctx, X, Y, pooled):
    from dct_amd.ops import nn as nnops
    from dct_amd.ops._native import native
    # "nn.NAME": a switch of ops/nn.py instead; "native.NAME": a native setter taking 0 / 1
    if FLAG.startswith("native."):
        getattr(native(), FLAG[7:])(int(pooled))
    else:
        setattr(nnops if FLAG.startswith("nn.") else ttm, FLAG[3:] if FLAG.startswith("nn.") else FLAG, pooled)
    torch.manual_seed(0)
    model = build_model("tabtransformer", 64, d_model=64, heads=4, layers=4, lr=1e-3)
    eng = AutogradEngine(model, ctx, 512, seed=42)
    rows = X.shape[0]
    perm = torch.randperm(rows, generator=torch.Generator().manual_seed(42))
    eng.attach_data(X, Y, perm[: int(0.8 * rows)], perm[int(0.8 * rows):])
    rd = eng.train_rows[: 512 * 260].to(ctx.device)
    loss = torch.zeros(260, device=ctx.device)
    eng.run_device_steps(rd, 0, 30, loss)  # warm-up + capture with this setting
    torch.cuda.synchronize()
    return eng, rd, loss


def timed(eng, rd, loss):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.run_device_steps(rd, 30, 200, loss)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / 200 * 1e3


def main():
    ctx = init_distributed("gpu")
    X, Y = make_tabular_device(200_000, 64, num_classes=2, device=ctx.device, dtype=torch.float32, seed=0)
    engs = {p: make(ctx, X, Y, p) for p in (True, False)}
    res = {True: [], False: []}
    for _ in range(4):
        for p in (True, False):
            res[p].append(timed(*engs[p]))
    for p in (True, False):
        print(f"{FLAG}={p}: ms/step {[round(v, 4) for v in res[p]]} min {min(res[p]):.4f} "
              f"loss[229] {float(engs[p][2][229]):.5f}", flush=True)


if __name__ == "__main__":
    main()
