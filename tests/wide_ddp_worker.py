"""Worker of the multigpu tier's wide-model cases (BASELINE.json configs 4 / 5 at DDP = W, one
process per GPU, RCCL over xGMI):

  tabular  - MLPClassifier on the graph engine (trainer/graph_engine.py: HIP-graph-replayed step
             executor, bf16 MFMA GEMMs, native bucket reducer launched per layer from backward);
  tt       - TabTransformer on the autograd engine over the fused HIP block kernels (native bucket
             reducer; block-group buckets launched as each group's grouped dW is issued).

Usage: wide_ddp_worker.py OUT_JSON_PREFIX KIND STEPS.  Every rank writes OUT_rank{r}.json with its
final flat parameters, the per-step losses it recorded and the reducer's bucket statistics; the
test (tests/test_multigpu.py) checks replica identity and the fp32 DDP emulation."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dct_amd  # noqa: E402,F401
from dct_amd.models.mlp import MLPClassifier  # noqa: E402
from dct_amd.models.tabtransformer import TabTransformer  # noqa: E402
from dct_amd.parallel.dist import init_distributed, shutdown  # noqa: E402
from dct_amd.trainer.engines import AutogradEngine, adam_hparams_from  # noqa: E402
from dct_amd.trainer.graph_engine import GraphMLPEngine  # noqa: E402
from dct_amd.trainer.trainer import seed_everything  # noqa: E402

# shapes: small enough for a quick tier, wide enough for the MFMA paths and >= 2 buckets
TAB = dict(features=64, hidden=(512, 512, 512), batch=128, rows=8192)  # 2.2 MB of grads: 2 buckets
TT = dict(features=64, d_model=64, heads=4, layers=4, batch=64, rows=4096)


def data(rows, feats, seed):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(rows, feats, generator=g)
    w = torch.randn(feats, generator=g)
    return X, ((X @ w) > 0).long()


def build(kind):
    """The model and data of KIND, identical on every rank and in the test's emulation."""
    seed_everything(11)
    if kind == "tabular":
        c = TAB
        model = MLPClassifier(c["features"], hidden=c["hidden"], num_classes=2, dropout=0.0, loss="mse", lr=1e-3)
    else:
        c = TT
        model = TabTransformer(num_features=c["features"], d_model=c["d_model"], heads=c["heads"], layers=c["layers"],
                               lr=1e-3)
    X, Y = data(c["rows"], c["features"], 5)
    n_tr = int(0.8 * c["rows"])
    return model, X, Y, torch.arange(n_tr), torch.arange(n_tr, c["rows"]), c["batch"]


def main():
    out, kind, steps = sys.argv[1], sys.argv[2], int(sys.argv[3])
    ctx = init_distributed("gpu")
    model, X, Y, tr, va, B = build(kind)
    dev = ctx.device
    loss = torch.zeros(steps, device=dev)
    if kind == "tabular":
        eng = GraphMLPEngine(model, ctx, B, seed=42, adam=adam_hparams_from(model.configure_optimizers()))
        eng.attach_data(X, Y, tr, va)
        n_items = eng.upload_epoch_indices(0, shuffle=True)
        eng.run_steps(n_items, steps, loss)
        flat = eng.p
    else:
        eng = AutogradEngine(model, ctx, B, seed=42)
        eng.attach_data(X.to(dev), Y.to(dev), tr, va)
        local = eng.epoch_local_indices(len(eng.train_rows), 0, True)
        rows = eng.train_rows[local].to(dev)
        eng.run_device_steps(rows, 0, steps, loss)
        flat = eng.flat_p
    torch.cuda.synchronize()
    red = eng.reducer
    info = {"params": flat.detach().cpu().tolist(), "losses": loss.cpu().tolist(), "rank": ctx.rank,
            "world": ctx.world_size, "backend": ctx.backend, "graph_used": bool(getattr(eng, "graph_used", False)),
            "num_buckets": red.num_buckets if red is not None else 0,
            "launched_before_finalize": getattr(red, "launched_before_finalize", None),
            "hook_launches": getattr(red, "hook_launches", None),
            "defer_launch": getattr(red, "defer_launch", None)}
    with open(f"{out}_rank{ctx.rank}.json", "w") as f:
        json.dump(info, f)
    shutdown(ctx)


if __name__ == "__main__":
    main()
