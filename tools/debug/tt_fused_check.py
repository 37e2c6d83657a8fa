"""Fused vs unfused TabTransformer training trajectories (eager, identical init and batches).

    python tools/debug/tt_fused_check.py [steps]
Prints per-step losses of: unfused, fused fwd only, fused fwd+bwd; then eval loss/acc of each.
"""
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import dct_amd  # noqa: E402,F401
from dct_amd.data.synthetic import make_tabular_device  # noqa: E402
from dct_amd.models import build_model  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    dev = torch.device("cuda", 0)
    X, Y = make_tabular_device(200_000, 64, num_classes=2, device=dev, dtype=torch.float32, seed=0)
    torch.manual_seed(0)
    base = build_model("tabtransformer", 64, d_model=64, heads=4, layers=4, lr=1e-3).to(dev)
    g = torch.Generator().manual_seed(1)
    batches = [torch.randint(0, 150_000, (512,), generator=g).to(dev) for _ in range(steps)]
    val = torch.arange(150_000, 150_000 + 8192, device=dev)
    modes = {"unfused": {"DCT_TT_FUSED": "0"}, "fwd_only": {"DCT_TT_FUSED": "1", "DCT_TT_FUSED_BWD": "0"},
             "fused": {"DCT_TT_FUSED": "1", "DCT_TT_FUSED_BWD": "1"}}
    res = {}
    for name, env in modes.items():
        os.environ.update(env)
        m = copy.deepcopy(base)
        opt = torch.optim.Adam(m.parameters(), lr=1e-3)
        losses = []
        for idx in batches:
            opt.zero_grad(set_to_none=True)
            loss = F.cross_entropy(m(X[idx]), Y[idx].long())
            loss.backward()
            opt.step()
            losses.append(loss.item())
        with torch.no_grad():
            lg = m(X[val])
            vl = F.cross_entropy(lg, Y[val].long()).item()
            va = (lg.argmax(1) == Y[val].long()).float().mean().item()
        res[name] = (losses, vl, va)
        print(name, "val_loss %.4f val_acc %.4f" % (vl, va), flush=True)
    for i in range(0, steps, max(1, steps // 20)):
        print(i, " ".join("%s=%.5f" % (k, v[0][i]) for k, v in res.items()))
    # eval of ONE model under both forward paths
    m = copy.deepcopy(base)
    with torch.no_grad():
        os.environ["DCT_TT_FUSED"] = "0"
        a = m(X[val])
        os.environ["DCT_TT_FUSED"] = "1"
        b = m(X[val])
    print("eval logits rel diff fused vs unfused: %.3e" % float((a - b).norm() / a.norm()))




def engine_check(steps=60):
    """Same comparison through the AutogradEngine (bound params, bf16 shadows, fused Adam,
    HIP graph capture after 3 eager steps) with the graph on and off."""
    from dct_amd.parallel.dist import init_distributed
    from dct_amd.trainer.engines import AutogradEngine
    from dct_amd.trainer.trainer import seed_everything

    ctx = init_distributed("gpu")
    dev = ctx.device
    X, Y = make_tabular_device(200_000, 64, num_classes=2, device=dev, dtype=torch.float32, seed=0)
    perm = torch.randperm(200_000, generator=torch.Generator().manual_seed(42))
    out = {}
    for name, env in {"unfused_graph": {"DCT_TT_FUSED": "0", "DCT_GRAPH": "1"},
                      "fused_graph": {"DCT_TT_FUSED": "1", "DCT_GRAPH": "1"},
                      "fused_eager": {"DCT_TT_FUSED": "1", "DCT_GRAPH": "0"},
                      "fwdonly_graph": {"DCT_TT_FUSED": "1", "DCT_TT_FUSED_BWD": "0", "DCT_GRAPH": "1"}}.items():
        os.environ.update({"DCT_TT_FUSED_BWD": "1"})
        os.environ.update(env)
        seed_everything(42)
        model = build_model("tabtransformer", 64, d_model=64, heads=4, layers=4, lr=1e-3)
        eng = AutogradEngine(model, ctx, 512, seed=42)
        eng.attach_data(X, Y, perm[:160_000], perm[160_000:])
        losses = []
        for i in range(steps):
            rows = perm[i * 512:(i + 1) * 512]
            losses.append(float(eng.train_step(rows, i)))
        out[name] = losses
        print(name, "graph_used", eng.graph_used, flush=True)
    for i in range(0, steps, max(1, steps // 20)):
        print(i, " ".join("%s=%.5f" % (k, v[i]) for k, v in out.items()), flush=True)


if __name__ == "__main__":
    if os.environ.get("ENGINE_CHECK"):
        engine_check(int(sys.argv[1]) if len(sys.argv) > 1 else 60)
    else:
        main()
