"""Graph-vs-eager divergence probe: full batches only vs a partial last batch; per-step loss diff."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

from test_graph_engine_gpu import _data, _engine  # noqa: E402

dims, B = [64, 256, 256, 2], 128
for extra in (0, 37):
    n = 40 * B + extra
    X, Y = _data(n, dims[0], seed=3)
    res = {}
    for tag in ("e", "g", "g2"):
        model, eng = _engine(dims, B, lr=1e-3, use_graph=(tag != "e"))
        rows = torch.arange(n)
        eng.attach_data(X, Y, rows, rows[:512])
        res[tag] = torch.cat([eng.train_epoch(ep).cpu() for ep in range(3)])
        res[tag + "_p"] = eng.p.cpu()
    for t in ("g", "g2"):
        d = (res[t] - res["e"]).abs()
        bad = (d > 1e-6).nonzero().flatten().tolist()
        print(f"extra={extra} {t} vs e: max {float(d.max()):.3g} first bad steps {bad[:8]} "
              f"params max diff {float((res[t + '_p'] - res['e_p']).abs().max()):.3g} finite {bool(torch.isfinite(res[t + '_p']).all())}")
