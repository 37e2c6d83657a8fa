"""Run-to-run spread of the graph engine on the test_graph_engine_gpu config.
argv[1]: run order, e.g. "ggee" / "eegg"; argv[2] = "keep" keeps every engine alive."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

from test_graph_engine_gpu import _data, _engine  # noqa: E402

order = sys.argv[1] if len(sys.argv) > 1 else "ggee"
keep = len(sys.argv) > 2 and sys.argv[2] == "keep"
dims, B = [64, 256, 256, 2], 128
X, Y = _data(40 * B + 37, dims[0], seed=3)
n = X.shape[0]
out, alive = [], []
for i, ch in enumerate(order):
    model, eng = _engine(dims, B, lr=1e-3, use_graph=(ch == "g"))
    rows = torch.arange(n)
    eng.attach_data(X, Y, rows[: 40 * B + 37], rows[:512])
    losses = torch.cat([eng.train_epoch(ep).cpu() for ep in range(3)])
    out.append((f"{ch}{i}", losses))
    if keep:
        alive.append(eng)
ref_tag, ref = out[0]
for tag, l in out[1:]:
    d = (l - ref).abs()
    first = int((d > 1e-6).nonzero()[0]) if (d > 1e-6).any() else -1
    print(order, "keep" if keep else "", ref_tag, "vs", tag, "max", float(d.max()), "first", first)
