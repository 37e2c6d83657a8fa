"""Fused peer all-reduce + Adam over xGMI mappings (csrc/xg_adam.hip, parallel/xgmi.py
allreduce_adam_, FusedMLPEngine._ddp_step with ``gx``).

Reference semantics: DDP averages the ranks' gradients, then every rank takes the same Adam step,
and ``sync_dist`` logs the mean loss (jobs/train_lightning_ddp.py:87-88,136).
Checked against plain-torch fp32: the rank-ordered gradient mean and ``torch.optim.Adam``.
W "ranks" share the one GPU: as streams of a fresh process (kernel level) or as processes with
IPC-mapped buffers (engine level)."""
import json
import os
import subprocess
import sys

import pytest
import torch
import torch.nn.functional as F

import dct_amd  # noqa: F401
from dct_amd.ops._native import native

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _torch_reference(p0, grads, W, steps, lr, wd):
    """grads[s][r]: rank r's gradient at step s (n = P + 1 floats, the last one the loss)."""
    P = p0.numel()
    p = torch.nn.Parameter(p0.clone())
    opt = torch.optim.Adam([p], lr=lr, weight_decay=wd)
    avgs = []
    for s in range(steps):
        acc = torch.zeros_like(grads[s][0])
        for r in range(W):
            acc += grads[s][r]
        avg = acc / W
        avgs.append(avg)
        p.grad = avg[:P].clone()
        opt.step()
    return p.detach(), avgs


def _in_process_run(W, steps, n, wd, out_path):
    """W ranks on W streams of one fresh process (streams map to distinct hardware queues only
    while the process has created few of them), peers = raw receive-buffer addresses."""
    from dct_amd.parallel.xgmi import allreduce_adam_

    nat = native()
    cuda = torch.device("cuda", 0)
    P = n - 1
    xs = [nat.PeerExchange(W, r, nat.xg_adam_buffer_bytes(n, W)) for r in range(W)]
    for x in xs:
        x.set_peers([y.recv for y in xs])
    gen = torch.Generator().manual_seed(7)
    p0 = torch.randn(P, generator=gen) * 0.1
    grads = [[torch.randn(n, generator=gen) for _ in range(W)] for _ in range(steps)]
    gd = [[g.to(cuda) for g in gs] for gs in grads]
    ps = [p0.to(cuda) for _ in range(W)]
    ms = [torch.zeros(P, device=cuda) for _ in range(W)]
    vs = [torch.zeros(P, device=cuda) for _ in range(W)]
    gb = [torch.zeros(n, device=cuda) for _ in range(W)]
    scs = [torch.zeros(1, dtype=torch.int32, device=cuda) for _ in range(W)]
    outs = [[] for _ in range(W)]
    streams = [torch.cuda.Stream(cuda) for _ in range(W)]
    torch.cuda.synchronize()
    for s in range(steps):
        for r in range(W):
            with torch.cuda.stream(streams[r]):
                gb[r].copy_(gd[s][r])
                scs[r].add_(1)  # the grad kernel's step-counter advance
                allreduce_adam_(xs[r], gb[r], ps[r], ms[r], vs[r], P, scs[r], 0.01, (0.9, 0.999), 1e-8, wd,
                                timeout=10.0)
                outs[r].append(gb[r].clone())
    torch.cuda.synchronize()
    json.dump({"status": [x.read_status() for x in xs], "p0": p0.tolist(),
               "grads": [[g.tolist() for g in gs] for gs in grads],
               "params": [p.cpu().tolist() for p in ps],
               "avg": [[o.cpu().tolist() for o in outs[r]] for r in range(W)]}, open(out_path, "w"))


def _spawn(fn, *args, timeout=300):
    code = (f"import sys; sys.path.insert(0, {ROOT!r}); sys.path.insert(0, {os.path.join(ROOT, 'tests')!r}); "
            f"import test_xg_adam_gpu as t; t.{fn}(*{args!r})")
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("W,n,wd", [(2, 17539, 0.0), (2, 1001, 0.01)])
def test_in_process_allreduce_adam_matches_torch(W, n, wd, tmp_path, cuda):
    """W = 2 only: a process's streams share GPU_MAX_HW_QUEUES (4) hardware queues round-robin,
    and two ranks on one queue would serialise (W = 4 runs as processes in the engine test)."""
    steps = 6
    out = tmp_path / "xa.json"
    r = _spawn("_in_process_run", W, steps, n, wd, str(out))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    res = json.loads(out.read_text())
    assert res["status"] == [0] * W
    ps = [torch.tensor(p) for p in res["params"]]
    for q in range(1, W):  # bit-identical replicas and averages
        assert torch.equal(ps[q], ps[0])
        assert res["avg"][q] == res["avg"][0]
    grads = [[torch.tensor(g) for g in gs] for gs in res["grads"]]
    want, avgs = _torch_reference(torch.tensor(res["p0"]), grads, W, steps, 0.01, wd)
    for s in range(steps):  # W a power of two: x (1/W) is exactly / W
        assert torch.equal(torch.tensor(res["avg"][0][s]), avgs[s]), s
    err = (ps[0] - want).abs()
    assert err.max() < 1e-5, err.max()


def _timeout_run(out_path):
    from dct_amd.parallel.xgmi import allreduce_adam_

    nat = native()
    n, P = 515, 514
    xs = [nat.PeerExchange(2, r, nat.xg_adam_buffer_bytes(n, 2)) for r in range(2)]
    for x in xs:
        x.set_peers([y.recv for y in xs])
    cuda = torch.device("cuda", 0)
    g = torch.ones(n, device=cuda)
    p = torch.full((P,), 0.5, device=cuda)
    m, v = torch.zeros(P, device=cuda), torch.zeros(P, device=cuda)
    sc = torch.ones(1, dtype=torch.int32, device=cuda)
    allreduce_adam_(xs[0], g, p, m, v, P, sc, 0.01, (0.9, 0.999), 1e-8, 0.0, timeout=0.2)  # rank 1 never runs
    torch.cuda.synchronize()
    st1 = xs[0].read_status()
    sc.add_(1)
    allreduce_adam_(xs[0], g, p, m, v, P, sc, 0.01, (0.9, 0.999), 1e-8, 0.0, timeout=5.0)  # skipped: failed
    torch.cuda.synchronize()
    json.dump({"st1": st1, "st2": xs[0].read_status(), "p": p.cpu().tolist(), "g": g.cpu().tolist()},
              open(out_path, "w"))


def test_allreduce_adam_timeout_is_bounded_and_sticky(tmp_path, cuda):
    """A rank whose peer never arrives gives up after the timeout, flags 0x80000000 | tag, leaves
    its parameters alone, and later launches return at once instead of spinning again."""
    out = tmp_path / "to.json"
    r = _spawn("_timeout_run", str(out), timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    res = json.loads(out.read_text())
    assert res["st1"] == (0x80000000 | 1) and res["st2"] == res["st1"]
    assert all(x == 0.5 for x in res["p"]) and all(x == 1.0 for x in res["g"])


def _ddp_reference(res, steps, B):
    from dct_amd.data.synthetic import weather_tensors
    from dct_amd.models.mlp import MLPClassifier

    X, Y = weather_tensors(3000, seed=1)
    torch.manual_seed(0)
    model = MLPClassifier(5, hidden=(128, 128), dropout=0.0)
    params = list(model.parameters())
    opt = torch.optim.Adam(params, lr=0.01)
    W = len(res)
    losses = []
    for s in range(steps):
        gsum = [torch.zeros_like(p) for p in params]
        lsum = 0.0
        for r in range(W):
            rows = torch.tensor(res[r]["rows"][s * B:(s + 1) * B])
            loss = F.cross_entropy(model(X[rows]), Y[rows])
            for a, g in zip(gsum, torch.autograd.grad(loss, params)):
                a += g
            lsum += loss.item()
        for p, g in zip(params, gsum):
            p.grad = g / W
        opt.step()
        losses.append(lsum / W)
    return torch.cat([p.detach().reshape(-1) for p in params]), torch.tensor(losses)


@pytest.mark.parametrize("W", [2, 4, 8])
def test_engine_ddp_step_with_peer_allreduce_adam(W, tmp_path, cuda):
    """FusedMLPEngine at world size W (processes sharing the GPU, IPC-mapped buffers): the 3x128
    DDP step path runs grad kernel -> fused peer all-reduce + Adam, graph-captured in chunks with
    an eager remainder; replicas stay bit-identical and follow torch DDP + Adam."""
    out = tmp_path / "gx.json"
    steps, B = 45, 4
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={W}",
                        "--master-addr=127.0.0.1", f"--master-port={29581 + W}",
                        os.path.join(ROOT, "tests", "gx_worker.py"), str(out), str(steps), str(B)],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = json.loads(out.read_text())
    for q in range(W):
        assert res[q]["gx"] and res[q]["ok"] and res[q]["graph_used"], res[q]["mode"]
        assert res[q]["mode"].startswith("fused-step+xgmi-allreduce-adam")
        assert res[q]["step_counter"] == steps
        assert res[q]["params"] == res[0]["params"] and res[q]["m"] == res[0]["m"]
        assert res[q]["losses"] == res[0]["losses"]
    want, want_l = _ddp_reference(res, steps, B)
    got = torch.tensor(res[0]["params"])
    err = (got - want).abs()
    assert err.median() < 2e-5 and err.max() < 2e-3, (err.median(), err.max())
    assert torch.allclose(torch.tensor(res[0]["losses"]), want_l, atol=2e-4, rtol=1e-3)
