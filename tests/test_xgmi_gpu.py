"""In-kernel data-parallel all-reduce (parallel/xgmi.py, csrc/mlp_wave_impl.h XG path).

Reference semantics: DDP averages every rank's gradients before an identical Adam step on each
rank (jobs/train_lightning_ddp.py:136), and ``sync_dist`` logs the mean loss.
Checked against a plain-torch fp32 emulation of W ranks (sum of per-rank grads in rank order / W,
then torch Adam)."""
import json
import os
import subprocess
import sys

import pytest
import torch
import torch.nn.functional as F

import dct_amd  # noqa: F401
from dct_amd.data.sampler import distributed_indices
from dct_amd.data.synthetic import weather_tensors
from dct_amd.ops._native import native
from dct_amd.ops.fused_mlp import FusedMLPKernel

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _net(seed=0):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(5, 64), torch.nn.ReLU(), torch.nn.Linear(64, 2))


def _flat(net):
    return torch.cat([t.detach().reshape(-1) for t in net.state_dict().values()])


def ddp_reference(net, X, Y, shards, B, steps, lr=0.01):
    """W-rank DDP emulation: per-rank CE grads, rank-ordered sum / W, one torch Adam step."""
    opt = torch.optim.Adam(net.parameters(), lr=lr)
    params = list(net.parameters())
    losses = []
    for s in range(steps):
        gsum = [torch.zeros_like(p) for p in params]
        lsum = 0.0
        for r, sh in enumerate(shards):
            rows = sh[s * B:(s + 1) * B]
            loss = F.cross_entropy(net(X[rows]), Y[rows])
            gs = torch.autograd.grad(loss, params)
            for a, g in zip(gsum, gs):
                a += g
            lsum += loss.item()
        for p, g in zip(params, gsum):
            p.grad = g / len(shards)
        opt.step()
        losses.append(lsum / len(shards))
    return _flat(net), torch.tensor(losses)


def _in_process_run(W, steps, B, out_path):
    """W 'ranks' as concurrent single-wave kernels on W streams of one GPU, peers = raw pointers."""
    nat = native()
    cuda = torch.device("cuda", 0)
    kern = FusedMLPKernel([5, 64, 2], bmax=4)
    assert kern.xg_supported(B)
    xs = [nat.PeerExchange(W, r, kern.xg_buffer_bytes(W)) for r in range(W)]
    for x in xs:
        x.set_peers([y.recv for y in xs])
    X, Y = weather_tensors(3000, seed=5)
    shards = [distributed_indices(3000, W, r, shuffle=True, seed=42, epoch=0) for r in range(W)]
    p0 = _flat(_net(1))
    ps = [p0.clone().to(cuda) for _ in range(W)]
    ms = [torch.zeros_like(ps[0]) for _ in range(W)]
    vs = [torch.zeros_like(ps[0]) for _ in range(W)]
    losses = [torch.zeros(steps, device=cuda) for _ in range(W)]
    scs = [torch.zeros(1, dtype=torch.int32, device=cuda) for _ in range(W)]
    Xd, Yd = X.to(cuda), Y.to(cuda, torch.int32)
    idx = [s.to(cuda, torch.int32) for s in shards]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(cuda) for _ in range(W)]
    for r in range(W):
        kern.train(ps[r], ms[r], vs[r], Xd, Yd, idx[r], n_items=idx[r].numel(), batch=B, steps=steps, t0=0,
                   lr=0.01, loss_out=losses[r], step_counter=scs[r], xg=xs[r], xg_timeout_s=5.0,
                   stream=streams[r].cuda_stream)
    torch.cuda.synchronize()
    json.dump({"status": [x.read_status() for x in xs], "steps": [int(sc.item()) for sc in scs],
               "params": [p.cpu().tolist() for p in ps], "losses": [l.cpu().tolist() for l in losses]},
              open(out_path, "w"))


def test_in_process_exchange_matches_ddp_reference(tmp_path, cuda):
    """Runs in a fresh process: streams of one process share GPU_MAX_HW_QUEUES hardware queues
    round-robin, so after other tests created streams the two 'ranks' could land on one queue
    and serialise (W > 2 runs as separate processes below)."""
    W, B, steps = 2, 4, 120
    out = tmp_path / "inproc.json"
    code = (f"import sys; sys.path.insert(0, {ROOT!r}); sys.path.insert(0, {os.path.join(ROOT, 'tests')!r}); "
            f"import test_xgmi_gpu as t; t._in_process_run({W}, {steps}, {B}, {str(out)!r})")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    res = json.loads(out.read_text())
    assert res["status"] == [0] * W and res["steps"] == [steps] * W
    ps = [torch.tensor(p) for p in res["params"]]
    ls = [torch.tensor(l) for l in res["losses"]]
    for r_ in range(1, W):  # bit-identical replicas, identical synced losses
        assert torch.equal(ps[r_], ps[0]) and torch.equal(ls[r_], ls[0])
    X, Y = weather_tensors(3000, seed=5)
    shards = [distributed_indices(3000, W, r_, shuffle=True, seed=42, epoch=0) for r_ in range(W)]
    want, want_l = ddp_reference(_net(1), X, Y, shards, B, steps)
    err = (ps[0] - want).abs()
    assert err.median() < 1e-5 and err.max() < 2e-3, (err.median(), err.max())
    assert torch.allclose(ls[0], want_l, atol=2e-4, rtol=1e-3)


def test_exchange_timeout_is_bounded_and_reported(cuda):
    """A rank whose peer never runs must give up after the timeout, flag it, and exit."""
    nat = native()
    kern = FusedMLPKernel([5, 64, 2], bmax=4)
    xs = [nat.PeerExchange(2, r, kern.xg_buffer_bytes(2)) for r in range(2)]
    for x in xs:
        x.set_peers([y.recv for y in xs])
    X, Y = weather_tensors(500, seed=0)
    p = _flat(_net()).to(cuda)
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    sc = torch.zeros(1, dtype=torch.int32, device=cuda)
    idx = torch.arange(400, dtype=torch.int32, device=cuda)
    kern.train(p, m, v, X.to(cuda), Y.to(cuda, torch.int32), idx, n_items=400, batch=4, steps=50, t0=0, lr=0.01,
               step_counter=sc, xg=xs[0], xg_timeout_s=0.2)
    torch.cuda.synchronize()
    assert xs[0].read_status() == 1  # tag of step 0
    assert int(sc.item()) == 0  # no step was applied
    assert torch.equal(p.cpu(), _flat(_net()))


@pytest.mark.parametrize("W", [2, 4, 8])
def test_multi_process_ipc_exchange(W, tmp_path, cuda):
    """Real IPC path: W processes, receive buffers exported/imported with hipIpc handles (W = 8:
    the exchange width of a full MI355X node, XW = 8 kernel variant)."""
    out = tmp_path / "xg.json"
    steps, B = 80, 4
    # one hardware queue per worker: W processes x GPU_MAX_HW_QUEUES (4) + this process's queues can exceed
    # the device's compute queue slots at W = 8, and a spinning rank whose peer's queue is not mapped
    # then times out (seen once at W = 8: status 2); on a real node every rank has a GPU of its own
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", GPU_MAX_HW_QUEUES="1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={W}",
                        "--master-addr=127.0.0.1", f"--master-port={29561 + W}",
                        os.path.join(ROOT, "tests", "xg_worker.py"), str(out), str(steps), str(B)],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = json.loads(out.read_text())
    assert res["status"] == 0 and res["step_counter"] == steps
    for i in range(3):  # device barrier: every rank left after the last rank arrived
        last_arrival = max(res["barrier"][r][i][0] for r in range(W))
        assert all(res["barrier"][r][i][1] >= last_arrival for r in range(W)), res["barrier"]
    ps = [torch.tensor(p) for p in res["params"]]
    p0 = ps[0]
    assert all(torch.equal(p, p0) for p in ps)
    X, Y = weather_tensors(4000, seed=3)
    shards = [distributed_indices(4000, W, r, shuffle=True, seed=42, epoch=0) for r in range(W)]
    want, want_l = ddp_reference(_net(0), X, Y, shards, B, steps)
    err = (p0 - want).abs()
    assert err.median() < 1e-5 and err.max() < 2e-3, (err.median(), err.max())
    assert torch.allclose(torch.tensor(res["losses"][0]), want_l, atol=2e-4, rtol=1e-3)



def _barrier_run(out_path):
    nat = native()
    cuda = torch.device("cuda", 0)
    xs = [nat.PeerExchange(2, r, 4096) for r in range(2)]
    for x in xs:
        x.set_peers([y.recv for y in xs])
    streams = [torch.cuda.Stream(cuda) for _ in range(2)]
    for _ in range(4):
        for r in range(2):
            xs[r].barrier(streams[r].cuda_stream, 5.0)
    torch.cuda.synchronize()
    met = [x.read_status() for x in xs]
    xs[0].barrier(streams[0].cuda_stream, 0.1)  # the peer never comes
    torch.cuda.synchronize()
    json.dump({"met": met, "timeout": xs[0].read_status()}, open(out_path, "w"))


def _barrier_later_tag_run(out_path):
    nat = native()
    a, b, c = (nat.PeerExchange(2, r, 4096) for r in (0, 1, 1))
    a.set_peers([a.recv, b.recv])
    c.set_peers([a.recv, c.recv])  # an impostor rank 1 whose own slot nobody writes
    st = torch.cuda.Stream(torch.device("cuda", 0))
    # rank 1 "leaves" barrier 1 and enters barrier 2 before rank 0 ever polled: rank 0's slot of
    # rank 1 already holds tag 2 when rank 0 runs barrier 1 (the impostor's own polls time out)
    c.barrier(st.cuda_stream, 0.05)
    c.barrier(st.cuda_stream, 0.05)
    torch.cuda.synchronize()
    a.barrier(st.cuda_stream, 2.0)
    torch.cuda.synchronize()
    json.dump({"a": a.read_status(), "c": c.read_status()}, open(out_path, "w"))


def test_device_barrier_accepts_a_later_tag(tmp_path, cuda):
    """a peer that already left barrier N may have overwritten its slot with tag N+1;
    barrier N must accept any tag at or past its own (wrap-safe compare) instead of spinning to
    the timeout and reporting a failure that did not happen."""
    out = tmp_path / "bar2.json"
    code = (f"import sys; sys.path.insert(0, {ROOT!r}); sys.path.insert(0, {os.path.join(ROOT, 'tests')!r}); "
            f"import test_xgmi_gpu as t; t._barrier_later_tag_run({str(out)!r})")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    res = json.loads(out.read_text())
    assert res["a"] == 0, hex(res["a"])
    assert res["c"] & 0x80000000  # the impostor itself did time out


def test_device_barrier_in_process_and_timeout(tmp_path, cuda):
    """Two 'ranks' on two streams of a fresh process meet in the device barrier four times (status
    stays 0); a rank whose peer never arrives gives up after the timeout and records
    0x80000000 | tag (tag = its 5th barrier)."""
    out = tmp_path / "bar.json"
    code = (f"import sys; sys.path.insert(0, {ROOT!r}); sys.path.insert(0, {os.path.join(ROOT, 'tests')!r}); "
            f"import test_xgmi_gpu as t; t._barrier_run({str(out)!r})")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    res = json.loads(out.read_text())
    assert res["met"] == [0, 0]
    assert res["timeout"] == (0x80000000 | 5)
