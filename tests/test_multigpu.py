"""Multi-GPU tier (``pytest -m multigpu``): the data-parallel paths across REAL devices - one
process per GPU, RCCL over xGMI, and the in-kernel xGMI exchange - against the single-process
emulation of averaged-gradient DDP (reference jobs/train_lightning_ddp.py:136).

Self-skips below 2 visible devices (the 1-GPU boxes of the per-round GPU tier); on a node it
runs W = 2 and W = min(8, devices).  Same worker as the CPU tier (tests/ddp_worker.py), so the
CPU gloo tests, the shared-GPU IPC rehearsals and this tier check one contract:
  * the fused engine 5-64-2 (in-kernel xGMI all-reduce; RCCL per step when disabled),
  * the fused engine 3x128 (grad-mode kernel + fused peer all-reduce/Adam kernel, or RCCL ncclAvg
    + flat Adam; graph-replayed),
  * the autograd engine (native BucketReducer on its comm stream) on the 5-64-2 MLP,
replicas bit-identical, parameters equal the emulation, only rank 0 writes checkpoints/MLflow.
"""
import json
import os
import subprocess
import sys

import pytest
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "ddp_worker.py")

pytestmark = [pytest.mark.gpu, pytest.mark.multigpu]


def _ndev() -> int:
    return torch.cuda.device_count() if torch.cuda.is_available() else 0


needs2 = pytest.mark.skipif(_ndev() < 2, reason="needs >= 2 GPUs on one node")


def _worlds():
    n = _ndev()
    return sorted({2, min(8, n)}) if n >= 2 else [2]


def _torchrun(nproc, port, args, env=None, timeout=600):
    e = dict(os.environ)
    e.update(env or {})
    e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={port}", WORKER] + [str(a) for a in args]
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=e)


def _emulate(rows, epochs, world, hidden=(64,), B=4, lr=0.01):
    from dct_amd.data.sampler import distributed_indices
    from dct_amd.data.synthetic import weather_tensors
    from dct_amd.models.mlp import MLPClassifier

    torch.manual_seed(42)
    x, y = weather_tensors(rows, seed=0)
    n_tr = int(0.8 * rows)
    tr_idx = torch.randperm(rows)[:n_tr]
    model = MLPClassifier(5, hidden=hidden, dropout=0.0)
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    params = list(model.parameters())
    for ep in range(epochs):
        shards = [tr_idx[distributed_indices(n_tr, world, r, shuffle=True, seed=42, epoch=ep)] for r in range(world)]
        for s in range((len(shards[0]) + B - 1) // B):
            gs = [torch.zeros_like(p) for p in params]
            for sh in shards:
                rb = sh[s * B:(s + 1) * B]
                loss = F.cross_entropy(model(x[rb]), y[rb])
                for a, g in zip(gs, torch.autograd.grad(loss, params)):
                    a += g
            for p, g in zip(params, gs):
                p.grad = g / world
            opt.step()
    return torch.cat([p.detach().reshape(-1) for p in params])


def _check(tmp_path, W, rows, epochs, hidden, tol):
    ps = [torch.tensor(json.loads((tmp_path / f"params_rank{r}.json").read_text())["params"]) for r in range(W)]
    for r in range(1, W):
        assert torch.equal(ps[0], ps[r]), (r, (ps[0] - ps[r]).abs().max())
    want = _emulate(rows, epochs, W, hidden)
    err = (ps[0] - want).abs()
    assert err.max() < tol, err.max()
    models = os.listdir(tmp_path / "models")
    assert "last.ckpt" in models and sum(m.startswith("weather-best-") for m in models) == 1
    info = json.loads((tmp_path / "params_rank0.json").read_text())
    return info


@needs2
@pytest.mark.parametrize("W", _worlds())
@pytest.mark.parametrize("mode", ["xgmi", "rccl"])
def test_fused_5_64_2_ddp_across_gpus(tmp_path, W, mode):
    rows, epochs = 600, 2
    r = _torchrun(W, 29711 + W, [tmp_path, epochs, rows, "gpu"], env={"DCT_ALLREDUCE": mode})
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    info = _check(tmp_path, W, rows, epochs, (64,), 2e-3)
    assert info["engine"] == "fused" and info["xg"] == (mode == "xgmi")


@needs2
@pytest.mark.parametrize("W", _worlds())
@pytest.mark.parametrize("gx", ["1", "0"])
def test_fused_3x128_ddp_across_gpus(tmp_path, W, gx):
    """gx=1: grad-mode kernel + fused peer all-reduce + Adam over xGMI (csrc/xg_adam.hip);
    gx=0: grad-mode kernel + RCCL ncclAvg + flat Adam."""
    rows, epochs = 600, 2
    r = _torchrun(W, 29731 + W + (10 if gx == "1" else 0), [tmp_path, epochs, rows, "gpu", "hidden=128,128"],
                  env={"DCT_XG_GRAD": gx})
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    info = _check(tmp_path, W, rows, epochs, (128, 128), 3e-3)
    assert info["gx"] == (gx == "1")


@needs2
@pytest.mark.parametrize("W", _worlds())
def test_autograd_engine_native_bucket_reducer_across_gpus(tmp_path, W):
    rows, epochs = 600, 1
    r = _torchrun(W, 29751 + W, [tmp_path, epochs, rows, "gpu", "engine=autograd"], env={"DCT_DEBUG": "1"})
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    info = _check(tmp_path, W, rows, epochs, (64,), 2e-3)
    assert info["engine"] == "autograd"
