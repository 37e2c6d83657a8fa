"""Tier-2 distributed tests on CPU (gloo), the reference's own execution model (two CPU
processes, one per "node", jobs/train_lightning_ddp.py:133-136): replicas stay identical,
the DDP update equals the single-process emulation of averaged gradients, only rank 0 writes
checkpoints / MLflow, resume from last.ckpt continues the run exactly, fault injection kills
the chosen rank."""
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

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "ddp_worker.py")


def _torchrun(nproc, port, args, env=None, timeout=600, max_restarts=0):
    e = dict(os.environ)
    e.update(env or {})
    e.pop("CUDA_VISIBLE_DEVICES", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={port}", f"--max-restarts={max_restarts}",
           WORKER] + [str(a) for a in args]
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=e)


def _emulate(rows, epochs, world, B=4, lr=0.01):
    """Single-process emulation of W-rank DDP: per-rank CE grads on DistributedSampler shards,
    averaged, one Adam step (plus the trainer's 80/20 split and sampler seeds)."""
    from dct_amd.models.mlp import MLPClassifier

    # same global-RNG sequence as the worker: seed 42 -> random_split's randperm -> model init
    torch.manual_seed(42)
    x, y = weather_tensors(rows, seed=0)
    n_tr = int(0.8 * rows)
    tr_idx = torch.randperm(rows)[:n_tr]
    model = MLPClassifier(5, hidden=(64,), dropout=0.0)
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    params = list(model.parameters())
    for ep in range(epochs):
        shards = [tr_idx[distributed_indices(n_tr, world, r, shuffle=True, seed=42, epoch=ep)] for r in range(world)]
        steps = (len(shards[0]) + B - 1) // B
        for s in range(steps):
            gs = [torch.zeros_like(p) for p in params]
            for sh in shards:
                rows_b = sh[s * B:(s + 1) * B]
                loss = F.cross_entropy(model(x[rows_b]), y[rows_b])
                for a, g in zip(gs, torch.autograd.grad(loss, params)):
                    a += g
            for p, g in zip(params, gs):
                p.grad = g / world
            opt.step()
    return torch.cat([p.detach().reshape(-1) for p in params])


@pytest.mark.slow
def test_two_rank_gloo_ddp_matches_emulation_and_rank0_io(tmp_path):
    rows, epochs = 600, 2
    r = _torchrun(2, 29631, [tmp_path, epochs, rows])
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    p0 = torch.tensor(json.loads((tmp_path / "params_rank0.json").read_text())["params"])
    p1 = torch.tensor(json.loads((tmp_path / "params_rank1.json").read_text())["params"])
    assert torch.equal(p0, p1), (p0 - p1).abs().max()
    want = _emulate(rows, epochs, 2)
    assert (p0 - want).abs().max() < 1e-4, (p0 - want).abs().max()
    models = sorted(os.listdir(tmp_path / "models"))
    assert "last.ckpt" in models and sum(m.startswith("weather-best-") for m in models) == 1
    exp_dirs = [d for d in os.listdir(tmp_path / "mlruns") if d.isdigit() and d != "0"]
    runs = [d for d in os.listdir(tmp_path / "mlruns" / exp_dirs[0]) if len(d) == 32]
    assert len(runs) == 1  # rank 0 only
    logged = set(os.listdir(tmp_path / "mlruns" / exp_dirs[0] / runs[0] / "metrics"))
    # reference keys plus the throughput extras
    assert {"train_loss", "val_loss", "val_acc", "epoch", "samples_per_sec", "step_time_ms", "allreduce_ms"} <= logged, logged


@pytest.mark.slow
def test_single_rank_matches_emulation(tmp_path):
    r = _torchrun(1, 29632, [tmp_path, 1, 400])
    assert r.returncode == 0, r.stderr[-3000:]
    p0 = torch.tensor(json.loads((tmp_path / "params_rank0.json").read_text())["params"])
    assert (p0 - _emulate(400, 1, 1)).abs().max() < 1e-4


@pytest.mark.slow
def test_resume_from_last_checkpoint_continues_exactly(tmp_path):
    full, part = tmp_path / "full", tmp_path / "part"
    full.mkdir()
    part.mkdir()
    assert _torchrun(1, 29633, [full, 2, 400]).returncode == 0
    assert _torchrun(1, 29634, [part, 1, 400]).returncode == 0
    r = _torchrun(1, 29635, [part, 2, 400, "resume"])
    assert r.returncode == 0, r.stderr[-3000:]
    a = json.loads((full / "params_rank0.json").read_text())
    b = json.loads((part / "params_rank0.json").read_text())
    assert a["global_step"] == b["global_step"]
    assert torch.allclose(torch.tensor(a["params"]), torch.tensor(b["params"]), atol=1e-6)


@pytest.mark.slow
def test_fault_injection_kills_the_chosen_rank(tmp_path):
    r = _torchrun(2, 29636, [tmp_path, 2, 400], env={"DCT_FAULT_RANK": "1", "DCT_FAULT_STEP": "7"}, timeout=300)
    assert r.returncode != 0
    assert "fault injection: rank 1 exits at step 7" in (r.stdout + r.stderr)


@pytest.mark.slow
def test_crash_then_relaunch_resumes_from_last_checkpoint(tmp_path):
    """Rank 1 killed mid-epoch 2; the relaunched job (--resume: what an Airflow retry or a torchrun
    elastic restart does - ckpt.resume_checkpoint) continues from last.ckpt written at the end of
    epoch 1 and finishes with exactly the uninterrupted run's parameters and step count
    (failure detection + checkpoint resume)."""
    full, faulty = tmp_path / "full", tmp_path / "faulty"
    full.mkdir()
    faulty.mkdir()
    rows, epochs = 400, 3  # 320 train rows / 2 ranks / batch 4 = 40 steps per epoch
    assert _torchrun(2, 29637, [full, epochs, rows]).returncode == 0
    r = _torchrun(2, 29638, [faulty, epochs, rows], env={"DCT_FAULT_RANK": "1", "DCT_FAULT_STEP": "60"})
    assert r.returncode != 0 and "fault injection: rank 1 exits at step 60" in (r.stdout + r.stderr)
    assert (faulty / "models" / "last.ckpt").exists()
    r = _torchrun(2, 29639, [faulty, epochs, rows, "resume"])
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    a = json.loads((full / "params_rank0.json").read_text())
    b = json.loads((faulty / "params_rank0.json").read_text())
    assert a["global_step"] == b["global_step"] == 120
    assert torch.allclose(torch.tensor(a["params"]), torch.tensor(b["params"]), atol=1e-6)


def test_resume_checkpoint_policy(tmp_path, monkeypatch):
    """Fresh launches start from scratch unless --resume (the reference never resumes); a torchrun
    elastic restart (TORCHELASTIC_RESTART_COUNT > 0) resumes from last.ckpt when it exists."""
    from dct_amd.ckpt import resume_checkpoint

    monkeypatch.delenv("TORCHELASTIC_RESTART_COUNT", raising=False)
    assert resume_checkpoint(str(tmp_path), False) is None
    assert resume_checkpoint(str(tmp_path), True) is None  # nothing to resume from
    (tmp_path / "last.ckpt").write_bytes(b"x")
    assert resume_checkpoint(str(tmp_path), False) is None
    assert resume_checkpoint(str(tmp_path), True) == str(tmp_path / "last.ckpt")
    monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", "1")
    assert resume_checkpoint(str(tmp_path), False) == str(tmp_path / "last.ckpt")
