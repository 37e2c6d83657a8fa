"""Trainer loop semantics on CPU (single process, autograd engine)."""
import pytest
import torch
from torch.utils.data import DataLoader, random_split

import dct_amd  # noqa: F401
from dct_amd.data.dataset import TensorPairDataset
from dct_amd.data.synthetic import weather_tensors
from dct_amd.models.mlp import MLPClassifier
from dct_amd.tracking import InMemoryLogger
from dct_amd.trainer import Trainer, seed_everything
from dct_amd.trainer.engines import AutogradEngine


def _fit(monkeypatch, simulate_replay: bool):
    """Fit one epoch; with ``simulate_replay`` the engine behaves like the GPU graph path: step 2
    is 'captured' (training_step runs once and its logged tensors are kept) and later steps are
    'replayed' (self.log never runs, so the Trainer sees no step logs)."""
    orig = AutogradEngine.train_step

    def train_step(self, rows, batch_idx):
        loss = orig(self, rows, batch_idx)
        if simulate_replay and batch_idx >= 2:
            trainer = self.model._trainer
            if batch_idx == 2:
                self.last_step_mode = "captured"
                # a captured graph's outputs are refreshed in place by every replay; mimic that
                self._static = loss.clone()
                trainer._step_logs = {"train_loss": (self._static, True)}
            else:
                self.last_step_mode = "replayed"
                self._static.copy_(loss)
                trainer._step_logs = {}
        return loss

    monkeypatch.setattr(AutogradEngine, "train_step", train_step)
    seed_everything(42)
    x, y = weather_tensors(240, seed=0)
    ds = TensorPairDataset(x, y)
    tr, va = random_split(ds, [192, 48])
    torch.manual_seed(0)
    model = MLPClassifier(5, hidden=(64,), dropout=0.0)
    logger = InMemoryLogger()
    t = Trainer(max_epochs=1, accelerator="cpu", engine="autograd", logger=logger, log_every_n_steps=5,
                num_sanity_val_steps=0, verbose=False)
    t.fit(model, DataLoader(tr, batch_size=4, shuffle=True), DataLoader(va, batch_size=4))
    return logger.history("train_loss"), t.callback_metrics["train_loss"]


def test_train_loss_is_logged_when_steps_are_graph_replays(monkeypatch):
    eager, last_e = _fit(monkeypatch, False)
    replay, last_r = _fit(monkeypatch, True)
    assert [s for s, _ in eager] == [s for s, _ in replay] == list(range(4, 48, 5))
    assert [v for _, v in eager] == pytest.approx([v for _, v in replay], abs=1e-6)
    assert last_r == pytest.approx(last_e, abs=1e-6)
