"""MLP model family.

``WeatherClassifier`` is the reference model, layer for layer
(jobs/train_lightning_ddp.py:51-88): ``net = Sequential(Linear(D,64), ReLU, Dropout(0.2),
Linear(64,2))``, cross-entropy, ``save_hyperparameters()`` -> ``{"input_dim": D}``, Adam(lr=0.01).
Its state_dict keys (``net.0.weight`` ... ``net.3.bias``) are the contract consumed by the
deployment ``score.py`` (dags/azure_manual_deploy.py:66-75,109).

``MLPClassifier`` generalises it (depth, widths, dropout, loss in {ce, mse}) and keeps the same
``net.<3*i>`` key scheme, which covers the BASELINE.json configs (3-layer/128-h weather MLP,
4-layer/1024-h x 256-feature tabular MLP).  Both expose ``fused_spec()`` so the trainer can run
them on the fused HIP kernels (small widths) or the bf16 MFMA GEMM path (large widths); the
torch ``forward`` is the CPU path and the numerical reference.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..trainer.module import TrainModule


class MLPClassifier(TrainModule):
    def __init__(self, input_dim: int, hidden: Sequence[int] = (64,), num_classes: int = 2, dropout: float = 0.2,
                 loss: str = "ce", lr: float = 0.01):
        super().__init__()
        self.save_hyperparameters()
        if loss not in ("ce", "mse"):
            raise ValueError("loss must be 'ce' or 'mse'")
        dims = [int(input_dim)] + [int(h) for h in hidden] + [int(num_classes)]
        layers: List[nn.Module] = []
        for i in range(len(dims) - 1):
            layers.append(nn.Linear(dims[i], dims[i + 1]))
            if i < len(dims) - 2:
                layers += [nn.ReLU(), nn.Dropout(dropout)]
        self.net = nn.Sequential(*layers)
        self.dims = dims
        self.dropout_p = float(dropout)
        self.loss_kind = loss
        self.lr = lr

    def forward(self, x):
        return self.net(x)

    def compute_loss(self, logits, y):
        if self.loss_kind == "ce":
            return F.cross_entropy(logits, y)
        return F.mse_loss(logits, F.one_hot(y, logits.shape[-1]).to(logits.dtype))

    def training_step(self, batch, batch_idx):
        x, y = batch
        loss = self.compute_loss(self(x), y)
        self.log("train_loss", loss, sync_dist=True)
        return loss

    def validation_step(self, batch, batch_idx):
        x, y = batch
        logits = self(x)
        loss = self.compute_loss(logits, y)
        acc = (torch.argmax(logits, dim=1) == y).float().mean()
        self.log("val_loss", loss, sync_dist=True, prog_bar=True)
        self.log("val_acc", acc, sync_dist=True, prog_bar=True)
        return loss

    def configure_optimizers(self):
        return torch.optim.Adam(self.parameters(), lr=self.lr)

    # ---- fused-engine contract
    def fused_spec(self):
        return {"dims": list(self.dims), "dropout": self.dropout_p, "loss": self.loss_kind}

    def linear_layers(self) -> List[nn.Linear]:
        return [m for m in self.net if isinstance(m, nn.Linear)]


class WeatherClassifier(MLPClassifier):
    """Reference model: Linear(D,64)-ReLU-Dropout(0.2)-Linear(64,2), CE, Adam(lr=0.01)."""

    def __init__(self, input_dim: int):
        super().__init__(input_dim=input_dim, hidden=(64,), num_classes=2, dropout=0.2, loss="ce", lr=0.01)
        # the reference records exactly {"input_dim": D} (save_hyperparameters at :53)
        self._set_hparams({"input_dim": int(input_dim)})


def build_mlp(name: str, input_dim: int, hidden: Optional[Sequence[int]] = None, num_classes: int = 2,
              dropout: float = 0.2, loss: str = "ce", lr: float = 0.01) -> MLPClassifier:
    if name == "weather":
        return WeatherClassifier(input_dim)
    # name -> (hidden widths, dropout, loss, lr); BASELINE.json configs 1-4
    presets = {
        "weather-mlp-3x128": ((128, 128), 0.2, "ce", 0.01),
        "tabular-mlp-4x1024": ((1024, 1024, 1024), 0.0, "mse", 1e-3),
    }
    if name in presets and hidden is None:
        hidden, dropout, loss, lr = presets[name]
    return MLPClassifier(input_dim, hidden=hidden or (64,), num_classes=num_classes, dropout=dropout, loss=loss, lr=lr)
