"""``TrainModule``: the LightningModule-shaped user API of the framework.

Users of the reference write a ``pl.LightningModule`` with ``training_step``,
``validation_step``, ``configure_optimizers``, ``self.log(..., sync_dist=True)`` and
``save_hyperparameters()`` (jobs/train_lightning_ddp.py:51-88) and load it back with
``load_from_checkpoint(path, **overrides)`` (dags/azure_manual_deploy.py:109).  The same
surface exists here, implemented natively (Lightning is not a dependency), so a reference
module ports by changing its base class; checkpoints it writes stay Lightning-2.1-loadable.
"""
from __future__ import annotations

import inspect
from typing import Any, Dict, Optional

import torch
import torch.nn as nn


class AttributeDict(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v


class TrainModule(nn.Module):
    def __init__(self):
        super().__init__()
        object.__setattr__(self, "_hparams", AttributeDict())
        object.__setattr__(self, "_hparams_name", None)
        object.__setattr__(self, "_trainer", None)
        object.__setattr__(self, "_logged", {})

    # ------------------------------------------------------------------ hparams
    def save_hyperparameters(self, *names: str):
        """Collect the __init__ arguments of the outermost constructor frame of ``self``."""
        frame = inspect.currentframe().f_back
        init_args: Dict[str, Any] = {}
        while frame is not None:
            code = frame.f_code
            if code.co_name == "__init__" and frame.f_locals.get("self") is self:
                info = inspect.getargvalues(frame)
                args = {k: info.locals[k] for k in info.args if k != "self"}
                if info.keywords and isinstance(info.locals.get(info.keywords), dict):
                    args.update(info.locals[info.keywords])
                init_args = args
            frame = frame.f_back
        if names:
            init_args = {k: v for k, v in init_args.items() if k in names}
        clean = {}
        for k, v in init_args.items():
            if isinstance(v, (list, tuple)):
                v = list(v)
            clean[k] = v
        self._set_hparams(clean)

    def _set_hparams(self, d: Dict[str, Any]):
        object.__setattr__(self, "_hparams", AttributeDict(d))
        object.__setattr__(self, "_hparams_name", "kwargs")

    @property
    def hparams(self) -> AttributeDict:
        return self._hparams

    # ------------------------------------------------------------------ trainer hooks
    @property
    def trainer(self):
        return self._trainer

    @property
    def global_rank(self) -> int:
        return self._trainer.global_rank if self._trainer is not None else 0

    @property
    def device(self) -> torch.device:
        for p in self.parameters():
            return p.device
        return torch.device("cpu")

    def log(self, name: str, value, sync_dist: bool = False, prog_bar: bool = False, on_step: Optional[bool] = None,
            on_epoch: Optional[bool] = None, batch_size: Optional[int] = None, logger: bool = True, **_):
        if self._trainer is not None:
            self._trainer._log_from_module(name, value, sync_dist=sync_dist, prog_bar=prog_bar, on_step=on_step,
                                           on_epoch=on_epoch, batch_size=batch_size)
        else:  # detached: a stored loss must not keep the autograd graph (and its streams) alive
            self._logged[name] = value.detach() if isinstance(value, torch.Tensor) else value

    def training_step(self, batch, batch_idx):  # pragma: no cover - abstract
        raise NotImplementedError

    def validation_step(self, batch, batch_idx):
        return None

    def configure_optimizers(self):
        return torch.optim.Adam(self.parameters(), lr=1e-3)

    def on_save_checkpoint(self, checkpoint: Dict[str, Any]) -> None:
        pass

    def on_load_checkpoint(self, checkpoint: Dict[str, Any]) -> None:
        pass

    # ------------------------------------------------------------------ loading
    @classmethod
    def load_from_checkpoint(cls, checkpoint_path: str, map_location=None, strict: bool = True, **kwargs):
        from ..ckpt.lightning_io import load_checkpoint

        ckpt = load_checkpoint(checkpoint_path, map_location=map_location or "cpu")
        hp = dict(ckpt.get("hyper_parameters", {}) or {})
        hp.update(kwargs)
        sig = inspect.signature(cls.__init__)
        accepts_var_kw = any(p.kind == p.VAR_KEYWORD for p in sig.parameters.values())
        if not accepts_var_kw:
            hp = {k: v for k, v in hp.items() if k in sig.parameters}
        model = cls(**hp)
        model.on_load_checkpoint(ckpt)
        model.load_state_dict(ckpt["state_dict"], strict=strict)
        return model
