"""``ModelCheckpoint`` with Lightning 2.1 semantics (jobs/train_lightning_ddp.py:103-110).

* filename template ``"weather-best-{epoch:02d}-{val_loss:.2f}"`` is expanded with metric names
  auto-inserted -> ``weather-best-epoch=03-val_loss=0.45.ckpt``; a clash gets ``-v1``, ``-v2``...;
* top-k on ``monitor`` with ``mode`` (min/max); the displaced best file is deleted;
* ``save_last=True`` writes ``last.ckpt`` after every save event;
* ``best_model_path`` / ``best_model_score`` / ``last_model_path`` / ``best_k_models`` and the
  callback ``state_dict`` stored in the checkpoint under Lightning's state key.
Only global rank 0 touches the filesystem; the trainer barriers all ranks afterwards.
"""
from __future__ import annotations

import math
import os
import re
from typing import Any, Callable, Dict, Optional

import torch

CHECKPOINT_NAME_LAST = "last"
FILE_EXTENSION = ".ckpt"


class ModelCheckpoint:
    def __init__(self, dirpath: Optional[str] = None, filename: Optional[str] = None, monitor: Optional[str] = None,
                 mode: str = "min", save_top_k: int = 1, save_last: Optional[bool] = None,
                 auto_insert_metric_name: bool = True, every_n_epochs: int = 1, verbose: bool = False):
        if mode not in ("min", "max"):
            raise ValueError("mode must be 'min' or 'max'")
        self.dirpath = dirpath
        self.filename = filename
        self.monitor = monitor
        self.mode = mode
        self.save_top_k = save_top_k
        self.save_last = save_last
        self.auto_insert_metric_name = auto_insert_metric_name
        self.every_n_epochs = every_n_epochs
        self.verbose = verbose
        self.best_k_models: Dict[str, float] = {}
        self.kth_best_model_path = ""
        self.best_model_score: Optional[float] = None
        self.best_model_path = ""
        self.last_model_path = ""
        self.current_score: Optional[float] = None
        self.kth_value = math.inf if mode == "min" else -math.inf

    # ------------------------------------------------------------------ naming
    @property
    def state_key(self) -> str:
        return ("ModelCheckpoint{" + f"'monitor': {self.monitor!r}, 'mode': {self.mode!r}, "
                f"'every_n_train_steps': 0, 'every_n_epochs': {self.every_n_epochs}, "
                "'train_time_interval': None}")

    def format_checkpoint_name(self, metrics: Dict[str, Any], ver: Optional[int] = None) -> str:
        filename = self.filename or "{epoch}-{step}"
        groups = re.findall(r"(\{.*?)[:\}]", filename)
        values = dict(metrics)
        for group in groups:
            name = group[1:]
            if self.auto_insert_metric_name:
                filename = filename.replace(group, name + "={" + name)
            if name not in values:
                values[name] = 0
            v = values[name]
            if isinstance(v, torch.Tensor):
                values[name] = v.item()
        filename = filename.format(**values)
        if ver is not None:
            filename = f"{filename}-v{ver}"
        return os.path.join(self.dirpath or ".", filename + FILE_EXTENSION)

    def _unique_path(self, metrics: Dict[str, Any], del_path: Optional[str]) -> str:
        path = self.format_checkpoint_name(metrics)
        ver = 1
        while os.path.exists(path) and path != del_path:
            path = self.format_checkpoint_name(metrics, ver=ver)
            ver += 1
        return path

    # ------------------------------------------------------------------ decisions
    def _better(self, current: float, ref: float) -> bool:
        if math.isnan(current):
            return False
        return current < ref if self.mode == "min" else current > ref

    def check_monitor_top_k(self, current: Optional[float]) -> bool:
        if current is None:
            return False
        if self.save_top_k == -1:
            return True
        if len(self.best_k_models) < self.save_top_k:
            return True
        return self._better(current, self.kth_value)

    def on_validation_end(self, metrics: Dict[str, Any], save_fn: Callable[[str], None], is_rank_zero: bool,
                          epoch: int) -> Optional[str]:
        """Apply top-k + save_last for the current metrics. ``save_fn(path)`` writes the file
        (it embeds ``self.state_dict()`` captured after this decision)."""
        if self.every_n_epochs < 1 or (epoch + 1) % self.every_n_epochs != 0:
            return None
        saved = None
        if self.save_top_k != 0 and self.monitor is not None:
            cur = metrics.get(self.monitor)
            cur = None if cur is None else float(cur)
            self.current_score = cur
            if self.check_monitor_top_k(cur):
                del_path = None
                if len(self.best_k_models) == self.save_top_k and self.save_top_k > 0:
                    del_path = self.kth_best_model_path
                    self.best_k_models.pop(del_path, None)
                path = self._unique_path(metrics, del_path)
                if math.isnan(cur):
                    # Lightning 2.1 _update_best_and_save: a NaN score is stored as the worst value,
                    # so it can never be the "best" checkpoint once a real score arrives
                    cur = float("inf") if self.mode == "min" else float("-inf")
                    self.current_score = cur
                self.best_k_models[path] = cur
                reverse = self.mode == "max"
                ordered = sorted(self.best_k_models.items(), key=lambda kv: kv[1], reverse=not reverse)
                # kth = worst kept
                self.kth_best_model_path, self.kth_value = ordered[0]
                best = sorted(self.best_k_models.items(), key=lambda kv: kv[1], reverse=reverse)[0]
                self.best_model_path, self.best_model_score = best
                if is_rank_zero:
                    save_fn(path)
                    if del_path and del_path != path and os.path.exists(del_path) and del_path != self.last_model_path:
                        os.remove(del_path)
                saved = path
        elif self.save_top_k != 0 and self.monitor is None:
            path = self._unique_path(metrics, self.best_model_path or None)
            prev = self.best_model_path
            self.best_model_path = path
            if is_rank_zero:
                save_fn(path)
                if prev and prev != path and os.path.exists(prev):
                    os.remove(prev)
            saved = path
        if self.save_last:
            last = os.path.join(self.dirpath or ".", CHECKPOINT_NAME_LAST + FILE_EXTENSION)
            self.last_model_path = last
            if is_rank_zero:
                save_fn(last)
        return saved

    # ------------------------------------------------------------------ state
    def state_dict(self) -> Dict[str, Any]:
        t = lambda x: None if x is None else torch.tensor(float(x))  # noqa: E731
        return {
            "monitor": self.monitor,
            "best_model_score": t(self.best_model_score),
            "best_model_path": self.best_model_path,
            "current_score": t(self.current_score),
            "dirpath": self.dirpath,
            "best_k_models": {k: torch.tensor(float(v)) for k, v in self.best_k_models.items()},
            "kth_best_model_path": self.kth_best_model_path,
            "kth_value": torch.tensor(float(self.kth_value)),
            "last_model_path": self.last_model_path,
        }

    def load_state_dict(self, sd: Dict[str, Any]):
        f = lambda x: None if x is None else float(x)  # noqa: E731
        if sd.get("dirpath") == self.dirpath:
            self.best_model_score = f(sd.get("best_model_score"))
            self.best_model_path = sd.get("best_model_path", "")
            self.best_k_models = {k: float(v) for k, v in sd.get("best_k_models", {}).items()}
            self.kth_best_model_path = sd.get("kth_best_model_path", "")
            kv = f(sd.get("kth_value"))
            if kv is not None:
                self.kth_value = kv
            self.last_model_path = sd.get("last_model_path", "")
        self.current_score = f(sd.get("current_score"))
