"""Lightning-2.1-compatible checkpoint files.

The reference's checkpoints are written by Lightning's ``ModelCheckpoint`` /
``trainer.save_checkpoint`` (jobs/train_lightning_ddp.py:103-110) and consumed by
``WeatherClassifier.load_from_checkpoint(path, input_dim=5)`` inside the Azure ``score.py``
(dags/azure_manual_deploy.py:109), which runs torch 2.1 + Lightning 2.1 on CPU.  A checkpoint
written here therefore has exactly the top-level keys of a Lightning 2.1 ``dump_checkpoint``
(``epoch, global_step, pytorch-lightning_version, state_dict, loops, callbacks,
optimizer_states, lr_schedulers, hparams_name, hyper_parameters``), fp32 CPU tensors only, and
only plain containers / tensors so it loads under ``torch.load(weights_only=True)`` (torch >= 2.6
default) as well as under torch 2.1's unpickler.  Writes are atomic (tmp file + rename).
"""
from __future__ import annotations

import os
import tempfile
from typing import Any, Dict, List, Optional

import torch

LIGHTNING_VERSION = "2.1.0"
CHECKPOINT_KEYS = (
    "epoch", "global_step", "pytorch-lightning_version", "state_dict", "loops", "callbacks",
    "optimizer_states", "lr_schedulers", "hparams_name", "hyper_parameters",
)


def _progress(ready: int, completed: Optional[int] = None, started: Optional[int] = None,
              processed: Optional[int] = None) -> Dict[str, int]:
    completed = ready if completed is None else completed
    d = {"ready": int(ready), "completed": int(completed)}
    if started is not None:
        d["started"] = int(started)
    if processed is not None:
        d["processed"] = int(processed)
    return d


def loops_state(epoch: int, global_step: int, batches_in_epoch: int, val_batches: int) -> Dict[str, Any]:
    """Lightning 2.1 ``loops`` entry (fit/validate/test/predict progress trackers)."""
    bp_total = _progress(global_step, global_step, global_step, global_step)
    bp_cur = _progress(batches_in_epoch, batches_in_epoch, batches_in_epoch, batches_in_epoch)
    vb = _progress(val_batches, val_batches, val_batches, val_batches)
    opt_step = {"total": _progress(global_step), "current": _progress(batches_in_epoch)}
    zero = {"total": _progress(global_step, global_step, global_step),
            "current": _progress(batches_in_epoch, batches_in_epoch, batches_in_epoch)}
    empty_batch = {"total": _progress(0, 0, 0, 0), "current": _progress(0, 0, 0, 0), "is_last_batch": False}
    return {
        "fit_loop": {
            "state_dict": {},
            "epoch_loop.state_dict": {"_batches_that_stepped": int(global_step)},
            "epoch_loop.batch_progress": {"total": bp_total, "current": bp_cur, "is_last_batch": True},
            "epoch_loop.scheduler_progress": {"total": _progress(0), "current": _progress(0)},
            "epoch_loop.automatic_optimization.state_dict": {},
            "epoch_loop.automatic_optimization.optim_progress": {"optimizer": {"step": opt_step, "zero_grad": zero}},
            "epoch_loop.manual_optimization.state_dict": {},
            "epoch_loop.manual_optimization.optim_step_progress": {"total": _progress(0), "current": _progress(0)},
            "epoch_loop.val_loop.state_dict": {},
            "epoch_loop.val_loop.batch_progress": {"total": vb, "current": vb, "is_last_batch": True},
            "epoch_progress": {"total": _progress(epoch + 1, epoch, epoch + 1, epoch + 1),
                               "current": _progress(epoch + 1, epoch, epoch + 1, epoch + 1)},
        },
        "validate_loop": {"state_dict": {}, "batch_progress": empty_batch},
        "test_loop": {"state_dict": {}, "batch_progress": empty_batch},
        "predict_loop": {"state_dict": {}, "batch_progress": {"total": _progress(0, 0, 0, 0),
                                                              "current": _progress(0, 0, 0, 0)}},
    }


def cpu_state_dict(sd: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    return {k: v.detach().to("cpu", torch.float32 if v.is_floating_point() else v.dtype).clone()
            for k, v in sd.items()}


def build_checkpoint(state_dict: Dict[str, torch.Tensor], epoch: int, global_step: int,
                     optimizer_states: Optional[List[Dict]] = None, callbacks: Optional[Dict[str, Dict]] = None,
                     hyper_parameters: Optional[Dict[str, Any]] = None, hparams_name: Optional[str] = "kwargs",
                     batches_in_epoch: int = 0, val_batches: int = 0) -> Dict[str, Any]:
    ckpt: Dict[str, Any] = {
        "epoch": int(epoch),
        "global_step": int(global_step),
        "pytorch-lightning_version": LIGHTNING_VERSION,
        "state_dict": cpu_state_dict(state_dict),
        "loops": loops_state(epoch, global_step, batches_in_epoch, val_batches),
        "callbacks": callbacks or {},
        "optimizer_states": optimizer_states or [],
        "lr_schedulers": [],
    }
    if hyper_parameters is not None:
        ckpt["hparams_name"] = hparams_name
        ckpt["hyper_parameters"] = dict(hyper_parameters)
    return ckpt


def save_checkpoint(ckpt: Dict[str, Any], path: str) -> str:
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    fd, tmp = tempfile.mkstemp(prefix=".tmp-", suffix=".ckpt", dir=d)
    os.close(fd)
    try:
        torch.save(ckpt, tmp)
        os.replace(tmp, path)
    finally:
        if os.path.exists(tmp):
            os.remove(tmp)
    return path


def load_checkpoint(path: str, map_location="cpu") -> Dict[str, Any]:
    """Safe load: never unpickles arbitrary objects (weights_only=True)."""
    return torch.load(path, map_location=map_location, weights_only=True)


def elastic_restart_count() -> int:
    """How many times torchrun has restarted this job's workers (0 on the first attempt)."""
    try:
        return int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0"))
    except ValueError:
        return 0


def resume_checkpoint(model_dir: str, requested: bool = False, name: str = "last.ckpt") -> Optional[str]:
    """The checkpoint ``Trainer.fit(ckpt_path=...)`` should resume from, or None.

    The reference always starts from scratch (train_lightning_ddp.py:143), so a fresh launch resumes
    only when asked (``--resume``).  A torchrun elastic RESTART (``--max-restarts``, after a rank
    failed) resumes from ``last.ckpt`` when one exists: the restarted workers continue the run at
    the epoch after the last completed one instead of silently retraining from epoch 0."""
    path = os.path.join(model_dir, name)
    if (requested or elastic_restart_count() > 0) and os.path.exists(path):
        return path
    return None
