"""Experiment loggers used by the trainer.

``MLFlowLogger`` mirrors ``pytorch_lightning.loggers.MLFlowLogger(experiment_name,
tracking_uri, log_model=True)`` (jobs/train_lightning_ddp.py:92-96): the run is created lazily
on global rank 0 only, hyper-parameters become params, metrics are logged with the global
step, and with ``log_model=True`` every checkpoint the ``ModelCheckpoint`` produced is uploaded
under ``model/checkpoints/<stem>/`` when the run is finalized.  ``experiment.log_artifact``
is exposed so the reference's explicit ``best_checkpoints`` upload (:157-161) works unchanged.
Metric calls are buffered and flushed as ``runs/log-batch`` requests of up to 1,000 metrics (MLflow's
cap; one HTTP round trip per flush instead of one per metric); the trainer also flushes at the end
of every epoch, so a run's metrics are visible epoch by epoch.
"""
from __future__ import annotations

import json
import os
from typing import Any, Dict, List, Optional

from .mlflow_client import MlflowClient


class Logger:
    def log_hyperparams(self, params: Dict[str, Any]): ...
    def log_metrics(self, metrics: Dict[str, float], step: int): ...
    def after_save_checkpoint(self, path: str): ...
    def finalize(self, status: str = "success"): ...
    def flush(self): ...


class InMemoryLogger(Logger):
    """Collects everything in memory (tests, benchmarks)."""

    def __init__(self):
        self.params: Dict[str, Any] = {}
        self.metrics: List[Dict[str, Any]] = []
        self.checkpoints: List[str] = []
        self.status = None

    def log_hyperparams(self, params):
        self.params.update(params)

    def log_metrics(self, metrics, step):
        self.metrics.append({"step": step, **{k: float(v) for k, v in metrics.items()}})

    def after_save_checkpoint(self, path):
        self.checkpoints.append(path)

    def finalize(self, status="success"):
        self.status = status

    def history(self, key: str):
        return [(m["step"], m[key]) for m in self.metrics if key in m]


class MLFlowLogger(Logger):
    def __init__(self, experiment_name: str = "lightning_logs", tracking_uri: Optional[str] = None,
                 log_model: bool = False, run_name: Optional[str] = None, tags: Optional[Dict[str, str]] = None,
                 flush_every: int = 1000):
        self.experiment_name = experiment_name
        self.tracking_uri = tracking_uri or os.environ.get("MLFLOW_TRACKING_URI")
        self.log_model = log_model
        self.run_name = run_name
        self.tags = dict(tags or {})
        self.flush_every = flush_every
        self._client: Optional[MlflowClient] = None
        self._run_id: Optional[str] = None
        self._experiment_id: Optional[str] = None
        self._buffer: List[Dict[str, Any]] = []
        self._checkpoints: List[str] = []
        self.rank_zero = True

    @property
    def experiment(self) -> MlflowClient:
        if self._client is None:
            self._client = MlflowClient(self.tracking_uri)
            self._experiment_id = self._client.get_or_create_experiment(self.experiment_name)
            info = self._client.create_run(self._experiment_id, run_name=self.run_name or "", tags=self.tags)
            self._run_id = info.run_id
        return self._client

    @property
    def run_id(self) -> Optional[str]:
        if self.rank_zero:
            _ = self.experiment
        return self._run_id

    @property
    def experiment_id(self):
        _ = self.experiment
        return self._experiment_id

    def log_hyperparams(self, params: Dict[str, Any]):
        if not self.rank_zero or not params:
            return
        flat = {}
        for k, v in params.items():
            flat[k] = json.dumps(v) if isinstance(v, (list, dict, tuple)) else v
        self.experiment.log_batch(self.run_id, params=[{"key": k, "value": v} for k, v in flat.items()])

    def log_metrics(self, metrics: Dict[str, float], step: int):
        if not self.rank_zero:
            return
        import time

        ts = int(time.time() * 1000)
        for k, v in metrics.items():
            self._buffer.append({"key": k, "value": float(v), "step": int(step), "timestamp": ts})
        if len(self._buffer) >= self.flush_every:
            self.flush()

    def log_metric_series(self, key: str, points, extra: Optional[Dict[str, float]] = None):
        """log_metrics({key: v, **extra}, step) for every (step, v) of points, in one call."""
        if not self.rank_zero:
            return
        import time

        ts = int(time.time() * 1000)
        ex = [(k, float(v)) for k, v in (extra or {}).items()]
        buf = self._buffer
        for step, v in points:
            buf.append({"key": key, "value": float(v), "step": int(step), "timestamp": ts})
            for k, xv in ex:
                buf.append({"key": k, "value": xv, "step": int(step), "timestamp": ts})
        if len(buf) >= self.flush_every:
            self.flush()

    def flush(self):
        if not self.rank_zero or not self._buffer:
            return
        buf, self._buffer = self._buffer, []
        for i in range(0, len(buf), 1000):  # MLflow caps log-batch at 1000 metrics
            self.experiment.log_batch(self.run_id, metrics=buf[i: i + 1000])

    def after_save_checkpoint(self, path: str):
        if path not in self._checkpoints:
            self._checkpoints.append(path)

    def finalize(self, status: str = "success"):
        if not self.rank_zero:
            return
        self.flush()
        if self.log_model:
            for p in self._checkpoints:
                if os.path.exists(p):
                    stem = os.path.splitext(os.path.basename(p))[0]
                    self.experiment.log_artifact(self.run_id, p, f"model/checkpoints/{stem}")
        state = {"success": "FINISHED", "failed": "FAILED", "finished": "FINISHED"}.get(status, "FINISHED")
        self.experiment.set_terminated(self.run_id, state)
