"""Dependency-free MLflow client (the ``mlflow`` package is not available offline).

Covers what the reference uses:
  * training side (jobs/train_lightning_ddp.py:92-96,155-161): experiment ``weather_forecasting``,
    run creation, params, metrics (``train_loss`` every 5 steps, ``val_loss``, ``val_acc``,
    ``epoch``), ``log_artifact(run_id, path, "best_checkpoints")``;
  * deploy side (dags/azure_manual_deploy.py:31-45): ``get_experiment_by_name``,
    ``search_runs(order_by=["metrics.val_loss ASC"], max_results=1)`` (latest value per run),
    ``download_artifacts(run_id, "best_checkpoints", dst)``.

Two stores behind one ``MlflowClient`` API:
  * ``RestStore`` - the MLflow 2.x REST API (``/api/2.0/mlflow/...``) of the tracking server
    (``http://mlflow-server:5000``); artifacts go straight to the run's ``artifact_uri`` when it
    is a filesystem path (the compose file shares ``/mlflow/artifacts`` by bind mount,
    docker-compose.yml:33,129,188) or through the ``mlflow-artifacts`` HTTP proxy.
  * ``FileStore`` - MLflow's own ``mlruns/`` file layout (meta.yaml, metrics/, params/, tags/,
    artifacts/), readable by a stock ``mlflow ui``; used for ``file:`` URIs and local paths.
"""
from __future__ import annotations

import json
import os
import re
import shutil
import time
import uuid
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence
from urllib.parse import quote, urlparse

RUN_STATUS = {"RUNNING": 1, "SCHEDULED": 2, "FINISHED": 3, "FAILED": 4, "KILLED": 5}
RUN_STATUS_NAME = {v: k for k, v in RUN_STATUS.items()}


def _now_ms() -> int:
    return int(time.time() * 1000)


@dataclass
class RunInfo:
    run_id: str
    experiment_id: str
    status: str
    start_time: int
    end_time: Optional[int]
    artifact_uri: str
    run_name: str = ""

    @property
    def run_uuid(self):
        return self.run_id


@dataclass
class RunData:
    metrics: Dict[str, float] = field(default_factory=dict)
    params: Dict[str, str] = field(default_factory=dict)
    tags: Dict[str, str] = field(default_factory=dict)


@dataclass
class Run:
    info: RunInfo
    data: RunData


@dataclass
class Experiment:
    experiment_id: str
    name: str
    artifact_location: str
    lifecycle_stage: str = "active"


def _parse_order_by(order_by: Optional[Sequence[str]]):
    keys = []
    for ob in order_by or []:
        parts = ob.strip().split()
        key = parts[0]
        asc = not (len(parts) > 1 and parts[1].upper() == "DESC")
        keys.append((key, asc))
    return keys


def _sort_runs(runs: List[Run], order_by) -> List[Run]:
    keys = _parse_order_by(order_by)
    for key, asc in reversed(keys):
        kind, _, name = key.partition(".")

        def getter(r, kind=kind, name=name):
            if kind == "metrics":
                return r.data.metrics.get(name)
            if kind == "params":
                return r.data.params.get(name)
            if kind == "attributes" or kind == "attribute":
                return getattr(r.info, name, None)
            return None

        present = [r for r in runs if getter(r) is not None]
        missing = [r for r in runs if getter(r) is None]
        present.sort(key=getter, reverse=not asc)
        runs = present + missing  # MLflow puts NULLs last
    if not keys:
        runs.sort(key=lambda r: r.info.start_time, reverse=True)
    return runs


# ----------------------------------------------------------------------------- file store
_EXP_ID_RE = re.compile(r"[0-9]{1,18}")
_RUN_ID_RE = re.compile(r"[0-9a-f]{32}")


class FileStore:
    def __init__(self, root: str):
        self.root = os.path.abspath(root)
        os.makedirs(self.root, exist_ok=True)
        if not os.path.exists(os.path.join(self.root, "0", "meta.yaml")):
            self._write_exp_meta("0", "Default")

    # yaml without dependency issues: MLflow's meta.yaml is simple key: value
    @staticmethod
    def _dump_yaml(path: str, d: Dict[str, Any]):
        import yaml

        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            yaml.safe_dump(d, f, default_flow_style=False, sort_keys=True)
        os.replace(tmp, path)

    @staticmethod
    def _load_yaml(path: str) -> Dict[str, Any]:
        import yaml

        with open(path) as f:
            return yaml.safe_load(f) or {}

    def _write_exp_meta(self, exp_id: str, name: str):
        d = os.path.join(self.root, exp_id)
        os.makedirs(d, exist_ok=True)
        self._dump_yaml(os.path.join(d, "meta.yaml"), {
            "artifact_location": "file://" + d,
            "creation_time": _now_ms(),
            "experiment_id": exp_id,
            "last_update_time": _now_ms(),
            "lifecycle_stage": "active",
            "name": name,
        })

    def list_experiments(self) -> List[Experiment]:
        out = []
        for e in sorted(os.listdir(self.root)):
            meta = os.path.join(self.root, e, "meta.yaml")
            if os.path.exists(meta):
                m = self._load_yaml(meta)
                out.append(Experiment(str(m["experiment_id"]), m["name"], m.get("artifact_location", ""),
                                      m.get("lifecycle_stage", "active")))
        return out

    def get_experiment_by_name(self, name: str) -> Optional[Experiment]:
        for e in self.list_experiments():
            if e.name == name and e.lifecycle_stage == "active":
                return e
        return None

    def create_experiment(self, name: str) -> str:
        if self.get_experiment_by_name(name) is not None:
            raise ValueError(f"experiment {name!r} already exists")
        ids = [int(e.experiment_id) for e in self.list_experiments() if e.experiment_id.isdigit()]
        exp_id = str(max(ids + [0]) + 1)
        self._write_exp_meta(exp_id, name)
        return exp_id

    @staticmethod
    def _check_exp_id(exp_id) -> str:
        """Experiment ids are decimal strings (MLflow's file store); anything else could walk out
        of the store root when joined into a path."""
        exp_id = str(exp_id)
        if not _EXP_ID_RE.fullmatch(exp_id):
            raise ValueError(f"invalid experiment id {exp_id!r}")
        return exp_id

    @staticmethod
    def _check_run_id(run_id) -> str:
        """Run ids are 32 lowercase hex characters (uuid4().hex, as MLflow creates them)."""
        run_id = str(run_id)
        if not _RUN_ID_RE.fullmatch(run_id):
            raise ValueError(f"invalid run id {run_id!r}")
        return run_id

    def _run_dir(self, run_id: str, exp_id: Optional[str] = None) -> str:
        run_id = self._check_run_id(run_id)
        if exp_id is not None:
            return os.path.join(self.root, self._check_exp_id(exp_id), run_id)
        for e in os.listdir(self.root):
            d = os.path.join(self.root, e, run_id)
            if os.path.isdir(d):
                return d
        raise KeyError(f"run {run_id} not found")

    def create_run(self, experiment_id: str, run_name: str = "", tags: Optional[Dict[str, str]] = None) -> RunInfo:
        experiment_id = self._check_exp_id(experiment_id)
        if not os.path.exists(os.path.join(self.root, experiment_id, "meta.yaml")):
            raise KeyError(f"experiment {experiment_id} not found")
        run_id = uuid.uuid4().hex
        d = os.path.join(self.root, experiment_id, run_id)
        for sub in ("metrics", "params", "tags", "artifacts"):
            os.makedirs(os.path.join(d, sub), exist_ok=True)
        art = "file://" + os.path.join(d, "artifacts")
        start = _now_ms()
        self._dump_yaml(os.path.join(d, "meta.yaml"), {
            "artifact_uri": art, "end_time": None, "entry_point_name": "", "experiment_id": experiment_id,
            "lifecycle_stage": "active", "run_id": run_id, "run_name": run_name, "run_uuid": run_id,
            "source_name": "", "source_type": 4, "source_version": "", "start_time": start,
            "status": RUN_STATUS["RUNNING"], "tags": [], "user_id": os.environ.get("USER", "dct"),
        })
        for k, v in (tags or {}).items():
            self.set_tag(run_id, k, v)
        if run_name:
            self.set_tag(run_id, "mlflow.runName", run_name)
        return RunInfo(run_id, experiment_id, "RUNNING", start, None, art, run_name)

    @staticmethod
    def _safe_key(k: str) -> str:
        if k.startswith("/") or ".." in k.split("/"):
            raise ValueError(f"invalid key {k!r}")
        return k

    def log_metric(self, run_id: str, key: str, value: float, timestamp: Optional[int] = None, step: int = 0):
        p = os.path.join(self._run_dir(run_id), "metrics", self._safe_key(key))
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "a") as f:
            f.write(f"{timestamp or _now_ms()} {float(value)} {int(step)}\n")

    def log_param(self, run_id: str, key: str, value: Any):
        p = os.path.join(self._run_dir(run_id), "params", self._safe_key(key))
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "w") as f:
            f.write(str(value))

    def set_tag(self, run_id: str, key: str, value: Any):
        p = os.path.join(self._run_dir(run_id), "tags", self._safe_key(key))
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "w") as f:
            f.write(str(value))

    def log_batch(self, run_id: str, metrics=(), params=(), tags=()):
        d = self._run_dir(run_id)  # validates the id and that the run exists, even for an empty batch
        # one append per metric KEY (lines in the batch's order), not an open + run lookup per value:
        # a 20k-step epoch logs 8k values (train_loss every 5 steps + epoch)
        lines: Dict[str, List[str]] = {}
        now = None
        for m in metrics:
            ts = m.get("timestamp")
            if not ts:
                now = now or _now_ms()
                ts = now
            lines.setdefault(self._safe_key(m["key"]), []).append(
                f"{ts} {float(m['value'])} {int(m.get('step', 0))}\n")
        for key, ls in lines.items():
            p = os.path.join(d, "metrics", key)
            if "/" in key:
                os.makedirs(os.path.dirname(p), exist_ok=True)
            with open(p, "a") as f:
                f.write("".join(ls))
        for p in params:
            self.log_param(run_id, p["key"], p["value"])
        for t in tags:
            self.set_tag(run_id, t["key"], t["value"])

    def update_run(self, run_id: str, status: str, end_time: Optional[int] = None):
        d = self._run_dir(run_id)
        meta = self._load_yaml(os.path.join(d, "meta.yaml"))
        meta["status"] = RUN_STATUS[status]
        meta["end_time"] = end_time or _now_ms()
        self._dump_yaml(os.path.join(d, "meta.yaml"), meta)

    def get_run(self, run_id: str) -> Run:
        d = self._run_dir(run_id)
        meta = self._load_yaml(os.path.join(d, "meta.yaml"))
        data = RunData()
        mdir = os.path.join(d, "metrics")
        for root, _, files in os.walk(mdir):
            for fn in files:
                key = os.path.relpath(os.path.join(root, fn), mdir)
                best = None
                with open(os.path.join(root, fn)) as f:
                    for line in f:
                        parts = line.split()
                        if len(parts) >= 2:
                            ts, val = int(parts[0]), float(parts[1])
                            st = int(parts[2]) if len(parts) > 2 else 0
                            # latest value = max (step, timestamp) like MLflow's latest_metrics
                            if best is None or (st, ts) >= (best[0], best[1]):
                                best = (st, ts, val)
                if best is not None:
                    data.metrics[key] = best[2]
        for sub, tgt in (("params", data.params), ("tags", data.tags)):
            sd = os.path.join(d, sub)
            for root, _, files in os.walk(sd):
                for fn in files:
                    with open(os.path.join(root, fn)) as f:
                        tgt[os.path.relpath(os.path.join(root, fn), sd)] = f.read()
        info = RunInfo(meta["run_id"], str(meta["experiment_id"]), RUN_STATUS_NAME.get(meta["status"], "RUNNING"),
                       meta["start_time"], meta.get("end_time"), meta["artifact_uri"], meta.get("run_name", ""))
        return Run(info, data)

    def metric_history(self, run_id: str, key: str) -> List[Dict[str, Any]]:
        p = os.path.join(self._run_dir(run_id), "metrics", self._safe_key(key))
        out = []
        if os.path.exists(p):
            with open(p) as f:
                for line in f:
                    ts, val, st = line.split()
                    out.append({"timestamp": int(ts), "value": float(val), "step": int(st)})
        return out

    def search_runs(self, experiment_ids: Sequence[str], order_by=None, max_results: int = 1000) -> List[Run]:
        runs = []
        for e in experiment_ids:
            d = os.path.join(self.root, self._check_exp_id(e))
            if not os.path.isdir(d):
                continue
            for r in os.listdir(d):
                if _RUN_ID_RE.fullmatch(r) and os.path.exists(os.path.join(d, r, "meta.yaml")):
                    run = self.get_run(r)
                    runs.append(run)
        return _sort_runs(runs, order_by)[:max_results]


# ----------------------------------------------------------------------------- REST store
class RestStore:
    def __init__(self, uri: str, timeout: float = 30.0, retries: int = 3):
        import requests

        self.base = uri.rstrip("/")
        self.timeout = timeout
        self.retries = retries
        self.s = requests.Session()
        tok = os.environ.get("MLFLOW_TRACKING_TOKEN")
        if tok:
            self.s.headers["Authorization"] = f"Bearer {tok}"

    def _call(self, method: str, endpoint: str, params=None, body=None):
        url = f"{self.base}/api/2.0/mlflow/{endpoint}"
        last = None
        for attempt in range(self.retries):
            try:
                r = self.s.request(method, url, params=params, json=body, timeout=self.timeout)
                if r.status_code == 404 and endpoint.startswith("experiments/get-by-name"):
                    return None
                if r.status_code >= 500:
                    last = RuntimeError(f"{method} {endpoint}: HTTP {r.status_code} {r.text[:200]}")
                    time.sleep(0.5 * (attempt + 1))
                    continue
                if r.status_code >= 400:
                    js = {}
                    try:
                        js = r.json()
                    except Exception:  # noqa: BLE001
                        pass
                    if js.get("error_code") == "RESOURCE_DOES_NOT_EXIST":
                        return None
                    raise RuntimeError(f"{method} {endpoint}: HTTP {r.status_code} {r.text[:300]}")
                return r.json() if r.content else {}
            except (ConnectionError, OSError) as e:  # requests.ConnectionError subclasses OSError
                last = e
                time.sleep(0.5 * (attempt + 1))
        raise RuntimeError(f"MLflow server unreachable at {self.base}: {last}")

    def get_experiment_by_name(self, name: str) -> Optional[Experiment]:
        js = self._call("GET", "experiments/get-by-name", params={"experiment_name": name})
        if not js or "experiment" not in js:
            return None
        e = js["experiment"]
        return Experiment(str(e["experiment_id"]), e["name"], e.get("artifact_location", ""),
                          e.get("lifecycle_stage", "active"))

    def create_experiment(self, name: str) -> str:
        return str(self._call("POST", "experiments/create", body={"name": name})["experiment_id"])

    @staticmethod
    def _run_from_json(js) -> Run:
        info = js["info"]
        data = js.get("data", {})
        metrics = {m["key"]: float(m["value"]) for m in data.get("metrics", [])}
        params = {p["key"]: p["value"] for p in data.get("params", [])}
        tags = {t["key"]: t["value"] for t in data.get("tags", [])}
        ri = RunInfo(info["run_id"], str(info["experiment_id"]), info.get("status", "RUNNING"),
                     int(info.get("start_time", 0)), info.get("end_time"), info.get("artifact_uri", ""),
                     info.get("run_name", ""))
        return Run(ri, RunData(metrics, params, tags))

    def create_run(self, experiment_id: str, run_name: str = "", tags: Optional[Dict[str, str]] = None) -> RunInfo:
        body = {"experiment_id": experiment_id, "start_time": _now_ms(), "run_name": run_name,
                "tags": [{"key": k, "value": str(v)} for k, v in (tags or {}).items()]}
        js = self._call("POST", "runs/create", body=body)
        return self._run_from_json(js["run"]).info

    def log_batch(self, run_id: str, metrics=(), params=(), tags=()):
        ts = _now_ms()
        body = {
            "run_id": run_id,
            "metrics": [{"key": m["key"], "value": float(m["value"]), "timestamp": int(m.get("timestamp") or ts),
                         "step": int(m.get("step", 0))} for m in metrics],
            "params": [{"key": p["key"], "value": str(p["value"])} for p in params],
            "tags": [{"key": t["key"], "value": str(t["value"])} for t in tags],
        }
        self._call("POST", "runs/log-batch", body=body)

    def log_metric(self, run_id: str, key: str, value: float, timestamp: Optional[int] = None, step: int = 0):
        self.log_batch(run_id, metrics=[{"key": key, "value": value, "timestamp": timestamp, "step": step}])

    def log_param(self, run_id: str, key: str, value: Any):
        self.log_batch(run_id, params=[{"key": key, "value": value}])

    def set_tag(self, run_id: str, key: str, value: Any):
        self.log_batch(run_id, tags=[{"key": key, "value": value}])

    def update_run(self, run_id: str, status: str, end_time: Optional[int] = None):
        self._call("POST", "runs/update", body={"run_id": run_id, "status": status, "end_time": end_time or _now_ms()})

    def get_run(self, run_id: str) -> Run:
        return self._run_from_json(self._call("GET", "runs/get", params={"run_id": run_id})["run"])

    def search_runs(self, experiment_ids: Sequence[str], order_by=None, max_results: int = 1000) -> List[Run]:
        body = {"experiment_ids": [str(e) for e in experiment_ids], "max_results": max_results,
                "order_by": list(order_by or [])}
        js = self._call("POST", "runs/search", body=body) or {}
        return [self._run_from_json(r) for r in js.get("runs", [])]

    # proxied artifacts (mlflow-artifacts:/...)
    def upload_artifact(self, rel_path: str, local_file: str):
        url = f"{self.base}/api/2.0/mlflow-artifacts/artifacts/{quote(rel_path)}"
        with open(local_file, "rb") as f:
            r = self.s.put(url, data=f, timeout=self.timeout * 10)
        if r.status_code >= 400:
            raise RuntimeError(f"artifact upload failed: HTTP {r.status_code} {r.text[:200]}")

    def list_artifacts_proxy(self, rel_path: str) -> List[Dict[str, Any]]:
        url = f"{self.base}/api/2.0/mlflow-artifacts/artifacts"
        r = self.s.get(url, params={"path": rel_path}, timeout=self.timeout)
        r.raise_for_status()
        return r.json().get("files", [])

    def download_artifact_proxy(self, rel_path: str, dst: str):
        url = f"{self.base}/api/2.0/mlflow-artifacts/artifacts/{quote(rel_path)}"
        r = self.s.get(url, timeout=self.timeout * 10, stream=True)
        r.raise_for_status()
        os.makedirs(os.path.dirname(dst), exist_ok=True)
        with open(dst, "wb") as f:
            for chunk in r.iter_content(1 << 20):
                f.write(chunk)


# ----------------------------------------------------------------------------- client
def _uri_to_path(uri: str) -> Optional[str]:
    if uri.startswith("file://"):
        return urlparse(uri).path
    if uri.startswith("file:"):
        return uri[5:]
    if "://" not in uri and not uri.startswith("mlflow-artifacts:"):
        return uri
    return None


class MlflowClient:
    def __init__(self, tracking_uri: Optional[str] = None):
        uri = tracking_uri or os.environ.get("MLFLOW_TRACKING_URI") or "./mlruns"
        self.tracking_uri = uri
        if uri.startswith("http://") or uri.startswith("https://"):
            self.store = RestStore(uri)
        else:
            self.store = FileStore(_uri_to_path(uri) or uri)

    @property
    def is_remote(self) -> bool:
        return isinstance(self.store, RestStore)

    def __getattr__(self, name):
        return getattr(self.store, name)

    def get_or_create_experiment(self, name: str) -> str:
        e = self.store.get_experiment_by_name(name)
        if e is not None:
            return e.experiment_id
        try:
            return self.store.create_experiment(name)
        except Exception:  # noqa: BLE001 - another rank/process created it concurrently
            e = self.store.get_experiment_by_name(name)
            if e is None:
                raise
            return e.experiment_id

    def set_terminated(self, run_id: str, status: str = "FINISHED"):
        self.store.update_run(run_id, status)

    # ------------------------------------------------------------------ artifacts
    def log_artifact(self, run_id: str, local_path: str, artifact_path: Optional[str] = None):
        run = self.store.get_run(run_id)
        base = run.info.artifact_uri
        name = os.path.basename(local_path)
        rel = os.path.join(artifact_path, name) if artifact_path else name
        local_root = _uri_to_path(base)
        if local_root is not None:
            dst = os.path.join(local_root, rel)
            os.makedirs(os.path.dirname(dst), exist_ok=True)
            if os.path.isdir(local_path):
                shutil.copytree(local_path, dst, dirs_exist_ok=True)
            else:
                shutil.copy2(local_path, dst)
            return dst
        if base.startswith("mlflow-artifacts:"):
            prefix = urlparse(base).path.lstrip("/")
            if os.path.isdir(local_path):
                for root, _, files in os.walk(local_path):
                    for fn in files:
                        p = os.path.join(root, fn)
                        self.store.upload_artifact(f"{prefix}/{rel}/{os.path.relpath(p, local_path)}", p)
            else:
                self.store.upload_artifact(f"{prefix}/{rel}", local_path)
            return f"{base}/{rel}"
        raise RuntimeError(f"unsupported artifact store {base!r}")

    def download_artifacts(self, run_id: str, path: str, dst_path: str) -> str:
        run = self.store.get_run(run_id)
        base = run.info.artifact_uri
        os.makedirs(dst_path, exist_ok=True)
        local_root = _uri_to_path(base)
        if local_root is not None:
            src = os.path.join(local_root, path)
            if not os.path.exists(src):
                raise FileNotFoundError(f"artifact {path!r} not found for run {run_id}")
            dst = os.path.join(dst_path, os.path.basename(path.rstrip("/")) or "artifacts")
            if os.path.isdir(src):
                shutil.copytree(src, dst, dirs_exist_ok=True)
            else:
                shutil.copy2(src, dst)
            return dst
        if base.startswith("mlflow-artifacts:"):
            prefix = urlparse(base).path.lstrip("/")
            dst = os.path.join(dst_path, os.path.basename(path.rstrip("/")))

            def walk(rel):
                for f in self.store.list_artifacts_proxy(f"{prefix}/{rel}"):
                    child = f"{rel}/{os.path.basename(f['path'])}"
                    if f.get("is_dir"):
                        walk(child)
                    else:
                        self.store.download_artifact_proxy(f"{prefix}/{child}",
                                                           os.path.join(dst_path, child))

            walk(path.rstrip("/"))
            return dst
        raise RuntimeError(f"unsupported artifact store {base!r}")
