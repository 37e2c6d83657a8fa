"""Minimal MLflow-compatible tracking server (stdlib only).

The reference runs ``mlflow server --backend-store-uri postgresql://... --default-artifact-root
/mlflow/artifacts`` as a compose service (docker-compose.yml:170-188).  ``mlflow`` is not
installable offline, so this module serves the subset of the MLflow 2.x REST API that the
pipeline uses (experiments get-by-name/create, runs create/get/update/search/log-batch,
metrics get-history, and the ``mlflow-artifacts`` proxy) on top of :class:`FileStore`, whose
on-disk layout a stock ``mlflow ui`` can read.  It is used by the tests and can stand in for the
real server on an air-gapped node:

    python -m dct_amd.tracking.server --port 5000 --root ./mlruns [--serve-artifacts]
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Optional
from urllib.parse import parse_qs, unquote, urlparse

from .mlflow_client import FileStore, RUN_STATUS, _sort_runs


def _run_json(run):
    i, d = run.info, run.data
    return {
        "info": {"run_id": i.run_id, "run_uuid": i.run_id, "experiment_id": i.experiment_id, "status": i.status,
                 "start_time": i.start_time, "end_time": i.end_time, "artifact_uri": i.artifact_uri,
                 "run_name": i.run_name, "lifecycle_stage": "active"},
        "data": {"metrics": [{"key": k, "value": v, "timestamp": 0, "step": 0} for k, v in d.metrics.items()],
                 "params": [{"key": k, "value": v} for k, v in d.params.items()],
                 "tags": [{"key": k, "value": v} for k, v in d.tags.items()]},
    }


class _State:
    def __init__(self, root: str, serve_artifacts: bool, artifacts_root: Optional[str]):
        self.store = FileStore(root)
        self.serve_artifacts = serve_artifacts
        self.artifacts_root = os.path.abspath(artifacts_root or os.path.join(root, "mlartifacts"))
        self.lock = threading.Lock()


def make_handler(state: _State):
    class H(BaseHTTPRequestHandler):
        def log_message(self, *a):  # quiet
            pass

        def _send(self, code, obj=None, raw: Optional[bytes] = None):
            body = raw if raw is not None else json.dumps(obj or {}).encode()
            self.send_response(code)
            self.send_header("Content-Type", "application/octet-stream" if raw is not None else "application/json")
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def _err(self, code, ec, msg):
            self._send(code, {"error_code": ec, "message": msg})

        def _body(self):
            n = int(self.headers.get("Content-Length") or 0)
            return json.loads(self.rfile.read(n) or b"{}") if n else {}

        def _art_path(self, rel):
            root = state.artifacts_root
            p = os.path.abspath(os.path.join(root, unquote(rel)))
            # component-wise containment: a plain prefix test lets "../mlartifacts_x/f" through
            if os.path.commonpath([root, p]) != root:
                raise PermissionError(rel)
            return p

        # ---------------------------------------------------------------- GET
        def do_GET(self):
            u = urlparse(self.path)
            q = {k: v[0] for k, v in parse_qs(u.query).items()}
            st = state.store
            try:
                if u.path == "/health":
                    return self._send(200, {"status": "OK"})
                if u.path == "/api/2.0/mlflow/experiments/get-by-name":
                    e = st.get_experiment_by_name(q.get("experiment_name", ""))
                    if e is None:
                        return self._err(404, "RESOURCE_DOES_NOT_EXIST", "experiment not found")
                    return self._send(200, {"experiment": {"experiment_id": e.experiment_id, "name": e.name,
                                                           "artifact_location": e.artifact_location,
                                                           "lifecycle_stage": e.lifecycle_stage}})
                if u.path == "/api/2.0/mlflow/runs/get":
                    return self._send(200, {"run": _run_json(st.get_run(q["run_id"]))})
                if u.path == "/api/2.0/mlflow/metrics/get-history":
                    return self._send(200, {"metrics": [dict(key=q["metric_key"], **m) for m in
                                                        st.metric_history(q["run_id"], q["metric_key"])]})
                if u.path == "/api/2.0/mlflow-artifacts/artifacts":
                    base = self._art_path(q.get("path", ""))
                    files = []
                    if os.path.isdir(base):
                        for f in sorted(os.listdir(base)):
                            fp = os.path.join(base, f)
                            files.append({"path": f, "is_dir": os.path.isdir(fp),
                                          **({} if os.path.isdir(fp) else {"file_size": os.path.getsize(fp)})})
                    return self._send(200, {"files": files})
                if u.path.startswith("/api/2.0/mlflow-artifacts/artifacts/"):
                    p = self._art_path(u.path[len("/api/2.0/mlflow-artifacts/artifacts/"):])
                    if not os.path.isfile(p):
                        return self._err(404, "RESOURCE_DOES_NOT_EXIST", "artifact not found")
                    with open(p, "rb") as f:
                        return self._send(200, raw=f.read())
                return self._err(404, "ENDPOINT_NOT_FOUND", u.path)
            except KeyError as e:
                return self._err(404, "RESOURCE_DOES_NOT_EXIST", str(e))
            except PermissionError as e:
                return self._err(403, "PERMISSION_DENIED", f"path outside the artifact root: {e}")
            except ValueError as e:
                return self._err(400, "INVALID_PARAMETER_VALUE", str(e))
            except Exception as e:  # noqa: BLE001
                return self._err(500, "INTERNAL_ERROR", repr(e))

        # ---------------------------------------------------------------- POST
        def do_POST(self):
            u = urlparse(self.path)
            st = state.store
            try:
                b = self._body()
                with state.lock:
                    if u.path == "/api/2.0/mlflow/experiments/create":
                        if st.get_experiment_by_name(b["name"]) is not None:
                            return self._err(400, "RESOURCE_ALREADY_EXISTS", "experiment exists")
                        return self._send(200, {"experiment_id": st.create_experiment(b["name"])})
                    if u.path == "/api/2.0/mlflow/runs/create":
                        tags = {t["key"]: t["value"] for t in b.get("tags", [])}
                        info = st.create_run(str(b["experiment_id"]), b.get("run_name", ""), tags)
                        if state.serve_artifacts:
                            art = f"mlflow-artifacts:/{info.experiment_id}/{info.run_id}/artifacts"
                            d = st._run_dir(info.run_id)
                            meta = st._load_yaml(os.path.join(d, "meta.yaml"))
                            meta["artifact_uri"] = art
                            st._dump_yaml(os.path.join(d, "meta.yaml"), meta)
                        return self._send(200, {"run": _run_json(st.get_run(info.run_id))})
                    if u.path == "/api/2.0/mlflow/runs/log-batch":
                        st.log_batch(b["run_id"], b.get("metrics", []), b.get("params", []), b.get("tags", []))
                        return self._send(200, {})
                    if u.path == "/api/2.0/mlflow/runs/update":
                        st.update_run(b["run_id"], b.get("status", "FINISHED"), b.get("end_time"))
                        return self._send(200, {"run_info": _run_json(st.get_run(b["run_id"]))["info"]})
                    if u.path == "/api/2.0/mlflow/runs/search":
                        runs = st.search_runs([str(e) for e in b.get("experiment_ids", [])],
                                              b.get("order_by") or None, int(b.get("max_results", 1000)))
                        return self._send(200, {"runs": [_run_json(r) for r in runs]})
                return self._err(404, "ENDPOINT_NOT_FOUND", u.path)
            except KeyError as e:
                return self._err(404, "RESOURCE_DOES_NOT_EXIST", str(e))
            except PermissionError as e:
                return self._err(403, "PERMISSION_DENIED", f"path outside the artifact root: {e}")
            except ValueError as e:
                return self._err(400, "INVALID_PARAMETER_VALUE", str(e))
            except Exception as e:  # noqa: BLE001
                return self._err(500, "INTERNAL_ERROR", repr(e))

        def do_PUT(self):
            u = urlparse(self.path)
            if not u.path.startswith("/api/2.0/mlflow-artifacts/artifacts/"):
                return self._err(404, "ENDPOINT_NOT_FOUND", u.path)
            try:
                p = self._art_path(u.path[len("/api/2.0/mlflow-artifacts/artifacts/"):])
                n = int(self.headers.get("Content-Length") or 0)
                os.makedirs(os.path.dirname(p), exist_ok=True)
                with open(p + ".part", "wb") as f:
                    remaining = n
                    while remaining > 0:
                        chunk = self.rfile.read(min(remaining, 1 << 20))
                        if not chunk:
                            break
                        f.write(chunk)
                        remaining -= len(chunk)
                os.replace(p + ".part", p)
                return self._send(200, {})
            except PermissionError as e:
                return self._err(403, "PERMISSION_DENIED", f"path outside the artifact root: {e}")
            except Exception as e:  # noqa: BLE001
                return self._err(500, "INTERNAL_ERROR", repr(e))

    return H


class TrackingServer:
    def __init__(self, root: str, host: str = "127.0.0.1", port: int = 0, serve_artifacts: bool = False,
                 artifacts_root: Optional[str] = None):
        self.state = _State(root, serve_artifacts, artifacts_root)
        self.httpd = ThreadingHTTPServer((host, port), make_handler(self.state))
        self.thread: Optional[threading.Thread] = None

    @property
    def url(self) -> str:
        h, p = self.httpd.server_address[:2]
        return f"http://{h}:{p}"

    def start(self) -> "TrackingServer":
        self.thread = threading.Thread(target=self.httpd.serve_forever, daemon=True)
        self.thread.start()
        return self

    def stop(self):
        self.httpd.shutdown()
        self.httpd.server_close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=5000)
    ap.add_argument("--root", default="./mlruns")
    ap.add_argument("--serve-artifacts", action="store_true")
    ap.add_argument("--artifacts-destination", default=None)
    a = ap.parse_args()
    srv = TrackingServer(a.root, a.host, a.port, a.serve_artifacts, a.artifacts_destination)
    print(f"tracking server on {srv.url} (store {os.path.abspath(a.root)})", flush=True)
    srv.httpd.serve_forever()


if __name__ == "__main__":
    main()
