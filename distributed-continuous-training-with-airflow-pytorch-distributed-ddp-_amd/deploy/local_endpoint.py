"""Local managed online endpoint: the Azure ML serving contract on this node.

The reference serves only through Azure ML managed online endpoints: a forced deployment
(dags/azure_manual_deploy.py:137-167) or a blue/green rollout with a 20 % shadow mirror and a 10 %
canary (dags/azure_auto_deploy.py:118-185), each deployment running the generated ``score.py``
(azure_manual_deploy.py:55-124).  This module serves the same contract locally - on the GPU node
next to the trainer, in CI, or anywhere without an Azure subscription:

* a **deployment** is a package directory written by :func:`deploy.package.prepare_package`
  (``model.ckpt``, ``score.py``, ``conda.yaml``).  It is loaded the way the Azure inference server
  loads it: ``score.py`` imported in a module namespace of its own with ``AZUREML_MODEL_DIR``
  pointing at the package, ``init()`` once, ``run(raw)`` per request;
* an **endpoint** sends each request to one deployment drawn by the ``traffic`` weights (or to the
  one named by the ``azureml-model-deployment`` header, as Azure does) and copies
  ``mirror_traffic[slot]`` percent of the requests to that slot in the background (shadow: the
  response is discarded; requests, errors and latency are counted);
* :class:`EndpointServer` serves an endpoint over HTTP - ``POST /score``, ``GET /`` (state and
  per-deployment statistics) - plus an admin API (``PUT /deployments/<name>``, ``DELETE
  /deployments/<name>``, ``PUT /traffic``).  The admin API ALWAYS needs the endpoint key (the
  Azure control plane it imitates is authenticated) and only loads packages that resolve inside
  the server's ``package_root``; the scoring routes need the key too unless the server is started
  with ``require_key=False`` (``--no-require-key``);
* :class:`LocalMLClient` is the subset of ``azure.ai.ml.MLClient`` that :mod:`deploy.azure` drives
  (``online_endpoints`` / ``online_deployments``), backed by in-process endpoints or by a running
  server's admin API, so ``force_deploy`` and ``automated_rollout`` run unchanged against a live
  local endpoint; :func:`health_probe` is the rollout's health gate (reference D11 had none).

    python -m dct_amd.deploy.local_endpoint --name weather-api --port 5001 --package $DEPLOY_DIR
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hmac
import importlib.util
import json
import os
import random
import threading
import time
import uuid
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from types import SimpleNamespace
from typing import Any, Callable, Dict, List, Optional, Tuple

_ENV_LOCK = threading.Lock()
MIRROR_MAX_PCT = 50  # Azure caps mirrored traffic at 50 %


class EndpointError(Exception):
    def __init__(self, status: int, message: str):
        super().__init__(message)
        self.status = status


class Deployment:
    """One loaded scoring package (score.py + model files)."""

    def __init__(self, name: str, package_dir: str, scoring_script: str = "score.py"):
        self.name = name
        self.package_dir = os.path.abspath(package_dir)
        self.scoring_script = scoring_script
        self.stats = {"requests": 0, "mirrored": 0, "errors": 0, "latency_s": 0.0}
        self._lock = threading.Lock()
        self.module = self._load()

    def _load(self):
        path = os.path.join(self.package_dir, self.scoring_script)
        if not os.path.isfile(path):
            raise EndpointError(400, f"scoring script {path} not found")
        spec = importlib.util.spec_from_file_location(f"_dct_score_{self.name}_{uuid.uuid4().hex[:8]}", path)
        mod = importlib.util.module_from_spec(spec)
        with _ENV_LOCK:  # init() resolves the model under AZUREML_MODEL_DIR, as on Azure
            prev = os.environ.get("AZUREML_MODEL_DIR")
            os.environ["AZUREML_MODEL_DIR"] = self.package_dir
            try:
                spec.loader.exec_module(mod)
                mod.init()
            finally:
                if prev is None:
                    os.environ.pop("AZUREML_MODEL_DIR", None)
                else:
                    os.environ["AZUREML_MODEL_DIR"] = prev
        return mod

    def score(self, raw: Any, mirrored: bool = False) -> Any:
        t0 = time.perf_counter()
        with self._lock:  # score.py keeps its model in module globals: one request at a time
            out = self.module.run(raw)
            s = self.stats
            s["mirrored" if mirrored else "requests"] += 1
            s["latency_s"] += time.perf_counter() - t0
            if isinstance(out, dict) and "error" in out:
                s["errors"] += 1
        return out

    def snapshot(self) -> Dict[str, Any]:
        with self._lock:
            return dict(self.stats, package_dir=self.package_dir, scoring_script=self.scoring_script)


class LocalEndpoint:
    """Deployments + traffic / mirror maps with Azure's routing semantics."""

    def __init__(self, name: str, auth_mode: str = "key", seed: int = 0, key: Optional[str] = None):
        self.name = name
        self.auth_mode = auth_mode
        # the key guards the admin API whatever the scoring auth mode is
        self.key = key or uuid.uuid4().hex
        self.deployments: Dict[str, Deployment] = {}
        self.traffic: Dict[str, int] = {}
        self.mirror_traffic: Dict[str, int] = {}
        self._rng = random.Random(seed)
        self._lock = threading.RLock()
        self._mirror_pool = cf.ThreadPoolExecutor(max_workers=2, thread_name_prefix=f"mirror-{name}")
        self._pending: List[cf.Future] = []

    # ------------------------------------------------------------------ control plane
    def add_deployment(self, name: str, package_dir: str, scoring_script: str = "score.py") -> Deployment:
        dep = Deployment(name, package_dir, scoring_script)  # init() outside the routing lock
        with self._lock:
            self.deployments[name] = dep
        return dep

    def remove_deployment(self, name: str):
        with self._lock:
            if self.traffic.get(name, 0) or self.mirror_traffic.get(name, 0):
                raise EndpointError(409, f"deployment {name!r} still receives traffic")
            self.deployments.pop(name, None)

    def set_traffic(self, traffic: Optional[Dict[str, Any]], mirror: Optional[Dict[str, Any]] = None):
        t = {k: int(v) for k, v in (traffic or {}).items()}
        m = {k: int(v) for k, v in (mirror or {}).items()}
        with self._lock:
            for slot, pct in list(t.items()) + list(m.items()):
                if pct < 0 or pct > 100:
                    raise EndpointError(400, f"traffic for {slot!r} must be within 0..100")
                if pct and slot not in self.deployments:
                    raise EndpointError(400, f"traffic to unknown deployment {slot!r}")
            if sum(t.values()) not in (0, 100):
                raise EndpointError(400, "live traffic must sum to 0 or 100")
            for slot, pct in m.items():
                if pct > MIRROR_MAX_PCT:
                    raise EndpointError(400, f"mirror traffic is capped at {MIRROR_MAX_PCT} %")
                if pct and t.get(slot, 0):
                    raise EndpointError(400, f"{slot!r} cannot receive live and mirrored traffic")
            self.traffic, self.mirror_traffic = t, m

    # ------------------------------------------------------------------ data plane
    def _pick(self) -> str:
        live = [(s, p) for s, p in sorted(self.traffic.items()) if p > 0]
        if not live:
            raise EndpointError(503, f"endpoint {self.name!r} has no live traffic")
        r = self._rng.uniform(0, 100)
        acc = 0.0
        for slot, pct in live:
            acc += pct
            if r < acc:
                return slot
        return live[-1][0]

    def invoke(self, raw: Any, deployment: Optional[str] = None) -> Tuple[str, Any]:
        """Route one request; returns (serving deployment, response)."""
        with self._lock:
            if deployment:
                if deployment not in self.deployments:
                    raise EndpointError(404, f"deployment {deployment!r} not found")
                target, shadows = deployment, []
            else:
                target = self._pick()
                shadows = [self.deployments[s] for s, p in sorted(self.mirror_traffic.items())
                           if p and s != target and s in self.deployments and self._rng.uniform(0, 100) < p]
            dep = self.deployments[target]
        out = dep.score(raw)
        for sh in shadows:
            self._pending.append(self._mirror_pool.submit(sh.score, raw, True))
        return target, out

    def drain(self, timeout: float = 30.0):
        """Wait for the mirrored requests issued so far (tests, graceful shutdown)."""
        pending, self._pending = self._pending, []
        cf.wait(pending, timeout=timeout)

    def state(self) -> Dict[str, Any]:
        with self._lock:
            return {"name": self.name, "auth_mode": self.auth_mode, "traffic": dict(self.traffic),
                    "mirror_traffic": dict(self.mirror_traffic),
                    "deployments": {n: d.snapshot() for n, d in self.deployments.items()}}


# ----------------------------------------------------------------------------- HTTP server
def _make_handler(srv: "EndpointServer"):
    ep = srv.endpoint

    class H(BaseHTTPRequestHandler):
        def log_message(self, *a):  # quiet
            pass

        def _send(self, code: int, obj: Any, headers: Optional[Dict[str, str]] = None):
            body = json.dumps(obj).encode()
            self.send_response(code)
            self.send_header("Content-Type", "application/json")
            self.send_header("Content-Length", str(len(body)))
            for k, v in (headers or {}).items():
                self.send_header(k, v)
            self.end_headers()
            self.wfile.write(body)

        def _body(self) -> bytes:
            n = int(self.headers.get("Content-Length") or 0)
            return self.rfile.read(n) if n else b""

        def _authorized(self, admin: bool = False) -> bool:
            if not admin and not (srv.require_key and ep.auth_mode == "key"):
                return True
            given = self.headers.get("Authorization", "").encode()
            if hmac.compare_digest(given, f"Bearer {ep.key}".encode()):
                return True
            self._send(401, {"error": "missing or invalid endpoint key"})
            return False

        def _run(self, fn: Callable[[], Tuple[int, Any, Optional[Dict[str, str]]]]):
            try:
                code, obj, hdr = fn()
                self._send(code, obj, hdr)
            except EndpointError as e:
                self._send(e.status, {"error": str(e)})
            except Exception as e:  # noqa: BLE001 - the endpoint must answer, not die
                self._send(500, {"error": repr(e)})

        def do_GET(self):
            if self.path.rstrip("/") in ("", "/health"):
                if not self._authorized():
                    return
                self._run(lambda: (200, ep.state(), None))
            else:
                self._send(404, {"error": f"no route {self.path}"})

        def do_POST(self):
            if self.path.rstrip("/") != "/score":
                return self._send(404, {"error": f"no route {self.path}"})
            if not self._authorized():
                return
            raw = self._body().decode("utf-8", errors="replace")
            want = self.headers.get("azureml-model-deployment") or None

            def go():
                slot, out = ep.invoke(raw, want)
                return 200, out, {"azureml-model-deployment": slot}
            self._run(go)

        def do_PUT(self):
            if not self._authorized(admin=True):
                return
            path = self.path.rstrip("/")
            try:
                body = json.loads(self._body() or b"{}")
            except ValueError:
                return self._send(400, {"error": "body is not JSON"})
            if path.startswith("/deployments/"):
                name = path[len("/deployments/"):]
                return self._run(lambda: (200, ep.add_deployment(name, srv.resolve_package(body["package_dir"]),
                                                                 _script_name(body.get("scoring_script"))).snapshot(),
                                          None))
            if path == "/traffic":
                def go():
                    ep.set_traffic(body.get("traffic"), body.get("mirror_traffic"))
                    return 200, ep.state(), None
                return self._run(go)
            self._send(404, {"error": f"no route {self.path}"})

        def do_DELETE(self):
            if not self._authorized(admin=True):
                return
            path = self.path.rstrip("/")
            if path.startswith("/deployments/"):
                name = path[len("/deployments/"):]

                def go():
                    ep.remove_deployment(name)
                    return 200, ep.state(), None
                return self._run(go)
            self._send(404, {"error": f"no route {self.path}"})

    return H


def _script_name(name: Optional[str]) -> str:
    """The scoring script is a file name inside the package, never a path."""
    name = name or "score.py"
    if os.path.basename(name) != name or not name.endswith(".py") or name.startswith("."):
        raise EndpointError(400, f"invalid scoring script name {name!r}")
    return name


class EndpointServer:
    """HTTP face of a :class:`LocalEndpoint`.

    ``package_root``: the directory admin-API deployments must resolve into (symlinks followed);
    ``None`` refuses every admin-API deployment.  ``require_key``: scoring routes need the key as
    well (admin routes always do)."""

    def __init__(self, endpoint: LocalEndpoint, host: str = "127.0.0.1", port: int = 0, require_key: bool = True,
                 package_root: Optional[str] = None):
        self.endpoint = endpoint
        self.require_key = require_key
        self.package_root = os.path.realpath(package_root) if package_root else None
        self.httpd = ThreadingHTTPServer((host, port), _make_handler(self))
        self.thread: Optional[threading.Thread] = None

    def resolve_package(self, package_dir: str) -> str:
        if self.package_root is None:
            raise EndpointError(403, "this endpoint server accepts no packages over the admin API (no package root)")
        p = os.path.realpath(package_dir)
        if os.path.commonpath([self.package_root, p]) != self.package_root:
            raise EndpointError(403, f"package {package_dir!r} is outside the server's package root")
        return p

    @property
    def url(self) -> str:
        h, p = self.httpd.server_address[:2]
        return f"http://{h}:{p}"

    def start(self) -> "EndpointServer":
        self.thread = threading.Thread(target=self.httpd.serve_forever, daemon=True)
        self.thread.start()
        return self

    def stop(self):
        self.httpd.shutdown()
        self.httpd.server_close()
        self.endpoint.drain()


# ----------------------------------------------------------------------------- MLClient subset
class _Done:
    def __init__(self, value=None):
        self._v = value

    def result(self):
        return self._v

    def wait(self):
        return self._v


class _RemoteEndpoint:
    """Admin-API view of one running EndpointServer (same methods as LocalEndpoint's control plane)."""

    def __init__(self, base_url: str, key: Optional[str] = None):
        import requests

        self.base = base_url.rstrip("/")
        self.s = requests.Session()
        if key:
            self.s.headers["Authorization"] = f"Bearer {key}"
        self.name = self.state()["name"]

    def _call(self, method: str, path: str, body=None, headers=None):
        r = self.s.request(method, self.base + path, json=body, headers=headers, timeout=600)
        try:
            js = r.json()
        except ValueError:
            js = {"error": r.text}
        if r.status_code >= 400:
            raise EndpointError(r.status_code, js.get("error", r.text) if isinstance(js, dict) else r.text)
        return r, js

    def state(self):
        return self._call("GET", "/")[1]

    def add_deployment(self, name, package_dir, scoring_script="score.py"):
        return self._call("PUT", f"/deployments/{name}", {"package_dir": os.path.abspath(package_dir),
                                                          "scoring_script": scoring_script})[1]

    def remove_deployment(self, name):
        self._call("DELETE", f"/deployments/{name}")

    def set_traffic(self, traffic, mirror=None):
        self._call("PUT", "/traffic", {"traffic": traffic or {}, "mirror_traffic": mirror or {}})

    def invoke(self, raw, deployment=None):
        hdr = {"azureml-model-deployment": deployment} if deployment else None
        r, js = self._call("POST", "/score", json.loads(raw) if isinstance(raw, str) else raw, hdr)
        return r.headers.get("azureml-model-deployment", ""), js


class LocalMLClient:
    """``azure.ai.ml.MLClient`` subset (``online_endpoints`` / ``online_deployments``) over local
    endpoints: in-process by default, or the admin API of a running :class:`EndpointServer`."""

    def __init__(self, base_url: Optional[str] = None, key: Optional[str] = None, seed: int = 0):
        self.seed = seed
        self.endpoints: Dict[str, Any] = {}
        if base_url:
            remote = _RemoteEndpoint(base_url, key)
            self.endpoints[remote.name] = remote
        self.online_endpoints = _Endpoints(self)
        self.online_deployments = _Deployments(self)

    def _endpoint(self, name: str):
        if name not in self.endpoints:
            raise KeyError(f"endpoint {name!r} not found")
        return self.endpoints[name]

    def invoke(self, endpoint_name: str, raw: Any, deployment: Optional[str] = None) -> Any:
        return self._endpoint(endpoint_name).invoke(raw, deployment)[1]

    def deployment_stats(self, endpoint_name: str, deployment: str) -> Dict[str, Any]:
        return self._endpoint(endpoint_name).state()["deployments"].get(deployment, {})


class _Endpoints:
    def __init__(self, client: LocalMLClient):
        self.c = client

    def get(self, name: str):
        st = self.c._endpoint(name).state()
        return SimpleNamespace(name=st["name"], auth_mode=st.get("auth_mode", "key"), traffic=dict(st["traffic"]),
                               mirror_traffic=dict(st["mirror_traffic"]), provisioning_state="Succeeded")

    def begin_create_or_update(self, endpoint):
        name = endpoint.name
        if name not in self.c.endpoints:
            self.c.endpoints[name] = LocalEndpoint(name, getattr(endpoint, "auth_mode", "key") or "key", self.c.seed)
        self.c.endpoints[name].set_traffic(getattr(endpoint, "traffic", None) or {},
                                           getattr(endpoint, "mirror_traffic", None) or {})
        return _Done(endpoint)

    def begin_delete(self, name: str):
        self.c.endpoints.pop(name, None)
        return _Done()


class _Deployments:
    def __init__(self, client: LocalMLClient):
        self.c = client

    def begin_create_or_update(self, d):
        ep = self.c._endpoint(d.endpoint_name)
        cc = getattr(d, "code_configuration", None)
        package = getattr(cc, "code", None) or getattr(getattr(d, "model", None), "path", None)
        if not package:
            raise EndpointError(400, f"deployment {d.name!r} has no package directory")
        ep.add_deployment(d.name, package, getattr(cc, "scoring_script", None) or "score.py")
        return _Done(d)

    def begin_delete(self, name: str, endpoint_name: str):
        self.c._endpoint(endpoint_name).remove_deployment(name)
        return _Done()

    def list(self, endpoint_name: str):
        return [SimpleNamespace(name=n, **v) for n, v in self.c._endpoint(endpoint_name).state()["deployments"].items()]


def health_probe(client: LocalMLClient, endpoint_name: str, sample: Optional[List[List[float]]] = None,
                 max_error_rate: float = 0.0) -> Callable[[str], bool]:
    """Rollout gate: the slot answers a sample request with probability rows summing to 1 and its
    error rate over the live / mirrored traffic it has served stays within ``max_error_rate``."""
    payload = json.dumps({"data": sample or [[0.0] * 5]})

    def probe(slot: str) -> bool:
        try:
            out = client.invoke(endpoint_name, payload, deployment=slot)
        except Exception:  # noqa: BLE001
            return False
        probs = out.get("probabilities") if isinstance(out, dict) else None
        if not probs or any(abs(sum(r) - 1.0) > 1e-3 for r in probs):
            return False
        st = client.deployment_stats(endpoint_name, slot)
        served = st.get("requests", 0) + st.get("mirrored", 0)
        return served == 0 or st.get("errors", 0) / served <= max_error_rate
    return probe


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="serve a scoring package with the Azure ML online-endpoint contract")
    ap.add_argument("--name", default=os.environ.get("ENDPOINT_NAME", "weather-api"))
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=5001)
    ap.add_argument("--package", default=os.environ.get("DEPLOY_DIR"), help="initial deployment (100 %% traffic)")
    ap.add_argument("--deployment", default=os.environ.get("DEPLOYMENT_NAME", "blue"))
    ap.add_argument("--no-require-key", dest="require_key", action="store_false",
                    help="serve /score and GET / without the key (the admin API always needs it)")
    ap.add_argument("--package-root", default=os.environ.get("DCT_PACKAGE_ROOT"),
                    help="admin-API deployments must resolve inside this directory "
                         "(default: DCT_PACKAGE_ROOT, else the parent of --package)")
    a = ap.parse_args(argv)
    # a shared key lets the deploy DAGs (DCT_LOCAL_ENDPOINT_KEY) drive the admin API
    ep = LocalEndpoint(a.name, key=os.environ.get("DCT_LOCAL_ENDPOINT_KEY") or None)
    if a.package:
        ep.add_deployment(a.deployment, a.package)
        ep.set_traffic({a.deployment: 100})
    root = a.package_root or (os.path.dirname(os.path.abspath(a.package)) if a.package else None)
    srv = EndpointServer(ep, a.host, a.port, a.require_key, package_root=root)
    shown = ep.key if not os.environ.get("DCT_LOCAL_ENDPOINT_KEY") else "from DCT_LOCAL_ENDPOINT_KEY"
    print(f"endpoint {a.name} on {srv.url} (key {shown}; package root {root})", flush=True)
    try:
        srv.httpd.serve_forever()
    except KeyboardInterrupt:
        pass
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
