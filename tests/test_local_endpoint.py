"""Local online endpoint (deploy/local_endpoint.py): the Azure serving contract without Azure (CPU)."""
import json
import os

import pytest
import requests
import torch

import dct_amd  # noqa: F401
from dct_amd.ckpt import build_checkpoint, save_checkpoint
from dct_amd.deploy.azure import AzureConfig, automated_rollout, force_deploy
from dct_amd.deploy.local_endpoint import (EndpointError, EndpointServer, LocalEndpoint, LocalMLClient,
                                          health_probe)
from dct_amd.deploy.package import write_conda_yaml, write_score_py
from dct_amd.models.mlp import WeatherClassifier

X = [[0.1, -0.2, 0.3, 0.0, 1.0], [1.0, 1.0, -1.0, 0.5, 0.0]]


def _package(d, seed, broken=False):
    """A prepare_package-style directory: model.ckpt (Lightning layout) + score.py + conda.yaml."""
    os.makedirs(d, exist_ok=True)
    torch.manual_seed(seed)
    model = WeatherClassifier(5)
    save_checkpoint(build_checkpoint(model.state_dict(), epoch=0, global_step=1, hyper_parameters={"input_dim": 5}),
                    os.path.join(d, "model.ckpt"))
    write_score_py(os.path.join(d, "score.py"))
    write_conda_yaml(os.path.join(d, "conda.yaml"))
    if broken:  # a deployment whose scoring fails at request time
        with open(os.path.join(d, "score.py"), "a") as f:
            f.write("\n\ndef run(raw_data):\n    return {'error': 'model exploded'}\n")
    model.eval()
    return model


def _probs(model, x):
    with torch.no_grad():
        return torch.softmax(model(torch.tensor(x)), dim=1)


def test_endpoint_routing_mirror_and_validation(tmp_path):
    m_blue = _package(str(tmp_path / "blue"), 0)
    m_green = _package(str(tmp_path / "green"), 1)
    ep = LocalEndpoint("ep", seed=3)
    ep.add_deployment("blue", str(tmp_path / "blue"))
    ep.add_deployment("green", str(tmp_path / "green"))
    with pytest.raises(EndpointError):
        ep.set_traffic({"blue": 60})  # must sum to 100
    with pytest.raises(EndpointError):
        ep.set_traffic({"blue": 100}, {"green": 60})  # mirror capped at 50 %
    with pytest.raises(EndpointError):
        ep.set_traffic({"blue": 100, "nope": 0}, {"nope": 10})  # unknown deployment
    with pytest.raises(EndpointError):
        ep.invoke(json.dumps({"data": X}))  # no live traffic yet
    ep.set_traffic({"blue": 100, "green": 0}, {"green": 20})  # shadow phase
    served = [ep.invoke(json.dumps({"data": X}))[0] for _ in range(200)]
    ep.drain()
    st = ep.state()["deployments"]
    assert set(served) == {"blue"}
    assert 10 <= st["green"]["mirrored"] <= 80 and st["green"]["requests"] == 0
    slot, out = ep.invoke(json.dumps({"data": X}), deployment="green")  # explicit routing header
    assert slot == "green" and torch.allclose(torch.tensor(out["probabilities"]), _probs(m_green, X), atol=1e-6)
    ep.set_traffic({"blue": 90, "green": 10})  # canary
    served = [ep.invoke(json.dumps({"data": X}))[0] for _ in range(400)]
    assert 10 <= served.count("green") <= 80
    _, out = ep.invoke(json.dumps({"data": X}), deployment="blue")
    assert torch.allclose(torch.tensor(out["probabilities"]), _probs(m_blue, X), atol=1e-6)
    with pytest.raises(EndpointError):
        ep.remove_deployment("green")  # still has traffic
    assert "error" in ep.invoke("{not json", deployment="blue")[1]  # score.py returns errors as data


def test_rollout_against_live_local_endpoint_in_process(tmp_path):
    _package(str(tmp_path / "v1"), 0)
    m2 = _package(str(tmp_path / "v2"), 1)
    client = LocalMLClient(seed=0)
    cfg = AzureConfig(endpoint_name="weather-api", deploy_dir=str(tmp_path / "v1"), wait_s=0)
    assert force_deploy(client, cfg) == "blue"
    assert client.online_endpoints.get("weather-api").traffic == {"blue": 100}
    cfg.deploy_dir = str(tmp_path / "v2")
    phases = []

    def traffic_during_phase(_s):  # requests arriving while the rollout waits in each phase
        for _ in range(100):
            client.invoke("weather-api", json.dumps({"data": X}))
        client.endpoints["weather-api"].drain()
        phases.append(client.online_endpoints.get("weather-api").traffic)

    r = automated_rollout(client, cfg, probe=health_probe(client, "weather-api"), sleep=traffic_during_phase)
    assert r == {"old_slot": "blue", "new_slot": "green", "status": "complete"}
    assert phases == [{"blue": 100, "green": 0}, {"blue": 90, "green": 10}]
    st = client.deployment_stats("weather-api", "green")
    assert st["mirrored"] > 0 and st["requests"] > 0 and st["errors"] == 0
    assert client.online_endpoints.get("weather-api").traffic == {"green": 100}
    assert [d.name for d in client.online_deployments.list("weather-api")] == ["green"]
    out = client.invoke("weather-api", json.dumps({"data": X}))
    assert torch.allclose(torch.tensor(out["probabilities"]), _probs(m2, X), atol=1e-6)


def test_rollout_health_gate_rolls_back_a_failing_slot(tmp_path):
    m1 = _package(str(tmp_path / "good"), 0)
    _package(str(tmp_path / "bad"), 1, broken=True)
    client = LocalMLClient()
    cfg = AzureConfig(endpoint_name="ep", deploy_dir=str(tmp_path / "good"), wait_s=0)
    force_deploy(client, cfg)
    cfg.deploy_dir = str(tmp_path / "bad")
    r = automated_rollout(client, cfg, probe=health_probe(client, "ep"), sleep=lambda s: None)
    assert r["status"] == "rolled_back_at_shadow"
    assert client.online_endpoints.get("ep").traffic == {"blue": 100}
    assert [d.name for d in client.online_deployments.list("ep")] == ["blue"]
    out = client.invoke("ep", json.dumps({"data": X}))
    assert torch.allclose(torch.tensor(out["probabilities"]), _probs(m1, X), atol=1e-6)


def test_http_server_admin_api_key_auth_and_remote_client(tmp_path):
    m1 = _package(str(tmp_path / "p1"), 0)
    m2 = _package(str(tmp_path / "p2"), 1)
    ep = LocalEndpoint("weather-api")
    srv = EndpointServer(ep, require_key=True, package_root=str(tmp_path)).start()
    try:
        assert requests.post(srv.url + "/score", json={"data": X}, timeout=30).status_code == 401
        client = LocalMLClient(base_url=srv.url, key=ep.key)
        cfg = AzureConfig(endpoint_name="weather-api", deploy_dir=str(tmp_path / "p1"), wait_s=0)
        force_deploy(client, cfg)
        hdr = {"Authorization": f"Bearer {ep.key}"}
        r = requests.post(srv.url + "/score", data=json.dumps({"data": X}), headers=hdr, timeout=30)
        assert r.status_code == 200 and r.headers["azureml-model-deployment"] == "blue"
        assert torch.allclose(torch.tensor(r.json()["probabilities"]), _probs(m1, X), atol=1e-6)
        cfg.deploy_dir = str(tmp_path / "p2")
        res = automated_rollout(client, cfg, probe=health_probe(client, "weather-api"), sleep=lambda s: None)
        assert res["status"] == "complete" and ep.traffic == {"green": 100}
        r = requests.post(srv.url + "/score", data=json.dumps({"data": X}), headers=hdr, timeout=30)
        assert r.headers["azureml-model-deployment"] == "green"
        assert torch.allclose(torch.tensor(r.json()["probabilities"]), _probs(m2, X), atol=1e-6)
        bad = requests.post(srv.url + "/score", data="{}", headers={**hdr, "azureml-model-deployment": "blue"},
                            timeout=30)
        assert bad.status_code == 404  # blue was deleted by the rollout
        state = requests.get(srv.url + "/", headers=hdr, timeout=30).json()
        assert list(state["deployments"]) == ["green"] and state["traffic"] == {"green": 100}
    finally:
        srv.stop()


def test_deploy_dags_against_a_local_endpoint_server(tmp_path, monkeypatch):
    """azure_manual_deploy then azure_automated_rollout (LocalDagRunner) with DCT_AZURE_BACKEND=local:
    MLflow best run -> package -> live local endpoint over its admin API, health-gated."""
    from dct_amd.orchestration import airflow_compat as af
    from dct_amd.orchestration import dags as dags_mod
    from dct_amd.orchestration.dags import build_manual_deploy_dag, build_rollout_dag
    from dct_amd.tracking import MlflowClient

    if af.HAVE_AIRFLOW:  # pragma: no cover
        pytest.skip("stand-in runner only")
    uri = "file://" + str(tmp_path / "mlruns")
    mc = MlflowClient(uri)
    run = mc.create_run(mc.get_or_create_experiment("weather_forecasting")).run_id
    model = _package(str(tmp_path / "trained"), 7)
    mc.log_batch(run, metrics=[{"key": "val_loss", "value": 0.3, "step": 1}])
    mc.log_artifact(run, str(tmp_path / "trained" / "model.ckpt"), "best_checkpoints")
    ep = LocalEndpoint("weather-api")
    srv = EndpointServer(ep, require_key=False, package_root=str(tmp_path)).start()
    try:
        for k, v in {"MLFLOW_TRACKING_URI": uri, "DCT_AZURE_BACKEND": "local", "DCT_LOCAL_ENDPOINT_URL": srv.url,
                     "DCT_LOCAL_ENDPOINT_KEY": ep.key,
                     "ENDPOINT_NAME": "weather-api", "DEPLOY_DIR": str(tmp_path / "deploy"),
                     "DCT_ROLLOUT_WAIT_S": "0"}.items():
            monkeypatch.setenv(k, v)
        monkeypatch.setattr(dags_mod, "_FAKE_CLIENT", None)
        runner = af.LocalDagRunner(sleep=lambda s: None)
        assert runner.run(build_manual_deploy_dag()).state == "success"
        assert ep.traffic == {"blue": 100}
        res = runner.run(build_rollout_dag())
        assert res.state == "success", res.errors
        assert ep.traffic == {"green": 100} and list(ep.deployments) == ["green"]
        r = requests.post(srv.url + "/score", data=json.dumps({"data": X}), timeout=30)
        assert torch.allclose(torch.tensor(r.json()["probabilities"]), _probs(model, X), atol=1e-6)
    finally:
        srv.stop()


def test_admin_api_always_needs_the_key_and_stays_inside_the_package_root(tmp_path):
    """The admin API loads and runs a package's score.py: it must need the endpoint key even when
    scoring is open, and must refuse packages outside the server's package root."""
    _package(str(tmp_path / "root" / "p1"), 0)
    _package(str(tmp_path / "outside"), 1)
    ep = LocalEndpoint("weather-api")
    srv = EndpointServer(ep, require_key=False, package_root=str(tmp_path / "root")).start()
    try:
        body = {"package_dir": str(tmp_path / "root" / "p1")}
        assert requests.put(srv.url + "/deployments/blue", json=body, timeout=30).status_code == 401
        bad = {"Authorization": "Bearer " + "0" * 32}
        assert requests.put(srv.url + "/deployments/blue", json=body, headers=bad, timeout=30).status_code == 401
        assert requests.delete(srv.url + "/deployments/blue", timeout=30).status_code == 401
        assert requests.put(srv.url + "/traffic", json={"traffic": {}}, timeout=30).status_code == 401
        hdr = {"Authorization": f"Bearer {ep.key}"}
        for pkg in (str(tmp_path / "outside"), str(tmp_path / "root" / ".." / "outside")):
            r = requests.put(srv.url + "/deployments/green", json={"package_dir": pkg}, headers=hdr, timeout=30)
            assert r.status_code == 403 and "green" not in ep.deployments
        os.symlink(str(tmp_path / "outside"), str(tmp_path / "root" / "link"))
        r = requests.put(srv.url + "/deployments/green", json={"package_dir": str(tmp_path / "root" / "link")},
                         headers=hdr, timeout=30)
        assert r.status_code == 403
        r = requests.put(srv.url + "/deployments/blue", json={**body, "scoring_script": "../x.py"}, headers=hdr,
                         timeout=30)
        assert r.status_code == 400
        assert requests.put(srv.url + "/deployments/blue", json=body, headers=hdr, timeout=30).status_code == 200
        assert requests.put(srv.url + "/traffic", json={"traffic": {"blue": 100}}, headers=hdr,
                            timeout=30).status_code == 200
        # scoring is open on this server (require_key=False)
        assert requests.post(srv.url + "/score", json={"data": X}, timeout=30).status_code == 200
    finally:
        srv.stop()
    closed = EndpointServer(LocalEndpoint("x")).start()  # no package root: admin deployments refused
    try:
        hdr = {"Authorization": f"Bearer {closed.endpoint.key}"}
        r = requests.put(closed.url + "/deployments/blue", json={"package_dir": str(tmp_path / "outside")},
                         headers=hdr, timeout=30)
        assert r.status_code == 403
    finally:
        closed.stop()
