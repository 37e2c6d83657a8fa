"""Lightning-compatible checkpoints, ModelCheckpoint semantics, MLflow client/server (CPU)."""
import os

import pytest
import torch

import dct_amd  # noqa: F401
from dct_amd.ckpt import CHECKPOINT_KEYS, ModelCheckpoint, build_checkpoint, load_checkpoint, save_checkpoint
from dct_amd.models.mlp import MLPClassifier, WeatherClassifier
from dct_amd.ops.optim import FlatAdam, adam_flat_
from dct_amd.tracking import MlflowClient, MLFlowLogger
from dct_amd.tracking.server import TrackingServer

REFERENCE_KEYS = {"net.0.weight", "net.0.bias", "net.3.weight", "net.3.bias"}


def test_weather_classifier_is_reference_architecture():
    m = WeatherClassifier(5)
    sd = m.state_dict()
    assert set(sd) == REFERENCE_KEYS
    assert sd["net.0.weight"].shape == (64, 5) and sd["net.3.weight"].shape == (2, 64)
    assert dict(m.hparams) == {"input_dim": 5}
    assert sum(p.numel() for p in m.parameters()) == 514
    assert isinstance(m.net[2], torch.nn.Dropout) and m.net[2].p == 0.2
    opt = m.configure_optimizers()
    assert isinstance(opt, torch.optim.Adam) and opt.param_groups[0]["lr"] == 0.01


def test_mlp_hparams_and_presets():
    m = MLPClassifier(7, hidden=(32, 16), num_classes=3, dropout=0.1, loss="mse")
    assert m.hparams["hidden"] == [32, 16] and m.hparams["loss"] == "mse"
    assert m.fused_spec()["dims"] == [7, 32, 16, 3]
    assert [k for k in m.state_dict()] == ["net.0.weight", "net.0.bias", "net.3.weight", "net.3.bias",
                                           "net.6.weight", "net.6.bias"]


def _ckpt(model, tmp_path, name="x.ckpt"):
    opt = FlatAdam(torch.cat([p.detach().reshape(-1) for p in model.parameters()]),
                   torch.zeros(sum(p.numel() for p in model.parameters())), [p.shape for p in model.parameters()],
                   lr=0.01)
    opt.g.normal_()
    opt.step()
    cb = ModelCheckpoint(dirpath=str(tmp_path), monitor="val_loss")
    ck = build_checkpoint(model.state_dict(), epoch=3, global_step=400, optimizer_states=[opt.state_dict()],
                          callbacks={cb.state_key: cb.state_dict()}, hyper_parameters=dict(model.hparams))
    return save_checkpoint(ck, str(tmp_path / name))


def test_checkpoint_layout_weights_only_and_load_from_checkpoint(tmp_path):
    m = WeatherClassifier(5)
    path = _ckpt(m, tmp_path)
    ck = torch.load(path, weights_only=True)  # no arbitrary unpickling needed
    assert set(ck) == set(CHECKPOINT_KEYS)
    assert ck["pytorch-lightning_version"] == "2.1.0" and ck["hparams_name"] == "kwargs"
    assert ck["epoch"] == 3 and ck["global_step"] == 400
    assert set(ck["state_dict"]) == REFERENCE_KEYS
    assert all(t.dtype == torch.float32 and t.device.type == "cpu" for t in ck["state_dict"].values())
    st = ck["optimizer_states"][0]
    assert set(st["state"][0]) == {"step", "exp_avg", "exp_avg_sq"}
    assert st["param_groups"][0]["betas"] == (0.9, 0.999) and st["param_groups"][0]["params"] == [0, 1, 2, 3]
    key = next(iter(ck["callbacks"]))
    assert key.startswith("ModelCheckpoint{'monitor': 'val_loss', 'mode': 'min'")
    assert "fit_loop" in ck["loops"] and "epoch_loop.state_dict" in ck["loops"]["fit_loop"]
    m2 = WeatherClassifier.load_from_checkpoint(path, input_dim=5)
    for k, v in m.state_dict().items():
        assert torch.equal(v, m2.state_dict()[k])


def test_flat_adam_state_dict_matches_torch_adam():
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(5, 8), torch.nn.ReLU(), torch.nn.Linear(8, 2))
    flat = torch.cat([p.detach().reshape(-1) for p in net.parameters()])
    g = torch.zeros_like(flat)
    fa = FlatAdam(flat.clone(), g, [p.shape for p in net.parameters()], lr=0.01)
    opt = torch.optim.Adam(net.parameters(), lr=0.01)
    for _ in range(3):
        grads = [torch.randn_like(p) for p in net.parameters()]
        for p, gg in zip(net.parameters(), grads):
            p.grad = gg
        opt.step()
        fa.g.copy_(torch.cat([gg.reshape(-1) for gg in grads]))
        fa.step()
    assert torch.allclose(fa.p, torch.cat([p.detach().reshape(-1) for p in net.parameters()]), atol=1e-6)
    a, b = fa.state_dict(), opt.state_dict()
    assert set(a["param_groups"][0]) == set(b["param_groups"][0])
    for i in b["state"]:
        assert torch.allclose(a["state"][i]["exp_avg"], b["state"][i]["exp_avg"], atol=1e-7)
        assert float(a["state"][i]["step"]) == float(b["state"][i]["step"])
    # torch can load our state dict
    opt.load_state_dict(a)


def test_model_checkpoint_naming_topk_and_last(tmp_path):
    cb = ModelCheckpoint(dirpath=str(tmp_path), filename="weather-best-{epoch:02d}-{val_loss:.2f}", monitor="val_loss",
                         mode="min", save_top_k=1, save_last=True)
    written = []

    def save(p):
        written.append(os.path.basename(p))
        open(p, "w").write("x")

    cb.on_validation_end({"val_loss": 0.61, "epoch": 0}, save, True, 0)
    assert written == ["weather-best-epoch=00-val_loss=0.61.ckpt", "last.ckpt"]
    cb.on_validation_end({"val_loss": 0.70, "epoch": 1}, save, True, 1)  # worse: only last
    assert written[-1] == "last.ckpt" and len(written) == 3
    cb.on_validation_end({"val_loss": 0.45, "epoch": 2}, save, True, 2)
    assert "weather-best-epoch=02-val_loss=0.45.ckpt" in written
    files = sorted(os.listdir(tmp_path))
    assert files == ["last.ckpt", "weather-best-epoch=02-val_loss=0.45.ckpt"]
    assert cb.best_model_path.endswith("epoch=02-val_loss=0.45.ckpt") and abs(cb.best_model_score - 0.45) < 1e-9
    st = cb.state_dict()
    assert st["best_model_path"] == cb.best_model_path and float(st["best_model_score"]) == pytest.approx(0.45)
    # name collision -> -v1
    cb2 = ModelCheckpoint(dirpath=str(tmp_path), filename="weather-best-{epoch:02d}-{val_loss:.2f}",
                          monitor="val_loss", save_top_k=-1)
    cb2.on_validation_end({"val_loss": 0.45, "epoch": 2}, save, True, 2)
    assert written[-1] == "weather-best-epoch=02-val_loss=0.45-v1.ckpt"


def test_file_store_client_roundtrip(tmp_path):
    c = MlflowClient(str(tmp_path / "mlruns"))
    exp = c.get_or_create_experiment("weather_forecasting")
    assert c.get_or_create_experiment("weather_forecasting") == exp
    runs = []
    for i, vl in enumerate([0.5, 0.3, 0.4]):
        info = c.create_run(exp)
        c.log_batch(info.run_id, metrics=[{"key": "val_loss", "value": vl + 1.0, "step": 0},
                                          {"key": "val_loss", "value": vl, "step": 10}],
                    params=[{"key": "input_dim", "value": 5}])
        f = tmp_path / f"m{i}.ckpt"
        f.write_text(f"model{i}")
        c.log_artifact(info.run_id, str(f), "best_checkpoints")
        c.set_terminated(info.run_id)
        runs.append(info.run_id)
    best = c.search_runs([exp], order_by=["metrics.val_loss ASC"], max_results=1)
    assert best[0].info.run_id == runs[1] and best[0].data.metrics["val_loss"] == pytest.approx(0.3)
    assert best[0].info.status == "FINISHED" and best[0].data.params["input_dim"] == "5"
    dst = c.download_artifacts(runs[1], "best_checkpoints", str(tmp_path / "dl"))
    assert open(os.path.join(dst, "m1.ckpt")).read() == "model1"


@pytest.mark.parametrize("proxy", [False, True])
def test_rest_client_against_tracking_server(tmp_path, proxy):
    srv = TrackingServer(str(tmp_path / "srv"), serve_artifacts=proxy).start()
    try:
        lg = MLFlowLogger("weather_forecasting", tracking_uri=srv.url, log_model=True)
        lg.log_hyperparams({"input_dim": 5})
        for s in range(12):
            lg.log_metrics({"train_loss": 1.0 / (s + 1)}, s)
        lg.log_metrics({"val_loss": 0.25, "epoch": 0}, 12)
        ck = tmp_path / "weather-best-epoch=00-val_loss=0.25.ckpt"
        ck.write_bytes(b"\x00ckpt")
        lg.after_save_checkpoint(str(ck))
        lg.finalize("success")
        lg.experiment.log_artifact(lg.run_id, str(ck), "best_checkpoints")
        c = MlflowClient(srv.url)
        e = c.get_experiment_by_name("weather_forecasting")
        runs = c.search_runs([e.experiment_id], order_by=["metrics.val_loss ASC"], max_results=1)
        r = runs[0]
        assert r.info.run_id == lg.run_id and r.info.status == "FINISHED"
        assert r.data.metrics["val_loss"] == pytest.approx(0.25) and r.data.params["input_dim"] == "5"
        assert r.info.artifact_uri.startswith("mlflow-artifacts:" if proxy else "file://")
        dst = c.download_artifacts(r.info.run_id, "best_checkpoints", str(tmp_path / "dl"))
        assert open(os.path.join(dst, ck.name), "rb").read() == b"\x00ckpt"
        hist = c.store.metric_history(r.info.run_id, "train_loss") if not c.is_remote else None
        assert hist is None
    finally:
        srv.stop()


def test_model_checkpoint_nan_first_score_does_not_lock_in(tmp_path):
    """Lightning 2.1 stores a NaN monitor value as +inf (min mode): the next real score replaces it."""
    cb = ModelCheckpoint(dirpath=str(tmp_path), filename="weather-best-{epoch:02d}-{val_loss:.2f}", monitor="val_loss",
                         mode="min", save_top_k=1, save_last=False)

    def save(p):
        open(p, "w").write("x")

    cb.on_validation_end({"val_loss": float("nan"), "epoch": 0}, save, True, 0)
    assert cb.best_model_score == float("inf")
    cb.on_validation_end({"val_loss": 0.9, "epoch": 1}, save, True, 1)
    assert cb.best_model_path.endswith("epoch=01-val_loss=0.90.ckpt") and cb.best_model_score == pytest.approx(0.9)
    assert sorted(os.listdir(tmp_path)) == ["weather-best-epoch=01-val_loss=0.90.ckpt"]
    (tmp_path / "max").mkdir()
    cbx = ModelCheckpoint(dirpath=str(tmp_path / "max"), monitor="val_acc", mode="max", save_top_k=1)
    cbx.on_validation_end({"val_acc": float("nan"), "epoch": 0}, save, True, 0)
    assert cbx.best_model_score == float("-inf")
    cbx.on_validation_end({"val_acc": 0.5, "epoch": 1}, save, True, 1)
    assert cbx.best_model_score == pytest.approx(0.5)


def test_tracking_server_rejects_paths_outside_its_roots(tmp_path):
    """Artifact paths are contained component-wise (a sibling dir sharing the root's name prefix is
    outside), and experiment / run ids must be MLflow-shaped before they reach a path."""
    import requests

    root = tmp_path / "srv"
    srv = TrackingServer(str(root), serve_artifacts=True).start()
    try:
        api = srv.url + "/api/2.0"
        sibling = str(srv.state.artifacts_root) + "_x"
        r = requests.put(api + "/mlflow-artifacts/artifacts/%2e%2e/" + os.path.basename(sibling) + "/f", data=b"x",
                         timeout=30)
        assert r.status_code == 403 and not os.path.exists(os.path.join(sibling, "f"))
        r = requests.put(api + "/mlflow-artifacts/artifacts/%2e%2e/%2e%2e/evil", data=b"x", timeout=30)
        assert r.status_code == 403 and not (tmp_path / "evil").exists()
        r = requests.post(api + "/mlflow/runs/create", json={"experiment_id": "../.."}, timeout=30)
        assert r.status_code == 400
        r = requests.post(api + "/mlflow/runs/create", json={"experiment_id": "977"}, timeout=30)
        assert r.status_code == 404
        for bad in ("../../0", "0" * 31 + "/", "a" * 33):
            r = requests.post(api + "/mlflow/runs/log-batch", json={"run_id": bad, "metrics": []}, timeout=30)
            assert r.status_code == 400, bad
            r = requests.get(api + "/mlflow/runs/get", params={"run_id": bad}, timeout=30)
            assert r.status_code == 400, bad
        r = requests.post(api + "/mlflow/runs/search", json={"experiment_ids": ["../"]}, timeout=30)
        assert r.status_code == 400
        ok = requests.put(api + "/mlflow-artifacts/artifacts/1/abc/artifacts/m.ckpt", data=b"y", timeout=30)
        assert ok.status_code == 200
    finally:
        srv.stop()
