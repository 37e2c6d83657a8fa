"""SURVEY §7.3 step 4 — the minimum end-to-end slice on one MI355X: raw CSV -> ETL (arrow engine,
reference semantics) -> jobs/train_ddp.py on the GPU (fused HIP engine) -> Lightning-layout
checkpoints + MLflow file-store run with best_checkpoints -> prepare_package -> score.py on CPU."""
import importlib.util
import json
import os
import subprocess
import sys

import pytest
import torch

import dct_amd  # noqa: F401
from dct_amd.ckpt import load_checkpoint
from dct_amd.data.etl import run_arrow_etl
from dct_amd.data.synthetic import make_weather_csv
from dct_amd.deploy.package import prepare_package
from dct_amd.tracking import MlflowClient

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_csv_to_scored_endpoint_package(tmp_path, cuda, monkeypatch):
    raw = tmp_path / "raw" / "weather.csv"
    make_weather_csv(str(raw), n=3000, seed=0)
    stats = run_arrow_etl(str(raw), str(tmp_path / "processed" / "data.parquet"), num_parts=2, verbose=False)
    assert set(stats) == {"Temperature", "Humidity", "Wind_Speed", "Cloud_Cover", "Pressure"}
    uri = "file://" + str(tmp_path / "mlruns")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "jobs", "train_ddp.py"), "--data-dir",
                        str(tmp_path / "processed"), "--model-dir", str(tmp_path / "models"), "--epochs", "3",
                        "--accelerator", "gpu", "--tracking-uri", uri],
                       capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "engine=fused" in r.stdout
    models = os.listdir(tmp_path / "models")
    best = [m for m in models if m.startswith("weather-best-epoch=")]
    assert "last.ckpt" in models and len(best) == 1
    ck = load_checkpoint(str(tmp_path / "models" / best[0]))
    assert ck["hyper_parameters"] == {"input_dim": 5} and ck["pytorch-lightning_version"] == "2.1.0"
    assert all(t.dtype == torch.float32 and t.device.type == "cpu" for t in ck["state_dict"].values())
    client = MlflowClient(uri)
    exp = client.get_experiment_by_name("weather_forecasting")
    run = client.search_runs([exp.experiment_id], order_by=["metrics.val_loss ASC"], max_results=1)[0]
    assert {"train_loss", "val_loss", "val_acc", "epoch"} <= set(run.data.metrics)
    deploy = tmp_path / "deploy"
    info = prepare_package(str(deploy), tracking_uri=uri,
                           norm_stats=str(tmp_path / "processed" / "data.parquet" / "_norm_stats.json"))
    assert info["run_id"] == run.info.run_id
    monkeypatch.setenv("AZUREML_MODEL_DIR", str(deploy))
    spec = importlib.util.spec_from_file_location("e2e_score", str(deploy / "score.py"))
    score = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(score)
    score.init()
    out = score.run(json.dumps({"data": [[20.0, 90.0, 10.0, 95.0, 1000.0], [20.0, 20.0, 10.0, 5.0, 1030.0]],
                                "raw": True}))
    p = torch.tensor(out["probabilities"])
    assert p.shape == (2, 2) and torch.allclose(p.sum(1), torch.ones(2), atol=1e-5)
    assert p[0, 1] > p[1, 1]  # humid, overcast, low pressure -> rain more likely
