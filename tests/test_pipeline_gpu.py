"""The whole continuous-training chain with the training on the MI355X.

spark_etl_pipeline (arrow engine) -> TriggerDagRun -> pytorch_training_pipeline (torchrun, one
rank per GPU, fused HIP engine) -> TriggerDagRun -> azure_automated_rollout against a LIVE local
online endpoint (deploy/local_endpoint.py over HTTP, DCT_AZURE_BACKEND=local), then a scoring
request through the endpoint.  The reference chain is dags/1_spark_etl.py:67-73 ->
dags/2_pytorch_training.py:94-100 -> dags/azure_auto_deploy.py:188-197 with score.py
(dags/azure_manual_deploy.py:79-124).
"""
import json
import os

import pytest
import requests
import torch

import dct_amd  # noqa: F401
from dct_amd.ckpt import load_checkpoint
from dct_amd.deploy.local_endpoint import EndpointServer, LocalEndpoint
from dct_amd.models.mlp import WeatherClassifier
from dct_amd.orchestration import airflow_compat as af
from test_orchestration_deploy import _local_targets

pytestmark = pytest.mark.gpu

X = [[0.1, -0.2, 0.3, 0.0, 1.0], [1.0, 1.0, -1.0, 0.5, 0.0]]


@pytest.mark.skipif(af.HAVE_AIRFLOW, reason="stand-in runner only")
def test_etl_gpu_training_rollout_and_scoring(tmp_path, monkeypatch, cuda):
    from dct_amd.data.synthetic import make_weather_csv
    from dct_amd.orchestration import dags as dags_mod
    from dct_amd.orchestration.dags import build_all

    (tmp_path / "raw").mkdir()
    make_weather_csv(str(tmp_path / "raw" / "weather.csv"), n=4000, seed=0)
    uri = "file://" + str(tmp_path / "mlruns")
    ep = LocalEndpoint("weather-ep")
    srv = EndpointServer(ep, require_key=True, package_root=str(tmp_path)).start()
    try:
        for k, v in {"MLFLOW_TRACKING_URI": uri, "DCT_AZURE_BACKEND": "local", "DCT_LOCAL_ENDPOINT_URL": srv.url,
                     "DCT_LOCAL_ENDPOINT_KEY": ep.key, "ENDPOINT_NAME": "weather-ep",
                     "DEPLOY_DIR": str(tmp_path / "deploy"), "DCT_ROLLOUT_WAIT_S": "0",
                     "DCT_MODEL_DIR": str(tmp_path / "models"),
                     "DCT_NORM_STATS": str(tmp_path / "processed" / "data.parquet" / "_norm_stats.json")}.items():
            monkeypatch.setenv(k, v)
        monkeypatch.setattr(dags_mod, "_FAKE_CLIENT", None)
        t = _local_targets(tmp_path, DCT_TRAIN_ARGS=f"--accelerator gpu --epochs 3 --tracking-uri {uri}",
                           MASTER_PORT="29541")
        runner = af.LocalDagRunner(follow_triggers=True, sleep=lambda s: None)
        res = runner.run(build_all(t)["spark_etl_pipeline"])
        states = {r.dag_id: (r.state, r.task_states, r.errors) for r in runner.results}
        assert res.state == "success", states
        assert [r.dag_id for r in runner.results] == ["spark_etl_pipeline", "pytorch_training_pipeline",
                                                       "azure_automated_rollout"]
        assert all(r.state == "success" for r in runner.results), states
        models = os.listdir(tmp_path / "models")
        best = [m for m in models if m.startswith("weather-best-")]
        assert "last.ckpt" in models and len(best) == 1
        assert ep.traffic == {"blue": 100}
        # the training task ran on the GPU engine: its logged train throughput is far above the CPU
        # autograd path's (~20k samples/s on these boxes)
        from dct_amd.tracking import MlflowClient

        mc = MlflowClient(uri)
        run = mc.search_runs([mc.get_experiment_by_name("weather_forecasting").experiment_id],
                             order_by=["metrics.val_loss ASC"], max_results=1)[0]
        assert run.data.metrics["samples_per_sec"] > 2e5, run.data.metrics
        # the endpoint serves the packaged best checkpoint: same probabilities as a CPU forward of it
        r = requests.post(srv.url + "/score", data=json.dumps({"data": X}),
                          headers={"Authorization": f"Bearer {ep.key}"}, timeout=30)
        assert r.status_code == 200, r.text
        probs = torch.tensor(r.json()["probabilities"])
        ck = load_checkpoint(str(tmp_path / "deploy" / "model.ckpt"))
        model = WeatherClassifier(5)
        model.load_state_dict(ck["state_dict"])
        model.eval()
        with torch.no_grad():
            want = torch.softmax(model(torch.tensor(X)), dim=1)
        assert torch.allclose(probs, want, atol=1e-6)
    finally:
        srv.stop()
