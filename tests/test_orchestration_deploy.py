"""DAG definitions, the local DAG runner, deployment packaging, score.py and the Azure rollout (CPU)."""
import datetime as dt
import importlib.util
import json
import os
import sys

import pytest
import torch

import dct_amd  # noqa: F401
from dct_amd.ckpt import build_checkpoint, save_checkpoint
from dct_amd.deploy.azure import (AzureConfig, FakeMLClient, automated_rollout, choose_slots, force_deploy)
from dct_amd.deploy.package import prepare_package
from dct_amd.models.mlp import WeatherClassifier
from dct_amd.orchestration import airflow_compat as af
from dct_amd.orchestration.dags import Targets, build_all
from dct_amd.tracking import MlflowClient

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# Reference task chains (dags/*.py: the `>>` lines)
REFERENCE_CHAINS = {
    "distributed_data_pipeline": ["start_pipeline", "check_spark_cluster", "spark_preprocessing",
                                  "verify_preprocessing_output", "check_pytorch_cluster", "copy_data_to_pytorch_nodes",
                                  "pytorch_lightning_ddp_training", "verify_model_checkpoint",
                                  "check_tensorboard_logs", "generate_training_report", "cleanup_and_prepare",
                                  "end_pipeline", "trigger_azure_rollout"],
    "spark_etl_pipeline": ["start_etl", "check_spark_cluster", "spark_preprocessing", "verify_output",
                           "trigger_training_dag"],
    "pytorch_training_pipeline": ["start_training", "cleanup_zombies", "check_gpu_cluster", "pytorch_ddp_training",
                                  "verify_model", "trigger_azure_rollout"],
    "azure_manual_deploy": ["prepare_package", "force_deploy_100"],
    "azure_automated_rollout": ["prepare_package", "deploy_new_slot", "shadow_traffic", "wait_shadow",
                                "canary_traffic", "wait_canary", "full_rollout"],
}


def _local_targets(tmp, **extra):
    env = {"DCT_EXEC_MODE": "local", "DCT_WORKDIR": ROOT, "DCT_PYTHON": sys.executable,
           "DCT_RAW_CSV": str(tmp / "raw" / "weather.csv"), "DCT_PROCESSED_OUT": str(tmp / "processed" / "data.parquet"),
           "DCT_DATA_DIR": str(tmp / "processed"), "DCT_MODEL_DIR": str(tmp / "models"), "DCT_GPUS_PER_NODE": "1",
           "MASTER_PORT": "29531"}
    env.update(extra)
    return Targets(env)


def test_dag_ids_and_task_chains_match_reference():
    dags = build_all(Targets({"DCT_EXEC_MODE": "docker"}))
    assert set(dags) == set(REFERENCE_CHAINS)
    for dag_id, chain in REFERENCE_CHAINS.items():
        dag = dags[dag_id]
        if af.HAVE_AIRFLOW:  # pragma: no cover
            continue
        assert [t.task_id for t in dag.topological_sort()] == chain
        for a, b in zip(chain, chain[1:]):
            assert b in dag.get_task(a).downstream_task_ids
    assert dags["distributed_data_pipeline"].schedule_interval == "@daily"
    assert dags["pytorch_training_pipeline"].schedule_interval is None
    # reference D2: the monolithic DAG must trigger a DAG that exists
    for dag_id in ("distributed_data_pipeline", "pytorch_training_pipeline"):
        assert dags[dag_id].get_task("trigger_azure_rollout").trigger_dag_id == "azure_automated_rollout"
    assert dags["spark_etl_pipeline"].get_task("trigger_training_dag").trigger_dag_id == "pytorch_training_pipeline"
    train = dags["distributed_data_pipeline"].get_task("pytorch_lightning_ddp_training")
    assert train.execution_timeout == dt.timedelta(hours=3) and train.retries == 1
    assert "torch.distributed.run" in train.bash_command and "docker exec pytorch-master" in train.bash_command
    assert "sleep 5" not in train.bash_command  # reference D9
    ckpt = dags["distributed_data_pipeline"].get_task("verify_model_checkpoint").bash_command
    assert "last.ckpt" in ckpt and "weather-best-" in ckpt  # reference D5
    zombies = dags["pytorch_training_pipeline"].get_task("cleanup_zombies").bash_command
    assert "pkill" not in zombies and ".trainer.pid" in zombies


def test_dag_folder_files_match_reference_names():
    """One DAG file per reference DAG file (dags/pipeline.py, 1_spark_etl.py, ...), each exposing its DAG."""
    files = {"pipeline.py": "distributed_data_pipeline", "1_spark_etl.py": "spark_etl_pipeline",
             "2_pytorch_training.py": "pytorch_training_pipeline", "azure_manual_deploy.py": "azure_manual_deploy",
             "azure_auto_deploy.py": "azure_automated_rollout"}
    assert set(files.values()) == set(REFERENCE_CHAINS)
    for fn, dag_id in files.items():
        spec = importlib.util.spec_from_file_location("dagfile_" + fn[:-3], os.path.join(ROOT, "dags", fn))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        assert mod.dag.dag_id == dag_id


def test_reference_named_job_entry_points(tmp_path):
    """jobs/preprocess.py and jobs/train_lightning_ddp.py forward to the framework jobs."""
    import subprocess
    import sys
    for job in ("preprocess.py", "train_lightning_ddp.py"):
        out = subprocess.run([sys.executable, os.path.join(ROOT, "jobs", job), "--help"], capture_output=True,
                             text=True, timeout=300)
        assert out.returncode == 0, out.stderr
        assert "--engine" in out.stdout


@pytest.mark.skipif(af.HAVE_AIRFLOW, reason="stand-in runner only")
def test_local_runner_retries_xcom_and_upstream_failed():
    calls = []
    with af.DAG("t_retry", default_args={"retries": 2, "retry_delay": dt.timedelta(seconds=7)}) as dag:
        def push(ti=None, **_):
            ti.xcom_push(key="k", value=41)
            return "ok"

        def flaky(ti=None, **_):
            calls.append(ti.try_number)
            if len(calls) < 2:
                raise RuntimeError("transient")
            return ti.xcom_pull(task_ids="a", key="k") + 1

        a = af.PythonOperator(task_id="a", python_callable=push)
        b = af.PythonOperator(task_id="b", python_callable=flaky)
        c = af.BashOperator(task_id="c", bash_command="exit 3", retries=0)
        d = af.BashOperator(task_id="d", bash_command="echo never")
        a >> b >> c >> d
    slept = []
    res = af.LocalDagRunner(sleep=slept.append).run(dag)
    assert res.task_states == {"a": "success", "b": "success", "c": "failed", "d": "upstream_failed"}
    assert calls == [1, 2] and slept == [7.0]
    assert res.xcom[("b", "return_value")] == 42 and res.state == "failed"
    assert "exit code 3" in res.errors["c"]


def _fake_mlflow_run(tmp, val_losses=(0.7, 0.4)):
    """Two finished runs with best_checkpoints artifacts; returns (uri, best_run_id)."""
    uri = "file://" + str(tmp / "mlruns")
    client = MlflowClient(uri)
    exp = client.get_or_create_experiment("weather_forecasting")
    best = None
    for i, vl in enumerate(val_losses):
        run = client.create_run(exp).run_id
        torch.manual_seed(i)
        model = WeatherClassifier(5)
        ck = tmp / f"weather-best-epoch={i:02d}-val_loss={vl:.2f}.ckpt"
        save_checkpoint(build_checkpoint(model.state_dict(), epoch=i, global_step=10,
                                         hyper_parameters={"input_dim": 5}), str(ck))
        client.log_batch(run, metrics=[{"key": "val_loss", "value": vl, "step": 1}])
        client.log_artifact(run, str(ck), "best_checkpoints")
        client.set_terminated(run)
        if best is None or vl < best[1]:
            best = (run, vl, model)
    return uri, best[0], best[2]


def _load_score(deploy_dir, monkeypatch):
    monkeypatch.setenv("AZUREML_MODEL_DIR", str(deploy_dir))
    spec = importlib.util.spec_from_file_location("score_under_test", os.path.join(deploy_dir, "score.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_prepare_package_picks_best_run_and_score_contract(tmp_path, monkeypatch):
    uri, best_run, best_model = _fake_mlflow_run(tmp_path)
    stats = tmp_path / "stats.json"
    stats.write_text(json.dumps({c: {"mean": 1.0, "std": 2.0} for c in
                                 ["Temperature", "Humidity", "Wind_Speed", "Cloud_Cover", "Pressure"]}))
    d = tmp_path / "deploy"
    d.mkdir()
    (d / "stale.txt").write_text("x")
    info = prepare_package(str(d), tracking_uri=uri, norm_stats=str(stats))
    assert info["run_id"] == best_run and abs(info["val_loss"] - 0.4) < 1e-9
    assert {"model.ckpt", "score.py", "conda.yaml", "norm_stats.json"} <= set(os.listdir(d))
    assert not (d / "stale.txt").exists()
    score = _load_score(d, monkeypatch)
    score.init()
    x = [[0.1, -0.2, 0.3, 0.0, 1.0], [1.0, 1.0, 1.0, 1.0, 1.0]]
    out = score.run(json.dumps({"data": x}))
    best_model.eval()
    want = torch.softmax(best_model(torch.tensor(x)), dim=1)
    assert torch.allclose(torch.tensor(out["probabilities"]), want, atol=1e-6)
    raw = score.run(json.dumps({"data": [[3.0] * 5], "raw": True}))
    assert torch.allclose(torch.tensor(raw["probabilities"]),
                          torch.softmax(best_model(torch.ones(1, 5)), dim=1), atol=1e-6)
    assert "error" in score.run("{not json")
    assert "error" in score.run(json.dumps({"data": [[1.0, 2.0]]}))


def test_score_finds_nested_checkpoint(tmp_path, monkeypatch):
    uri, _, _ = _fake_mlflow_run(tmp_path, (0.5,))
    d = tmp_path / "pkg"
    prepare_package(str(d), tracking_uri=uri)
    nested = tmp_path / "azure_model" / "deployment_staging"
    nested.mkdir(parents=True)
    os.replace(d / "model.ckpt", nested / "model.ckpt")
    monkeypatch.setenv("AZUREML_MODEL_DIR", str(tmp_path / "azure_model"))
    spec = importlib.util.spec_from_file_location("score_nested", os.path.join(d, "score.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    mod.init()
    assert len(mod.run({"data": [[0.0] * 5]})["probabilities"][0]) == 2


def test_prepare_package_errors(tmp_path):
    uri = "file://" + str(tmp_path / "empty")
    with pytest.raises(ValueError):
        prepare_package(str(tmp_path / "d"), tracking_uri=uri)
    with pytest.raises(ValueError):
        prepare_package("", tracking_uri=uri)


def test_slot_choice_and_blue_green_rollout():
    assert choose_slots({}) == ("blue", "blue")
    assert choose_slots({"blue": 100}) == ("blue", "green")
    assert choose_slots({"blue": 10, "green": 90}) == ("green", "blue")
    cfg = AzureConfig(endpoint_name="weather-ep", deploy_dir="/pkg", wait_s=0)
    client = FakeMLClient()
    assert force_deploy(client, cfg) == "blue"
    assert client.online_endpoints.get("weather-ep").traffic == {"blue": 100}
    r = automated_rollout(client, cfg, sleep=lambda s: None)
    assert r == {"old_slot": "blue", "new_slot": "green", "status": "complete"}
    traffic_log = [e[2:] for e in client.log if e[0] == "endpoint"]
    assert ({"blue": 100, "green": 0}, {"green": 20}) in traffic_log
    assert ({"blue": 90, "green": 10}, {}) in traffic_log
    assert client.online_endpoints.get("weather-ep").traffic == {"green": 100}
    assert ("delete_deployment", "blue") in client.log
    # health gate: probe fails during canary -> everything back on green, blue removed
    probes = []

    def probe(slot):
        probes.append(slot)
        return len(probes) < 2  # healthy in shadow, unhealthy in canary

    r2 = automated_rollout(client, cfg, probe=probe, sleep=lambda s: None)
    assert r2["status"] == "rolled_back_at_canary" and r2["old_slot"] == "green" and probes == ["blue", "blue"]
    assert client.online_endpoints.get("weather-ep").traffic == {"green": 100}
    assert ("weather-ep", "blue") not in client.deployments


def test_force_deploy_recreates_failed_endpoint():
    cfg = AzureConfig(endpoint_name="ep", deploy_dir="/pkg")
    client = FakeMLClient()
    force_deploy(client, cfg)
    client.endpoints["ep"].provisioning_state = "Failed"
    force_deploy(client, cfg)
    assert ("delete_endpoint", "ep") in client.log
    assert client.online_endpoints.get("ep").traffic == {"blue": 100}


@pytest.mark.slow
@pytest.mark.skipif(af.HAVE_AIRFLOW, reason="stand-in runner only")
def test_end_to_end_etl_train_rollout_local(tmp_path, monkeypatch):
    """spark_etl_pipeline (arrow engine) -> pytorch_training_pipeline (torchrun, CPU) ->
    azure_automated_rollout (fake Azure client), chained by TriggerDagRunOperator."""
    from dct_amd.data.synthetic import make_weather_csv
    from dct_amd.orchestration import dags as dags_mod

    (tmp_path / "raw").mkdir()
    make_weather_csv(str(tmp_path / "raw" / "weather.csv"), n=400, seed=0)
    uri = "file://" + str(tmp_path / "mlruns")
    monkeypatch.setenv("MLFLOW_TRACKING_URI", uri)
    monkeypatch.setenv("DCT_AZURE_FAKE", "1")
    monkeypatch.setenv("DEPLOY_DIR", str(tmp_path / "deploy"))
    monkeypatch.setenv("ENDPOINT_NAME", "weather-ep")
    monkeypatch.setenv("DCT_ROLLOUT_WAIT_S", "0")
    monkeypatch.setenv("DCT_MODEL_DIR", str(tmp_path / "models"))
    monkeypatch.setenv("DCT_NORM_STATS", str(tmp_path / "processed" / "data.parquet" / "_norm_stats.json"))
    monkeypatch.setattr(dags_mod, "_FAKE_CLIENT", FakeMLClient())
    t = _local_targets(tmp_path, DCT_TRAIN_ARGS=f"--accelerator cpu --epochs 2 --tracking-uri {uri}")
    dags = build_all(t)
    runner = af.LocalDagRunner(follow_triggers=True, sleep=lambda s: None)
    res = runner.run(dags["spark_etl_pipeline"])
    states = {r.dag_id: (r.state, r.task_states, r.errors) for r in runner.results}
    assert res.state == "success", states
    assert [r.dag_id for r in runner.results] == ["spark_etl_pipeline", "pytorch_training_pipeline",
                                                   "azure_automated_rollout"]
    assert all(r.state == "success" for r in runner.results), states
    models = os.listdir(tmp_path / "models")
    assert "last.ckpt" in models and any(m.startswith("weather-best-") for m in models)
    client = dags_mod._FAKE_CLIENT
    assert client.online_endpoints.get("weather-ep").traffic == {"blue": 100}
    assert {"model.ckpt", "score.py", "conda.yaml", "norm_stats.json"} <= set(os.listdir(tmp_path / "deploy"))


def test_train_3x128_package_and_serve(tmp_path, monkeypatch):
    """serve what you train.  jobs/train_ddp.py trains BASELINE's weather-mlp-3x128
    (5-128-128-2) for one epoch on CPU into an MLflow file store; prepare_package derives the
    architecture from the best checkpoint (not the reference's one hidden layer), and score.py's
    init()/run() serve it: probabilities [n, 2] equal to the trained model's softmax.  The
    reference 5-64-2 package keeps working (test above)."""
    import subprocess
    import sys

    from dct_amd.ckpt.lightning_io import load_checkpoint
    from dct_amd.models.mlp import build_mlp

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    uri = "file://" + str(tmp_path / "mlruns")
    r = subprocess.run([sys.executable, os.path.join(root, "jobs", "train_ddp.py"), "--model", "weather-mlp-3x128",
                        "--epochs", "1", "--synthetic-rows", "400", "--accelerator", "cpu",
                        "--model-dir", str(tmp_path / "models"), "--tracking-uri", uri],
                       capture_output=True, text=True, timeout=600, env=dict(os.environ, WORLD_SIZE="1"))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    d = tmp_path / "deploy"
    info = prepare_package(str(d), tracking_uri=uri)
    ck = load_checkpoint(info["checkpoint"])
    assert ck["state_dict"]["net.3.weight"].shape == (128, 128) and ck["state_dict"]["net.6.weight"].shape == (2, 128)
    model = build_mlp("weather-mlp-3x128", 5)
    model.load_state_dict(ck["state_dict"])
    model.eval()
    score = _load_score(d, monkeypatch)
    score.init()
    x = torch.randn(7, 5).tolist()
    out = score.run(json.dumps({"data": x}))
    probs = torch.tensor(out["probabilities"])
    assert probs.shape == (7, 2)
    assert torch.allclose(probs, torch.softmax(model(torch.tensor(x)), dim=1), atol=1e-6)
    assert "error" in score.run(json.dumps({"data": [[1.0, 2.0]]}))


def test_mlp_architecture_from_state_dict():
    from dct_amd.deploy.package import mlp_architecture
    from dct_amd.models.mlp import WeatherClassifier, build_mlp

    assert mlp_architecture(WeatherClassifier(5).state_dict()) == {"input_dim": 5, "hidden": [64], "classes": 2}
    assert mlp_architecture(build_mlp("tabular-mlp-4x1024", 256).state_dict()) == {
        "input_dim": 256, "hidden": [1024, 1024, 1024], "classes": 2}
    with pytest.raises(ValueError):
        mlp_architecture({"blocks.0.weight": torch.zeros(2, 2)})


def test_train_tabtransformer_package_and_serve(tmp_path, monkeypatch):
    """BASELINE config 5 is servable.  jobs/train_ddp.py trains a TabTransformer
    (5 feature tokens, the weather data) for one epoch on CPU into an MLflow file store;
    prepare_package recognises the checkpoint and writes a score.py that re-declares the model in
    plain torch from its hyper-parameters; init()/run() give the trained model's softmax."""
    import subprocess
    import sys

    from dct_amd.ckpt.lightning_io import load_checkpoint
    from dct_amd.models import build_model

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    uri = "file://" + str(tmp_path / "mlruns")
    r = subprocess.run([sys.executable, os.path.join(root, "jobs", "train_ddp.py"), "--model", "tabtransformer",
                        "--epochs", "1", "--synthetic-rows", "400", "--accelerator", "cpu",
                        "--model-dir", str(tmp_path / "models"), "--tracking-uri", uri],
                       capture_output=True, text=True, timeout=600, env=dict(os.environ, WORLD_SIZE="1"))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    d = tmp_path / "deploy"
    info = prepare_package(str(d), tracking_uri=uri)
    assert "model family: tabtransformer" in (d / "score.py").read_text()
    ck = load_checkpoint(info["checkpoint"])
    hp = ck["hyper_parameters"]
    model = build_model("tabtransformer", hp["num_features"], **{k: hp[k] for k in ("d_model", "heads", "layers")})
    model.load_state_dict(ck["state_dict"])
    model.eval()
    score = _load_score(d, monkeypatch)
    score.init()
    x = torch.randn(6, hp["num_features"]).tolist()
    out = score.run(json.dumps({"data": x}))
    probs = torch.tensor(out["probabilities"])
    assert probs.shape == (6, 2)
    with torch.no_grad():
        want = torch.softmax(model(torch.tensor(x)), dim=1)
    assert torch.allclose(probs, want, atol=1e-5), (probs - want).abs().max()
    assert "error" in score.run(json.dumps({"data": [[1.0, 2.0]]}))


def test_prepare_package_refuses_unknown_architecture(tmp_path):
    """A checkpoint of no servable family fails packaging with an error naming the problem."""
    uri = "file://" + str(tmp_path / "mlruns")
    client = MlflowClient(uri)
    exp = client.get_or_create_experiment("weather_forecasting")
    run = client.create_run(exp).run_id
    ck = tmp_path / "odd.ckpt"
    save_checkpoint(build_checkpoint({"encoder.weight": torch.zeros(4, 4)}, epoch=0, global_step=1,
                                     hyper_parameters={}), str(ck))
    client.log_batch(run, metrics=[{"key": "val_loss", "value": 0.5, "step": 1}])
    client.log_artifact(run, str(ck), "best_checkpoints")
    with pytest.raises(ValueError, match="unsupported architecture"):
        prepare_package(str(tmp_path / "d"), tracking_uri=uri)
    from dct_amd.deploy.package import tabtransformer_architecture

    with pytest.raises(ValueError, match="heads"):
        from dct_amd.models.tabtransformer import TabTransformer

        tabtransformer_architecture(TabTransformer(num_features=5, d_model=16, heads=2, layers=2).state_dict(), {})
