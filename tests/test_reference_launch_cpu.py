"""The reference's own launch style (docker-compose.yml:119-124,138-143; dags/2_pytorch_training.py:
55-61): two PLAIN ``python3 jobs/train_lightning_ddp.py`` processes - no torchrun, no ``RANK`` -
one per "node", told only ``WORLD_SIZE=2``, ``NODE_RANK=0/1``, ``MASTER_ADDR``, ``MASTER_PORT``.
``parallel.dist.resolve_env`` must derive rank = NODE_RANK; the job reads a Spark-shaped
``data.parquet`` (``*_norm`` + ``label_encoded``), trains with gloo DDP on CPU, keeps the replicas
identical, and only rank 0 writes checkpoints and the MLflow run."""
import json
import os
import subprocess
import sys

import numpy as np
import pandas as pd
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JOB = os.path.join(ROOT, "jobs", "train_lightning_ddp.py")
TORCHRUN_KEYS = ("RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK", "TORCHELASTIC_RUN_ID",
                 "TORCHELASTIC_RESTART_COUNT", "CUDA_VISIBLE_DEVICES")


def _parquet(path, rows=240, seed=0):
    rng = np.random.default_rng(seed)
    cols = ["Temperature", "Humidity", "Wind_Speed", "Cloud_Cover", "Pressure"]
    df = pd.DataFrame({f"{c}_norm": rng.standard_normal(rows) for c in cols})
    df["label_encoded"] = (df["Humidity_norm"] + 0.3 * rng.standard_normal(rows) > 0).astype("int32")
    os.makedirs(path, exist_ok=True)
    df.to_parquet(os.path.join(path, "data.parquet"))


@pytest.mark.slow
def test_two_plain_processes_node_rank_launch(tmp_path):
    data = tmp_path / "processed"
    _parquet(str(data))
    models, mlruns, dump = tmp_path / "models", tmp_path / "mlruns", tmp_path / "params"
    port = 29671
    procs = []
    for node_rank in (0, 1):
        env = {k: v for k, v in os.environ.items() if k not in TORCHRUN_KEYS}
        env.update(WORLD_SIZE="2", NODE_RANK=str(node_rank), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   MLFLOW_TRACKING_URI="file://" + str(mlruns))
        cmd = [sys.executable, JOB, "--data-dir", str(data), "--model-dir", str(models), "--epochs", "2",
               "--accelerator", "cpu", "--tracking-uri", "file://" + str(mlruns), "--dump-params", str(dump)]
        procs.append(subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env,
                                      cwd=str(tmp_path)))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=300)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out)
    for p, out in zip(procs, outs):
        assert p.returncode == 0, out[-3000:]
    r0 = json.loads((dump / "params_rank0.json").read_text())
    r1 = json.loads((dump / "params_rank1.json").read_text())
    assert r0["world_size"] == r1["world_size"] == 2
    assert r0["params"] == r1["params"]  # DDP replicas bit-identical
    # 240 rows -> 192 train -> 96 per rank -> 24 steps per epoch, 2 epochs
    assert r0["global_step"] == r1["global_step"] == 48
    files = sorted(os.listdir(models))
    assert "last.ckpt" in files and sum(f.startswith("weather-best-") for f in files) == 1, files
    exps = [d for d in os.listdir(mlruns) if d.isdigit() and d != "0"]
    assert len(exps) == 1
    runs = [d for d in os.listdir(mlruns / exps[0]) if len(d) == 32]
    assert len(runs) == 1  # rank 0 only
    arts = mlruns / exps[0] / runs[0] / "artifacts" / "best_checkpoints"
    assert any(f.endswith(".ckpt") for f in os.listdir(arts))
    assert "Model uploaded to MLflow" in outs[0] and "Model uploaded to MLflow" not in outs[1]
