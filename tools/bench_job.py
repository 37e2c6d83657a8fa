#!/usr/bin/env python3
"""End-to-end wall-clock of the reference TRAINING JOB (not just the step): the second half of
BASELINE.json's headline metric ("samples/sec ...; epoch wall-clock").

Reference job (jobs/train_lightning_ddp.py:90-166): parquet -> WeatherDataset -> 80/20 split ->
10 epochs of batch-4 Adam steps with a full validation pass per epoch, ModelCheckpoint (top-1 +
last.ckpt), MLflow logging every 5 steps, best_checkpoints upload.  Here the same job runs through
jobs/train_ddp.py (fused HIP engine on the GPU, or the autograd engine with --accelerator cpu)
on a synthetic raw CSV pushed through the ETL first:

    python tools/bench_job.py --rows 100000 --epochs 10 [--accelerator cpu]

Prints one JSON line: ETL seconds, job wall-clock (process start to exit), per-epoch wall-clock
(train + validation + checkpoint + logging, from the trainer's own clock) and train samples/s.
"""
import argparse
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rows", type=int, default=100_000)
    p.add_argument("--epochs", type=int, default=10)
    p.add_argument("--accelerator", default="gpu")
    p.add_argument("--no-mlflow", action="store_true")
    p.add_argument("--model", default="", help="jobs/train_ddp.py --model (default: the job's own)")
    p.add_argument("--keep", action="store_true", help="keep the work directory (data, checkpoints, mlruns)")
    a = p.parse_args()

    from dct_amd.data.etl import run_arrow_etl
    from dct_amd.data.synthetic import make_weather_csv

    work = tempfile.mkdtemp(prefix="dct_job_")
    try:
        return _run(a, work, run_arrow_etl, make_weather_csv)
    finally:
        if not a.keep:
            shutil.rmtree(work, ignore_errors=True)


def _run(a, work, run_arrow_etl, make_weather_csv):
    raw = os.path.join(work, "raw", "weather.csv")
    make_weather_csv(raw, n=a.rows, seed=0)
    t0 = time.perf_counter()
    run_arrow_etl(raw, os.path.join(work, "processed", "data.parquet"), num_parts=2, verbose=False)
    etl_s = time.perf_counter() - t0

    cmd = [sys.executable, os.path.join(ROOT, "jobs", "train_ddp.py"), "--data-dir", os.path.join(work, "processed"),
           "--model-dir", os.path.join(work, "models"), "--epochs", str(a.epochs), "--accelerator", a.accelerator,
           "--tracking-uri", "file://" + os.path.join(work, "mlruns")]
    if a.no_mlflow:
        cmd.append("--no-mlflow")
    if a.model:
        cmd += ["--model", a.model]
    t0 = time.perf_counter()
    r = subprocess.run(cmd, capture_output=True, text=True, cwd=ROOT)
    job_s = time.perf_counter() - t0
    if r.returncode != 0:
        sys.stderr.write(r.stdout[-4000:] + r.stderr[-4000:])
        return r.returncode
    epochs = [float(m.group(1)) for m in re.finditer(r"epoch_time=([0-9.]+)s", r.stdout)]
    sps = [float(m.group(1)) for m in re.finditer(r"train_samples/s=([0-9.]+)", r.stdout)]
    engine = re.search(r"engine=(\S+)", r.stdout)
    out = {
        "metric": "reference training job wall-clock (ETL'd parquet, 10 epochs, val, ckpt, MLflow)",
        "accelerator": a.accelerator,
        "model": a.model or "job default",
        "engine": engine.group(1) if engine else None,
        "rows": a.rows,
        "epochs": a.epochs,
        "etl_s": round(etl_s, 3),
        "job_wall_s": round(job_s, 3),
        "epoch_wall_s": [round(e, 4) for e in epochs],
        "epoch_wall_s_median": round(sorted(epochs)[len(epochs) // 2], 4) if epochs else None,
        "train_samples_per_s_median": round(sorted(sps)[len(sps) // 2]) if sps else None,
        "data": "synthetic raw CSV through the ETL",
    }
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
