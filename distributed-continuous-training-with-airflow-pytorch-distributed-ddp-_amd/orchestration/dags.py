"""The five pipeline DAGs (reference dags/*.py), built by functions so that the same definitions
serve a real Airflow deployment and the local runner.

DAG ids, task ids, schedules, retries and timeouts follow the reference:
  * ``distributed_data_pipeline`` (@daily, 13 tasks, pipeline.py:29-281)
  * ``spark_etl_pipeline`` (@daily, 1_spark_etl.py:14-73) -> triggers ``pytorch_training_pipeline``
  * ``pytorch_training_pipeline`` (manual/triggered, 2_pytorch_training.py:13-100) -> triggers
    ``azure_automated_rollout``
  * ``azure_manual_deploy`` (azure_manual_deploy.py:170-173)
  * ``azure_automated_rollout`` (azure_auto_deploy.py:188-197)
MI355X-first differences (deliberate, documented):
  * training is ``torchrun`` one-process-per-GPU on the trainer node(s) with elastic restarts,
    instead of two ``docker exec ... &`` + ``sleep 5`` (reference D9); the GPU health check really
    checks the GPUs and the native HIP extension;
  * verification looks for the checkpoints the trainer actually writes (``last.ckpt``,
    ``weather-best-*.ckpt``; reference D5), cleanup keeps the newest 3 of those;
  * the monolithic DAG triggers the rollout DAG that exists (reference D2 triggered
    ``azure_smart_rollout``);
  * stale trainers are stopped by PID file, never by process-name pattern.
Execution target: ``DCT_EXEC_MODE=docker`` (default, the compose topology: ``docker exec
<container> ...``) or ``local`` (commands run on the Airflow worker itself, e.g. when Airflow runs
on the GPU node, and in tests).
"""
from __future__ import annotations

import datetime as _dt
import os
import shlex
from typing import Dict, Optional

from .airflow_compat import DAG, BashOperator, PythonOperator, TriggerDagRunOperator

DEFAULT_ARGS = {
    "owner": "airflow",
    "depends_on_past": False,
    "email_on_failure": False,
    "email_on_retry": False,
    "retries": 1,
    "retry_delay": _dt.timedelta(minutes=5),
}


def _env(name: str, default: str) -> str:
    return os.environ.get(name, default)


class Targets:
    """Where each stage's commands run, resolved from the environment at DAG-build time."""

    def __init__(self, env: Optional[Dict[str, str]] = None):
        e = dict(os.environ if env is None else env)
        self.mode = e.get("DCT_EXEC_MODE", "docker")
        self.spark = e.get("DCT_SPARK_CONTAINER", "spark-master")
        self.trainer = e.get("DCT_TRAINER_CONTAINER", "pytorch-master")
        self.workdir = e.get("DCT_WORKDIR", "/workspace")
        self.python = e.get("DCT_PYTHON", "python3")
        self.etl_engine = e.get("DCT_ETL_ENGINE", "spark" if self.mode == "docker" else "arrow")
        self.raw_csv = e.get("DCT_RAW_CSV", "/opt/spark/data/raw/weather.csv")
        self.processed = e.get("DCT_PROCESSED_OUT", "/opt/spark/data/processed/data.parquet")
        self.data_dir = e.get("DCT_DATA_DIR", "/workspace/data/processed")
        self.model_dir = e.get("DCT_MODEL_DIR", "/workspace/data/models")
        self.nnodes = e.get("DCT_NNODES", "1")
        self.gpus_per_node = e.get("DCT_GPUS_PER_NODE", "8")
        self.master_addr = e.get("MASTER_ADDR", "127.0.0.1")
        self.master_port = e.get("MASTER_PORT", "29500")
        self.node_rank = e.get("NODE_RANK", "0")
        self.train_args = e.get("DCT_TRAIN_ARGS", "")

    def on(self, container: str, cmd: str) -> str:
        if self.mode == "local":
            return cmd
        return f"docker exec {container} bash -lc {shlex.quote(cmd)}"

    # ---------------------------------------------------------------- commands
    def spark_health(self) -> str:
        if self.etl_engine == "spark":
            return self.on(self.spark, "curl -sf http://localhost:8080 > /dev/null && echo 'Spark master is up'")
        return self.on(self.spark, f"{self.python} -c 'import pyarrow, pandas; print(\"arrow ETL engine ready\")'")

    def etl(self, adaptive: bool = True) -> str:
        job = f"{self.workdir}/jobs/etl_job.py"
        if self.etl_engine == "spark":
            confs = "--conf spark.executor.memory=1g --conf spark.driver.memory=1g"
            if adaptive:
                confs += " --conf spark.sql.adaptive.enabled=true"
            inner = (f"/opt/spark/bin/spark-submit --master spark://spark-master:7077 --deploy-mode client {confs} "
                     f"/opt/spark/jobs/etl_job.py --engine spark --input {self.raw_csv} --output {self.processed}")
        else:
            inner = f"{self.python} {job} --engine arrow --input {self.raw_csv} --output {self.processed}"
        return self.on(self.spark, inner)

    def verify_processed(self) -> str:
        p = shlex.quote(self.processed)
        return self.on(self.spark, f"test -d {p} && test -f {p}/_SUCCESS && ls -lh {p} && du -sh {p}")

    def trainer_health(self) -> str:
        check = ("import torch, dct_amd; n = torch.cuda.device_count(); print('torch', torch.__version__, "
                 "'hip', torch.version.hip, 'gpus', n); "
                 "from dct_amd.ops._native import native; print('native', native().arch_name(0)) if n else None")
        return self.on(self.trainer, f"cd {self.workdir} && {self.python} -c {shlex.quote(check)}")

    def data_visible(self) -> str:
        return self.on(self.trainer, f"test -d {shlex.quote(self.data_dir)}/data.parquet && echo 'data visible'")

    def train(self) -> str:
        pidfile = f"{self.model_dir}/.trainer.pid"
        inner = (
            f"mkdir -p {self.model_dir} && cd {self.workdir} && "
            f"{self.python} -m torch.distributed.run --nnodes={self.nnodes} --node-rank={self.node_rank} "
            f"--nproc-per-node={self.gpus_per_node} --master-addr={self.master_addr} "
            f"--master-port={self.master_port} --max-restarts=1 "
            f"jobs/train_ddp.py --data-dir {self.data_dir} --model-dir {self.model_dir} {self.train_args} & "
            f"echo $! > {pidfile}; wait $!; rc=$?; rm -f {pidfile}; exit $rc"
        )
        return self.on(self.trainer, inner)

    def stop_stale_trainer(self) -> str:
        pidfile = f"{self.model_dir}/.trainer.pid"
        inner = (f"if [ -f {pidfile} ]; then pid=$(cat {pidfile}); "
                 f"kill -TERM $pid 2>/dev/null && echo stopped stale trainer $pid; rm -f {pidfile}; fi; true")
        return self.on(self.trainer, inner)

    def verify_checkpoint(self) -> str:
        d = shlex.quote(self.model_dir)
        return self.on(self.trainer, f"ls -lh {d} && test -f {d}/last.ckpt && ls {d}/weather-best-*.ckpt > /dev/null")

    def check_logs(self) -> str:
        d = shlex.quote(self.model_dir)
        return self.on(self.trainer, f"ls {d}/*.ckpt > /dev/null 2>&1 && echo 'training outputs present' || "
                                     "echo 'no training outputs yet (first run)'")

    def cleanup(self, keep: int = 3) -> str:
        d = shlex.quote(self.model_dir)
        return self.on(self.trainer, f"cd {d} 2>/dev/null || exit 0; ls -t weather-best-*.ckpt 2>/dev/null | "
                                     f"tail -n +{keep + 1} | xargs -r rm -f; echo cleanup done")


def _banner(msg: str) -> str:
    return f"echo '================================================================'; echo {shlex.quote(msg)}; date"


def print_training_summary(ds=None, run_id=None, **context):
    """generate_training_report (pipeline.py:17-27): run summary + best checkpoint if visible."""
    lines = ["TRAINING PIPELINE SUMMARY", f"Execution Date: {ds}", f"DAG Run ID: {run_id}",
             "Data Preprocessing: COMPLETED", "Distributed DDP Training (MI355X, RCCL): COMPLETED"]
    md = os.environ.get("DCT_MODEL_DIR")
    if md and os.path.isdir(md):
        best = sorted(f for f in os.listdir(md) if f.startswith("weather-best-"))
        if best:
            lines.append(f"Best checkpoint: {best[-1]}")
    print("\n".join(lines))
    return lines[-1]


def build_pipeline_dag(t: Optional[Targets] = None) -> DAG:
    t = t or Targets()
    with DAG("distributed_data_pipeline", default_args=DEFAULT_ARGS,
             description="Complete pipeline: Spark preprocessing -> MI355X DDP training -> rollout",
             schedule_interval="@daily", start_date=_dt.datetime(2023, 1, 1), catchup=False,
             tags=["spark", "preprocessing", "ddp", "mi355x", "distributed"]) as dag:
        start = BashOperator(task_id="start_pipeline", bash_command=_banner("DISTRIBUTED DATA PIPELINE STARTED"))
        spark_ok = BashOperator(task_id="check_spark_cluster", bash_command=t.spark_health())
        etl = BashOperator(task_id="spark_preprocessing", bash_command=t.etl(),
                           execution_timeout=_dt.timedelta(minutes=30))
        verify = BashOperator(task_id="verify_preprocessing_output", bash_command=t.verify_processed())
        torch_ok = BashOperator(task_id="check_pytorch_cluster", bash_command=t.trainer_health())
        data_ok = BashOperator(task_id="copy_data_to_pytorch_nodes", bash_command=t.data_visible())
        train = BashOperator(task_id="pytorch_lightning_ddp_training", bash_command=t.train(),
                             execution_timeout=_dt.timedelta(hours=3))
        ckpt = BashOperator(task_id="verify_model_checkpoint", bash_command=t.verify_checkpoint())
        logs = BashOperator(task_id="check_tensorboard_logs", bash_command=t.check_logs())
        report = PythonOperator(task_id="generate_training_report", python_callable=print_training_summary)
        cleanup = BashOperator(task_id="cleanup_and_prepare", bash_command=t.cleanup())
        end = BashOperator(task_id="end_pipeline", bash_command=_banner("DISTRIBUTED DATA PIPELINE COMPLETED"))
        trig = TriggerDagRunOperator(task_id="trigger_azure_rollout", trigger_dag_id="azure_automated_rollout",
                                     wait_for_completion=False)
        start >> spark_ok >> etl >> verify >> torch_ok >> data_ok >> train >> ckpt >> logs >> report >> cleanup
        cleanup >> end >> trig
    return dag


def build_spark_etl_dag(t: Optional[Targets] = None) -> DAG:
    t = t or Targets()
    args = {k: v for k, v in DEFAULT_ARGS.items() if k != "email_on_retry"}
    with DAG("spark_etl_pipeline", default_args=args, description="Step 1: Spark Data Preprocessing",
             schedule_interval="@daily", start_date=_dt.datetime(2025, 1, 1), catchup=False,
             tags=["spark", "etl"]) as dag:
        start = BashOperator(task_id="start_etl", bash_command="echo 'SPARK ETL PIPELINE STARTED'")
        ok = BashOperator(task_id="check_spark_cluster", bash_command=t.spark_health())
        etl = BashOperator(task_id="spark_preprocessing", bash_command=t.etl(adaptive=False),
                           execution_timeout=_dt.timedelta(minutes=30))
        verify = BashOperator(task_id="verify_output", bash_command=t.verify_processed())
        trig = TriggerDagRunOperator(task_id="trigger_training_dag", trigger_dag_id="pytorch_training_pipeline",
                                     wait_for_completion=False)
        start >> ok >> etl >> verify >> trig
    return dag


def build_training_dag(t: Optional[Targets] = None) -> DAG:
    t = t or Targets()
    args = {"owner": "airflow", "depends_on_past": False, "retries": 1, "retry_delay": _dt.timedelta(minutes=5)}
    with DAG("pytorch_training_pipeline", default_args=args, description="Step 2: MI355X DDP Training",
             schedule_interval=None, start_date=_dt.datetime(2025, 1, 1), catchup=False,
             tags=["pytorch", "ddp", "training", "mi355x"]) as dag:
        start = BashOperator(task_id="start_training", bash_command="echo 'TRAINING PIPELINE STARTED'")
        zombies = BashOperator(task_id="cleanup_zombies", bash_command=t.stop_stale_trainer())
        gpus = BashOperator(task_id="check_gpu_cluster", bash_command=t.trainer_health())
        train = BashOperator(task_id="pytorch_ddp_training", bash_command=t.train(),
                             execution_timeout=_dt.timedelta(hours=3))
        verify = BashOperator(task_id="verify_model", bash_command=t.verify_checkpoint())
        trig = TriggerDagRunOperator(task_id="trigger_azure_rollout", trigger_dag_id="azure_automated_rollout",
                                     wait_for_completion=False)
        start >> zombies >> gpus >> train >> verify >> trig
    return dag


# ------------------------------------------------------------------------------- deploy tasks
_FAKE_CLIENT = None


def _backend() -> str:
    if os.environ.get("DCT_AZURE_FAKE", "0") == "1":
        return "fake"
    return os.environ.get("DCT_AZURE_BACKEND", "azure").lower()


def get_azure_client():
    """The deployment target of the two deploy DAGs (``DCT_AZURE_BACKEND``):
    ``azure`` (default) - the real MLClient; ``fake`` (or ``DCT_AZURE_FAKE=1``) - an in-memory fake
    for dry runs; ``local`` - the local online endpoint (deploy/local_endpoint.py): the server at
    ``DCT_LOCAL_ENDPOINT_URL`` (key ``DCT_LOCAL_ENDPOINT_KEY``) or, without a URL, in this process."""
    from ..deploy.azure import AzureConfig, FakeMLClient, get_ml_client

    global _FAKE_CLIENT
    backend = _backend()
    if backend in ("fake", "local"):
        if _FAKE_CLIENT is None:
            if backend == "fake":
                _FAKE_CLIENT = FakeMLClient()
            else:
                from ..deploy.local_endpoint import LocalMLClient

                _FAKE_CLIENT = LocalMLClient(os.environ.get("DCT_LOCAL_ENDPOINT_URL") or None,
                                             os.environ.get("DCT_LOCAL_ENDPOINT_KEY") or None)
        return _FAKE_CLIENT
    return get_ml_client(AzureConfig.from_env())


def _health_gate(client, cfg, old: str, new: str, phase: str):
    """Before widening traffic to the new slot: on the local backend probe it (sample request +
    error rate over what it served so far) and roll back to the old slot if it is unhealthy
    (reference D11 only slept between phases)."""
    if _backend() != "local" or new == old:
        return
    from ..deploy.azure import rollback
    from ..deploy.local_endpoint import health_probe

    if not health_probe(client, cfg.endpoint_name)(new):
        rollback(client, cfg, old, new)
        raise RuntimeError(f"deployment {new!r} failed its health check during {phase}; rolled back to {old!r}")


def task_prepare_package(**context):
    from ..deploy.azure import AzureConfig
    from ..deploy.package import prepare_package

    cfg = AzureConfig.from_env()
    info = prepare_package(cfg.deploy_dir, tracking_uri=os.environ.get("MLFLOW_TRACKING_URI", "http://mlflow-server:5000"),
                           norm_stats=os.environ.get("DCT_NORM_STATS"))
    return info["run_id"]


def task_force_deploy(**context):
    from ..deploy.azure import AzureConfig, force_deploy

    return force_deploy(get_azure_client(), AzureConfig.from_env())


def task_deploy_new_slot(ti=None, **context):
    from ..deploy.azure import AzureConfig, deploy_new_slot

    slots = deploy_new_slot(get_azure_client(), AzureConfig.from_env())
    ti.xcom_push(key="new_slot", value=slots["new_slot"])
    ti.xcom_push(key="old_slot", value=slots["old_slot"])
    return slots["new_slot"]


def _slots(ti):
    return (ti.xcom_pull(task_ids="deploy_new_slot", key="old_slot"),
            ti.xcom_pull(task_ids="deploy_new_slot", key="new_slot"))


def task_shadow(ti=None, **context):
    from ..deploy.azure import AzureConfig, start_shadow

    old, new = _slots(ti)
    start_shadow(get_azure_client(), AzureConfig.from_env(), old, new)


def task_canary(ti=None, **context):
    from ..deploy.azure import AzureConfig, start_canary

    old, new = _slots(ti)
    client, cfg = get_azure_client(), AzureConfig.from_env()
    _health_gate(client, cfg, old, new, "shadow")
    start_canary(client, cfg, old, new)


def task_full_rollout(ti=None, **context):
    from ..deploy.azure import AzureConfig, full_rollout

    old, new = _slots(ti)
    client, cfg = get_azure_client(), AzureConfig.from_env()
    _health_gate(client, cfg, old, new, "canary")
    full_rollout(client, cfg, old, new)


def build_manual_deploy_dag() -> DAG:
    with DAG("azure_manual_deploy", start_date=_dt.datetime(2025, 1, 1), schedule_interval=None,
             tags=["azure", "manual"]) as dag:
        t1 = PythonOperator(task_id="prepare_package", python_callable=task_prepare_package)
        t2 = PythonOperator(task_id="force_deploy_100", python_callable=task_force_deploy,
                            execution_timeout=_dt.timedelta(minutes=40))
        t1 >> t2
    return dag


def build_rollout_dag() -> DAG:
    wait = os.environ.get("DCT_ROLLOUT_WAIT_S", "30")
    with DAG("azure_automated_rollout", start_date=_dt.datetime(2025, 1, 1), schedule_interval=None,
             tags=["azure", "auto"]) as dag:
        t1 = PythonOperator(task_id="prepare_package", python_callable=task_prepare_package)
        t2 = PythonOperator(task_id="deploy_new_slot", python_callable=task_deploy_new_slot,
                            execution_timeout=_dt.timedelta(minutes=40))
        t3 = PythonOperator(task_id="shadow_traffic", python_callable=task_shadow)
        t4 = BashOperator(task_id="wait_shadow", bash_command=f"sleep {shlex.quote(wait)}")
        t5 = PythonOperator(task_id="canary_traffic", python_callable=task_canary)
        t6 = BashOperator(task_id="wait_canary", bash_command=f"sleep {shlex.quote(wait)}")
        t7 = PythonOperator(task_id="full_rollout", python_callable=task_full_rollout)
        t1 >> t2 >> t3 >> t4 >> t5 >> t6 >> t7
    return dag


def build_all(t: Optional[Targets] = None) -> Dict[str, DAG]:
    t = t or Targets()
    dags = [build_pipeline_dag(t), build_spark_etl_dag(t), build_training_dag(t), build_manual_deploy_dag(),
            build_rollout_dag()]
    return {d.dag_id: d for d in dags}
