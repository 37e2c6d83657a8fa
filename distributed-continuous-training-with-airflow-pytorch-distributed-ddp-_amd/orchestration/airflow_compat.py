"""Airflow 2.x compatibility layer + a local DAG executor.

When ``apache-airflow`` is importable the real ``DAG``/``BashOperator``/``PythonOperator``/
``TriggerDagRunOperator`` are re-exported and the DAG definitions in ``orchestration.dags`` are
ordinary Airflow DAGs (the reference deploys them to an Airflow 2.7.1 LocalExecutor,
docker-compose.yml:193-230).  Without Airflow (this image, CI, an air-gapped trainer node)
minimal stand-ins with the same constructor arguments and ``>>`` dependency syntax are used,
and :class:`LocalDagRunner` executes a DAG run in topological order with the operator
semantics the reference relies on: ``retries``/``retry_delay`` from ``default_args``,
``execution_timeout``, bash exit codes, XCom push/pull, Jinja-free context (``ds``, ``run_id``,
``ti``, ``dag_run.conf``) and fire-and-forget ``TriggerDagRunOperator`` (optionally executed
inline, so a full ETL -> train -> deploy chain can be run end to end without a scheduler).
"""
from __future__ import annotations

import datetime as _dt
import os
import subprocess
import time
import traceback
import uuid
from typing import Any, Callable, Dict, Iterable, List, Optional

try:  # pragma: no cover - exercised only where Airflow is installed
    from airflow import DAG  # type: ignore
    from airflow.operators.bash import BashOperator  # type: ignore
    from airflow.operators.python import PythonOperator  # type: ignore
    from airflow.operators.trigger_dagrun import TriggerDagRunOperator  # type: ignore

    HAVE_AIRFLOW = True
except Exception:  # noqa: BLE001
    HAVE_AIRFLOW = False

_CURRENT_DAG: List["DAG"] = []
DAG_REGISTRY: Dict[str, "DAG"] = {}

if not HAVE_AIRFLOW:

    class DAG:  # type: ignore[no-redef]
        def __init__(self, dag_id: str, default_args: Optional[Dict[str, Any]] = None, description: str = "",
                     schedule_interval: Any = None, schedule: Any = None, start_date: Optional[_dt.datetime] = None,
                     catchup: bool = True, tags: Optional[List[str]] = None, max_active_runs: int = 16, **kwargs):
            self.dag_id = dag_id
            self.default_args = dict(default_args or {})
            self.description = description
            self.schedule_interval = schedule_interval if schedule is None else schedule
            self.start_date = start_date
            self.catchup = catchup
            self.tags = list(tags or [])
            self.max_active_runs = max_active_runs
            self.task_dict: Dict[str, "BaseOperator"] = {}
            DAG_REGISTRY[dag_id] = self

        def __enter__(self):
            _CURRENT_DAG.append(self)
            return self

        def __exit__(self, *exc):
            _CURRENT_DAG.pop()
            return False

        @property
        def tasks(self) -> List["BaseOperator"]:
            return list(self.task_dict.values())

        @property
        def task_ids(self) -> List[str]:
            return list(self.task_dict)

        def get_task(self, task_id: str) -> "BaseOperator":
            return self.task_dict[task_id]

        def topological_sort(self) -> List["BaseOperator"]:
            indeg = {t: len(op.upstream_task_ids) for t, op in self.task_dict.items()}
            ready = [t for t in self.task_dict if indeg[t] == 0]
            order = []
            while ready:
                t = ready.pop(0)
                order.append(self.task_dict[t])
                for d in sorted(self.task_dict[t].downstream_task_ids):
                    indeg[d] -= 1
                    if indeg[d] == 0:
                        ready.append(d)
            if len(order) != len(self.task_dict):
                raise ValueError(f"DAG {self.dag_id} has a cycle")
            return order

    class BaseOperator:
        def __init__(self, task_id: str, dag: Optional[DAG] = None, retries: Optional[int] = None,
                     retry_delay: Optional[_dt.timedelta] = None, execution_timeout: Optional[_dt.timedelta] = None,
                     trigger_rule: str = "all_success", **kwargs):
            self.task_id = task_id
            self.dag = dag or (_CURRENT_DAG[-1] if _CURRENT_DAG else None)
            if self.dag is None:
                raise RuntimeError(f"operator {task_id} created outside a DAG")
            da = self.dag.default_args
            self.retries = da.get("retries", 0) if retries is None else retries
            self.retry_delay = da.get("retry_delay", _dt.timedelta(minutes=5)) if retry_delay is None else retry_delay
            self.execution_timeout = execution_timeout or da.get("execution_timeout")
            self.trigger_rule = trigger_rule
            self.owner = da.get("owner", "airflow")
            self.upstream_task_ids: set = set()
            self.downstream_task_ids: set = set()
            self.extra = kwargs
            if task_id in self.dag.task_dict:
                raise ValueError(f"duplicate task_id {task_id}")
            self.dag.task_dict[task_id] = self

        def set_downstream(self, other):
            for o in (other if isinstance(other, (list, tuple)) else [other]):
                self.downstream_task_ids.add(o.task_id)
                o.upstream_task_ids.add(self.task_id)

        def __rshift__(self, other):
            self.set_downstream(other)
            return other

        def __lshift__(self, other):
            for o in (other if isinstance(other, (list, tuple)) else [other]):
                o.set_downstream(self)
            return other

        def __rrshift__(self, other):
            for o in (other if isinstance(other, (list, tuple)) else [other]):
                o.set_downstream(self)
            return self

        def execute(self, context: Dict[str, Any]):  # pragma: no cover - abstract
            raise NotImplementedError

    class BashOperator(BaseOperator):  # type: ignore[no-redef]
        def __init__(self, task_id: str, bash_command: str, env: Optional[Dict[str, str]] = None,
                     append_env: bool = True, **kwargs):
            super().__init__(task_id, **kwargs)
            self.bash_command = bash_command
            self.env = env
            self.append_env = append_env

        def execute(self, context):
            env = dict(os.environ) if (self.append_env or self.env is None) else {}
            env.update(self.env or {})
            timeout = self.execution_timeout.total_seconds() if self.execution_timeout else None
            r = subprocess.run(["bash", "-c", self.bash_command], env=env, capture_output=True, text=True,
                               timeout=timeout)
            context["log"].append(r.stdout + r.stderr)
            if r.returncode != 0:
                raise RuntimeError(f"Bash command failed with exit code {r.returncode}:\n{r.stdout[-2000:]}"
                                   f"{r.stderr[-2000:]}")
            lines = [l for l in r.stdout.splitlines() if l.strip()]
            return lines[-1] if lines else None

    class PythonOperator(BaseOperator):  # type: ignore[no-redef]
        def __init__(self, task_id: str, python_callable: Callable, op_args: Optional[Iterable] = None,
                     op_kwargs: Optional[Dict[str, Any]] = None, provide_context: bool = False, **kwargs):
            super().__init__(task_id, **kwargs)
            self.python_callable = python_callable
            self.op_args = list(op_args or [])
            self.op_kwargs = dict(op_kwargs or {})

        def execute(self, context):
            import inspect

            sig = inspect.signature(self.python_callable)
            kw = dict(self.op_kwargs)
            if any(p.kind == p.VAR_KEYWORD for p in sig.parameters.values()):
                kw.update({k: v for k, v in context.items() if k != "log"})
            else:
                kw.update({k: v for k, v in context.items() if k in sig.parameters})
            return self.python_callable(*self.op_args, **kw)

    class TriggerDagRunOperator(BaseOperator):  # type: ignore[no-redef]
        def __init__(self, task_id: str, trigger_dag_id: str, wait_for_completion: bool = False,
                     conf: Optional[Dict[str, Any]] = None, **kwargs):
            super().__init__(task_id, **kwargs)
            self.trigger_dag_id = trigger_dag_id
            self.wait_for_completion = wait_for_completion
            self.conf = conf

        def execute(self, context):
            runner = context.get("runner")
            if runner is not None:
                runner.triggered.append(self.trigger_dag_id)
                if runner.follow_triggers:
                    if self.trigger_dag_id not in DAG_REGISTRY:
                        raise RuntimeError(f"DagRun trigger to unknown DAG {self.trigger_dag_id!r}")
                    res = runner.run(DAG_REGISTRY[self.trigger_dag_id], conf=self.conf)
                    if self.wait_for_completion and res.state != "success":
                        raise RuntimeError(f"triggered DAG {self.trigger_dag_id} failed")
            return self.trigger_dag_id


class TaskInstance:
    def __init__(self, task_id: str, xcom: Dict):
        self.task_id = task_id
        self._xcom = xcom
        self.try_number = 1

    def xcom_push(self, key: str, value: Any):
        self._xcom[(self.task_id, key)] = value

    def xcom_pull(self, task_ids: Optional[str] = None, key: str = "return_value"):
        return self._xcom.get((task_ids or self.task_id, key))


class DagRunResult:
    def __init__(self, dag_id: str, run_id: str):
        self.dag_id = dag_id
        self.run_id = run_id
        self.state = "running"
        self.task_states: Dict[str, str] = {}
        self.tries: Dict[str, int] = {}
        self.logs: Dict[str, List[str]] = {}
        self.xcom: Dict = {}
        self.errors: Dict[str, str] = {}


class LocalDagRunner:
    """Executes DAG runs in-process (no scheduler, no database)."""

    def __init__(self, follow_triggers: bool = False, retry_delay_scale: float = 1.0,
                 sleep: Callable[[float], None] = time.sleep):
        self.follow_triggers = follow_triggers
        self.retry_delay_scale = retry_delay_scale
        self.sleep = sleep
        self.triggered: List[str] = []
        self.results: List[DagRunResult] = []

    def run(self, dag, execution_date: Optional[_dt.datetime] = None, conf: Optional[Dict] = None) -> DagRunResult:
        execution_date = execution_date or _dt.datetime.now()
        res = DagRunResult(dag.dag_id, f"manual__{execution_date.isoformat()}_{uuid.uuid4().hex[:6]}")
        self.results.append(res)
        failed = False
        for op in dag.topological_sort():
            ups = [res.task_states.get(u) for u in op.upstream_task_ids]
            if failed or any(s != "success" for s in ups):
                if op.trigger_rule == "all_done" and all(s is not None for s in ups):
                    pass
                else:
                    res.task_states[op.task_id] = "upstream_failed"
                    continue
            ti = TaskInstance(op.task_id, res.xcom)
            log: List[str] = []
            context = {"ds": execution_date.strftime("%Y-%m-%d"), "ts": execution_date.isoformat(),
                       "run_id": res.run_id, "execution_date": execution_date, "ti": ti, "task_instance": ti,
                       "dag": dag, "task": op, "params": {}, "dag_run": _DagRunConf(conf or {}),
                       "runner": self, "log": log}
            attempt = 0
            while True:
                attempt += 1
                ti.try_number = attempt
                try:
                    out = op.execute(context)
                    if out is not None:
                        ti.xcom_push("return_value", out)
                    res.task_states[op.task_id] = "success"
                    break
                except Exception as e:  # noqa: BLE001
                    res.errors[op.task_id] = "".join(traceback.format_exception_only(type(e), e))
                    if attempt > op.retries:
                        res.task_states[op.task_id] = "failed"
                        failed = True
                        break
                    res.task_states[op.task_id] = "up_for_retry"
                    self.sleep(op.retry_delay.total_seconds() * self.retry_delay_scale)
            res.tries[op.task_id] = attempt
            res.logs[op.task_id] = log
        res.state = "failed" if failed else "success"
        return res


class _DagRunConf:
    def __init__(self, conf):
        self.conf = conf
