"""Airflow DAG-folder entry point: registers the five pipeline DAGs.

Mount the repository at ``/workspace`` on the Airflow scheduler/webserver and point
``AIRFLOW__CORE__DAGS_FOLDER`` at this directory (see docker/compose.yaml).  All logic lives in
``dct_amd.orchestration.dags``; this file only exposes the DAG objects at module level, which is
how Airflow discovers them.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import dct_amd  # noqa: E402,F401
from dct_amd.orchestration.dags import build_all  # noqa: E402

for _dag_id, _dag in build_all().items():
    globals()[_dag_id] = _dag
