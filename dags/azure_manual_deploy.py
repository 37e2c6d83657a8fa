"""Airflow DAG file for ``azure_manual_deploy`` (reference: dags/azure_manual_deploy.py): prepare_package -> force_deploy_100.

Mount the repository at ``/workspace`` and point ``AIRFLOW__CORE__DAGS_FOLDER`` at this directory
(docker/compose.yaml).  The DAG itself is built by ``dct_amd.orchestration.dags.build_manual_deploy_dag``; this
file only exposes it at module level, which is how Airflow discovers DAGs.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import dct_amd  # noqa: E402,F401
from dct_amd.orchestration.dags import build_manual_deploy_dag  # noqa: E402

dag = build_manual_deploy_dag()
