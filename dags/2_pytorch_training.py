"""Airflow DAG file for ``pytorch_training_pipeline`` (reference: dags/2_pytorch_training.py): stale-trainer cleanup -> cluster check -> torchrun DDP training -> verify -> rollout trigger.

Mount the repository at ``/workspace`` and point ``AIRFLOW__CORE__DAGS_FOLDER`` at this directory
(docker/compose.yaml).  The DAG itself is built by ``dct_amd.orchestration.dags.build_training_dag``; this
file only exposes it at module level, which is how Airflow discovers DAGs.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import dct_amd  # noqa: E402,F401
from dct_amd.orchestration.dags import build_training_dag  # noqa: E402

dag = build_training_dag()
