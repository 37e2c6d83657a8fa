"""Airflow DAG file for ``spark_etl_pipeline`` (reference: dags/1_spark_etl.py): daily Spark ETL, then triggers pytorch_training_pipeline.

Mount the repository at ``/workspace`` and point ``AIRFLOW__CORE__DAGS_FOLDER`` at this directory
(docker/compose.yaml).  The DAG itself is built by ``dct_amd.orchestration.dags.build_spark_etl_dag``; this
file only exposes it at module level, which is how Airflow discovers DAGs.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import dct_amd  # noqa: E402,F401
from dct_amd.orchestration.dags import build_spark_etl_dag  # noqa: E402

dag = build_spark_etl_dag()
