"""Reference-named ETL entry point (reference: jobs/preprocess.py, run as
``spark-submit /opt/spark/jobs/preprocess.py`` with no arguments, dags/pipeline.py:73-79).

Same defaults as the reference (``/opt/spark/data/raw/weather.csv`` ->
``/opt/spark/data/processed/data.parquet``); the engine is picked automatically (Spark when
pyspark is importable, else the Arrow engine with identical semantics).  All logic lives in
``jobs/etl_job.py``; extra flags are forwarded.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from etl_job import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
