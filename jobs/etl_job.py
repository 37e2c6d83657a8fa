"""Weather ETL job: raw CSV -> ``data.parquet`` directory (reference: jobs/preprocess.py:5-55).

Engines (``--engine``):
  * ``spark`` - submitted with ``spark-submit`` on the Spark cluster; one aggregation job for all
    feature statistics (``dct_amd.data.etl.spark_etl``);
  * ``arrow`` - single-node pyarrow/pandas with the same semantics (used on the training node, in
    tests, and wherever pyspark is not installed);
  * ``auto``  - spark if pyspark imports, else arrow.
Both write ``_norm_stats.json`` next to the part files so serving can normalise raw requests.

    spark-submit --master spark://spark-master:7077 jobs/etl_job.py --engine spark
    python jobs/etl_job.py --engine arrow --input raw/weather.csv --output processed/data.parquet
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import dct_amd  # noqa: E402,F401
from dct_amd.data.etl import run_arrow_etl, spark_etl  # noqa: E402


def _have_pyspark() -> bool:
    try:
        import pyspark  # noqa: F401

        return True
    except Exception:  # noqa: BLE001
        return False


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description="weather ETL")
    p.add_argument("--input", default="/opt/spark/data/raw/weather.csv")
    p.add_argument("--output", default="/opt/spark/data/processed/data.parquet")
    p.add_argument("--engine", choices=("spark", "arrow", "auto"), default="auto")
    p.add_argument("--num-parts", type=int, default=1, help="arrow engine: part files to write")
    a = p.parse_args(argv)
    engine = a.engine
    if engine == "auto":
        engine = "spark" if _have_pyspark() else "arrow"
    print("=" * 80)
    print(f"Weather preprocessing ({engine} engine): {a.input} -> {a.output}")
    print("=" * 80)
    if not os.path.exists(a.input):
        print(f"input not found: {a.input}", file=sys.stderr)
        return 2
    if engine == "spark":
        from pyspark.sql import SparkSession

        spark = SparkSession.builder.appName("WeatherPreprocessing").getOrCreate()
        try:
            stats = spark_etl(spark, a.input, a.output)
        finally:
            spark.stop()
        with open(os.path.join(a.output, "_norm_stats.json"), "w") as f:
            json.dump(stats, f, indent=1)
    else:
        run_arrow_etl(a.input, a.output, num_parts=a.num_parts)
    print("Preprocessing complete")
    return 0


if __name__ == "__main__":
    sys.exit(main())
