"""ETL: raw weather CSV -> label-encoded, z-scored Parquet dataset.

Contract (reference ``jobs/preprocess.py``):
  * read CSV with a header and inferred schema (:18);
  * ``label_encoded = 1 if Rain == "rain" else 0`` (null Rain -> 0, Spark ``when`` semantics) (:23-25);
  * for each of the 5 features: z-score with the column mean and the **sample** standard
    deviation (Spark ``stddev`` = ``stddev_samp``), std == 0 -> 1.0 (:32-41);
    nulls are ignored by the aggregates and stay null in the output; a column with fewer
    than two non-null values has a null stddev -> the normalised column is all null;
  * write ``<f>_norm`` x5 (double) + ``label_encoded`` (int32) as a Parquet *directory* with
    overwrite semantics (:48-51).

Two engines implement it:
  * ``spark``  - the orchestrated engine on the Spark cluster (``jobs/preprocess.py``).  All five
    (mean, stddev) pairs come from ONE aggregation job instead of one job per feature.
  * ``arrow``  - a single-node pyarrow/pandas implementation with identical semantics, used on the
    training node, in tests (pyspark is not installable offline) and for large synthetic sets.
"""
from __future__ import annotations

import os
import shutil
import uuid
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from ..config import FEATURE_COLUMNS, LABEL_COLUMN, LABEL_SOURCE_COLUMN, NORM_SUFFIX


def column_stats(values: np.ndarray) -> Tuple[Optional[float], Optional[float]]:
    """(mean, sample std) ignoring NaN, Spark null semantics (None when undefined)."""
    v = values[~np.isnan(values)]
    if v.size == 0:
        return None, None
    mean = float(v.mean())
    if v.size < 2:
        return mean, None
    return mean, float(v.std(ddof=1))


def normalize_frame(df, feature_cols: Sequence[str] = FEATURE_COLUMNS):
    """Apply the reference transformation to a pandas DataFrame; returns (out_df, stats)."""
    import pandas as pd

    missing = [c for c in list(feature_cols) + [LABEL_SOURCE_COLUMN] if c not in df.columns]
    if missing:
        raise ValueError(f"input is missing required columns: {missing}")
    out = {}
    stats: Dict[str, Dict[str, Optional[float]]] = {}
    for c in feature_cols:
        col = pd.to_numeric(df[c], errors="coerce").to_numpy(dtype=np.float64)
        mean, std = column_stats(col)
        stats[c] = {"mean": mean, "std": std}
        if mean is None or std is None:
            out[f"{c}{NORM_SUFFIX}"] = np.full(len(col), np.nan)
            continue
        std_val = std if std != 0 else 1.0  # preprocess.py:36
        out[f"{c}{NORM_SUFFIX}"] = (col - mean) / std_val
    rain = df[LABEL_SOURCE_COLUMN]
    label = (rain == "rain").fillna(False).to_numpy().astype(np.int32)
    out[LABEL_COLUMN] = label
    cols = [f"{c}{NORM_SUFFIX}" for c in feature_cols] + [LABEL_COLUMN]
    return pd.DataFrame(out, columns=cols), stats


def write_parquet_dir(df, output_path: str, num_parts: int = 1) -> List[str]:
    """Write a Spark-style Parquet directory (part files + _SUCCESS), overwrite mode."""
    import pyarrow as pa
    import pyarrow.parquet as pq

    if os.path.isdir(output_path):
        shutil.rmtree(output_path)
    elif os.path.exists(output_path):
        os.remove(output_path)
    os.makedirs(output_path, exist_ok=True)
    job = uuid.uuid4()
    n = len(df)
    num_parts = max(1, min(num_parts, n)) if n else 1
    bounds = np.linspace(0, n, num_parts + 1).astype(np.int64)
    paths = []
    for i in range(num_parts):
        part = df.iloc[bounds[i] : bounds[i + 1]]
        table = pa.Table.from_pandas(part, preserve_index=False)
        p = os.path.join(output_path, f"part-{i:05d}-{job}-c000.snappy.parquet")
        pq.write_table(table, p, compression="snappy")
        paths.append(p)
    open(os.path.join(output_path, "_SUCCESS"), "w").close()
    return paths


def run_arrow_etl(raw_csv: str, output_path: str, feature_cols: Sequence[str] = FEATURE_COLUMNS,
                  num_parts: int = 1, verbose: bool = True):
    """Single-node ETL with the Spark job's semantics. Returns the per-feature stats."""
    import pandas as pd

    if verbose:
        print("=" * 80)
        print("Weather data preprocessing (arrow engine)")
        print("=" * 80)
        print(f"Reading data from: {raw_csv}")
    df = pd.read_csv(raw_csv)
    if verbose:
        print(df.head(20).to_string())
        print("Encoding target variable 'Rain'...")
        print("Normalizing features...")
    out, stats = normalize_frame(df, feature_cols)
    if verbose:
        print(f"Saving processed data to: {output_path}")
    write_parquet_dir(out, output_path, num_parts=num_parts)
    # Persist the normalisation statistics next to the data (fixes the reference's train/serve
    # skew D7: stats were computed and thrown away).
    import json

    with open(os.path.join(output_path, "_norm_stats.json"), "w") as f:
        json.dump(stats, f, indent=1)
    if verbose:
        print("Preprocessing complete")
    return stats


def spark_etl(spark, raw_csv: str, output_path: str, feature_cols: Sequence[str] = FEATURE_COLUMNS):
    """Spark engine: one aggregation job for all feature stats (pyspark must be importable)."""
    from pyspark.sql import functions as F

    df = spark.read.csv(raw_csv, header=True, inferSchema=True)
    df.show()
    df = df.withColumn(LABEL_COLUMN, F.when(F.col(LABEL_SOURCE_COLUMN) == "rain", 1).otherwise(0))
    aggs = []
    for c in feature_cols:
        aggs += [F.mean(F.col(c)).alias(f"{c}__mean"), F.stddev(F.col(c)).alias(f"{c}__std")]
    row = df.agg(*aggs).first()
    stats = {}
    for c in feature_cols:
        mean, std = row[f"{c}__mean"], row[f"{c}__std"]
        stats[c] = {"mean": mean, "std": std}
        std_val = std if std != 0 else 1.0
        df = df.withColumn(f"{c}{NORM_SUFFIX}", (F.col(c) - F.lit(mean)) / F.lit(std_val))
    final_cols = [f"{c}{NORM_SUFFIX}" for c in feature_cols] + [LABEL_COLUMN]
    df.select(final_cols).write.mode("overwrite").parquet(output_path)
    return stats
