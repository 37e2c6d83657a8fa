"""Synthetic data generators (no network: datasets cannot be downloaded).

* ``make_weather_csv``     - a raw ``weather.csv`` with the reference's columns
  (Temperature, Humidity, Wind_Speed, Cloud_Cover, Pressure, Rain) and a learnable rain rule,
  the input of the ETL stage (README.md:66-69).
* ``make_processed_parquet`` - skip the ETL: write ``<f>_norm`` + ``label_encoded`` directly.
* ``make_tabular_device``  - the BASELINE.json large config (rows x 256 features) generated
  directly in HBM (100M x 256 bf16 = 51 GB fits the 288 GB of one MI355X).
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import numpy as np

from ..config import FEATURE_COLUMNS, LABEL_COLUMN, NORM_SUFFIX


def _weather_arrays(n: int, seed: int):
    rng = np.random.default_rng(seed)
    temp = rng.normal(18.0, 8.0, n)
    hum = np.clip(rng.normal(65.0, 18.0, n), 5, 100)
    wind = np.abs(rng.normal(12.0, 6.0, n))
    cloud = np.clip(rng.normal(50.0, 28.0, n), 0, 100)
    press = rng.normal(1013.0, 9.0, n)
    logit = 0.06 * (hum - 65) + 0.05 * (cloud - 50) - 0.12 * (press - 1013) - 0.04 * (temp - 18)
    p = 1.0 / (1.0 + np.exp(-logit))
    rain = rng.random(n) < p
    return temp, hum, wind, cloud, press, rain


def make_weather_csv(path: str, n: int = 2000, seed: int = 0) -> str:
    import pandas as pd

    temp, hum, wind, cloud, press, rain = _weather_arrays(n, seed)
    df = pd.DataFrame({
        "Temperature": temp, "Humidity": hum, "Wind_Speed": wind,
        "Cloud_Cover": cloud, "Pressure": press,
        "Rain": np.where(rain, "rain", "no rain"),
    })
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    df.to_csv(path, index=False)
    return path


def make_processed_parquet(data_dir: str, n: int = 2000, seed: int = 0, num_parts: int = 2) -> str:
    """Write ``<data_dir>/data.parquet/`` exactly as the ETL would produce it."""
    import pandas as pd

    from .etl import normalize_frame, write_parquet_dir

    temp, hum, wind, cloud, press, rain = _weather_arrays(n, seed)
    raw = pd.DataFrame({
        "Temperature": temp, "Humidity": hum, "Wind_Speed": wind,
        "Cloud_Cover": cloud, "Pressure": press,
        "Rain": np.where(rain, "rain", "no rain"),
    })
    out, _ = normalize_frame(raw)
    path = os.path.join(data_dir, "data.parquet")
    write_parquet_dir(out, path, num_parts=num_parts)
    return path


def weather_tensors(n: int, seed: int = 0, dim: int = 5):
    """(features fp32 [n, dim], labels int64 [n]) in the processed (z-scored) space."""
    import torch

    temp, hum, wind, cloud, press, rain = _weather_arrays(n, seed)
    x = np.stack([temp, hum, wind, cloud, press], 1)
    x = (x - x.mean(0)) / x.std(0, ddof=1)
    if dim != 5:
        rng = np.random.default_rng(seed + 1)
        extra = rng.standard_normal((n, max(0, dim - 5)))
        x = np.concatenate([x, extra], 1)[:, :dim]
    return torch.from_numpy(x.astype(np.float32)), torch.from_numpy(rain.astype(np.int64))


def make_tabular_device(rows: int, feats: int, num_classes: int = 2, device="cuda", dtype=None,
                        seed: int = 0, chunk: int = 1 << 22):
    """Large synthetic tabular set generated in place on the device (chunked, no host copy).

    Chunks stay below 2^31 fp32 elements per GEMV (hipBLAS fails on larger operands)."""
    import torch

    dtype = dtype or torch.bfloat16
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    x = torch.empty(rows, feats, device=device, dtype=dtype)
    y = torch.empty(rows, device=device, dtype=torch.int32)
    w = torch.randn(feats, generator=g, device=device, dtype=torch.float32)
    for s in range(0, rows, chunk):
        e = min(rows, s + chunk)
        blk = torch.randn(e - s, feats, generator=g, device=device, dtype=torch.float32)
        x[s:e] = blk.to(dtype)
        y[s:e] = ((blk @ w) > 0).to(torch.int32) % num_classes
    return x, y
