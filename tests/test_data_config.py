"""Config, ETL semantics, dataset contract, split/sharding parity (CPU)."""
import math
import os

import numpy as np
import pandas as pd
import pytest
import torch

import dct_amd  # noqa: F401
from dct_amd.config import FEATURE_COLUMNS, PipelineConfig, default_config
from dct_amd.data.dataset import WeatherDataset
from dct_amd.data.etl import column_stats, normalize_frame, run_arrow_etl, write_parquet_dir
from dct_amd.data.sampler import distributed_indices, seeded_random_split
from dct_amd.data.synthetic import make_processed_parquet, make_weather_csv


def test_config_defaults_equal_reference_constants():
    c = PipelineConfig()
    assert c.data.batch_size == 4 and c.optim.lr == 0.01 and c.train.max_epochs == 10
    assert c.data.train_fraction == 0.8 and c.train.seed == 42 and c.train.log_every_n_steps == 5
    assert tuple(c.model.hidden) == (64,) and c.model.dropout == 0.2
    assert c.ckpt.filename == "weather-best-{epoch:02d}-{val_loss:.2f}" and c.ckpt.save_last
    assert c.tracking.experiment_name == "weather_forecasting"
    assert c.tracking.tracking_uri == "http://mlflow-server:5000"


def test_config_env_overrides_reference_names():
    c = default_config({"WORLD_SIZE": "2", "NODE_RANK": "1", "MASTER_ADDR": "pytorch-master", "MASTER_PORT": "29500",
                        "MLFLOW_TRACKING_URI": "file:/tmp/x", "DCT_BATCH_SIZE": "8", "DCT_HIDDEN": "128,128"})
    assert c.dist.world_size == 2 and c.dist.rank == 1 and c.dist.master_addr == "pytorch-master"
    assert c.tracking.tracking_uri == "file:/tmp/x" and c.data.batch_size == 8
    assert tuple(c.model.hidden) == (128, 128)


def test_config_roundtrip_yaml(tmp_path):
    import yaml

    p = tmp_path / "c.yaml"
    p.write_text(yaml.safe_dump({"train": {"max_epochs": 3}, "data": {"batch_size": 16}}))
    c = PipelineConfig.load(str(p))
    assert c.train.max_epochs == 3 and c.data.batch_size == 16
    with pytest.raises(KeyError):
        PipelineConfig.from_dict({"train": {"nope": 1}})


def test_column_stats_sample_std_and_nulls():
    v = np.array([1.0, 2.0, 3.0, np.nan])
    mean, std = column_stats(v)
    assert mean == 2.0 and abs(std - 1.0) < 1e-12  # ddof=1 like Spark stddev_samp
    assert column_stats(np.array([5.0])) == (5.0, None)
    assert column_stats(np.array([np.nan])) == (None, None)


def test_normalize_frame_reference_semantics():
    df = pd.DataFrame({
        "Temperature": [10.0, 20.0, 30.0, None],
        "Humidity": [50.0, 50.0, 50.0, 50.0],  # std == 0 -> divide by 1.0
        "Wind_Speed": [1, 2, 3, 4],
        "Cloud_Cover": [0.0, 10.0, 20.0, 30.0],
        "Pressure": [1000.0, 1010.0, 1020.0, 1030.0],
        "Rain": ["rain", "no rain", None, "rain"],
    })
    out, stats = normalize_frame(df)
    assert list(out.columns) == [f"{c}_norm" for c in FEATURE_COLUMNS] + ["label_encoded"]
    assert out["label_encoded"].tolist() == [1, 0, 0, 1]
    assert out["label_encoded"].dtype == np.int32
    t = out["Temperature_norm"].to_numpy()
    assert np.allclose(t[:3], [-1.0, 0.0, 1.0]) and np.isnan(t[3])
    assert np.allclose(out["Humidity_norm"], 0.0)
    w = out["Wind_Speed_norm"].to_numpy()
    assert np.isclose(w.mean(), 0) and np.isclose(w.std(ddof=1), 1.0)


def test_arrow_etl_writes_spark_style_dir(tmp_path):
    raw = make_weather_csv(str(tmp_path / "raw" / "weather.csv"), n=300)
    out = str(tmp_path / "processed" / "data.parquet")
    os.makedirs(out)
    open(os.path.join(out, "stale.parquet"), "w").write("garbage")  # overwrite semantics
    stats = run_arrow_etl(raw, out, verbose=False)
    files = os.listdir(out)
    assert "_SUCCESS" in files and "stale.parquet" not in files
    assert any(f.startswith("part-00000-") and f.endswith(".snappy.parquet") for f in files)
    ds = WeatherDataset(str(tmp_path / "processed"), verbose=False)
    assert ds.features.shape == (300, 5) and ds.features.dtype == torch.float32
    assert ds.labels.dtype == torch.int64 and set(ds.labels.unique().tolist()) <= {0, 1}
    assert ds.feature_cols == [f"{c}_norm" for c in FEATURE_COLUMNS]
    x, y = ds[3]
    assert x.shape == (5,) and y.dim() == 0
    assert set(stats) == set(FEATURE_COLUMNS)


def test_dataset_error_contract(tmp_path):
    with pytest.raises(FileNotFoundError, match="Did the Spark preprocessing step finish"):
        WeatherDataset(str(tmp_path))
    d = tmp_path / "bad"
    (d / "data.parquet").mkdir(parents=True)
    (d / "data.parquet" / "part-0.parquet").write_text("not parquet")
    with pytest.raises(RuntimeError, match="Failed to read Parquet file"):
        WeatherDataset(str(d), verbose=False)
    d2 = tmp_path / "nonorm"
    write_parquet_dir(pd.DataFrame({"a": [1.0], "label_encoded": [1]}), str(d2 / "data.parquet"))
    with pytest.raises(ValueError, match="No columns ending with '_norm'"):
        WeatherDataset(str(d2), verbose=False)


def test_processed_parquet_multi_part(tmp_path):
    make_processed_parquet(str(tmp_path), n=1001, num_parts=3)
    ds = WeatherDataset(str(tmp_path), verbose=False)
    assert len(ds) == 1001


def test_random_split_parity_with_torch():
    from torch.utils.data import TensorDataset, random_split

    n = 1003
    torch.manual_seed(42)
    tr, va = random_split(TensorDataset(torch.arange(n)), [int(0.8 * n), n - int(0.8 * n)])
    a, b = seeded_random_split(n, 0.8, 42)
    assert a.tolist() == list(tr.indices) and b.tolist() == list(va.indices)


@pytest.mark.parametrize("n,world", [(100, 1), (101, 2), (7, 4), (3, 8), (1000, 3)])
@pytest.mark.parametrize("shuffle", [True, False])
def test_distributed_indices_match_torch_sampler(n, world, shuffle):
    from torch.utils.data.distributed import DistributedSampler

    for epoch in (0, 3):
        for rank in range(world):
            s = DistributedSampler(range(n), num_replicas=world, rank=rank, shuffle=shuffle, seed=42)
            s.set_epoch(epoch)
            want = list(iter(s))
            got = distributed_indices(n, world, rank, shuffle=shuffle, seed=42, epoch=epoch).tolist()
            assert got == want
