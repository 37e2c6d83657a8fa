"""Property tests (hypothesis) for the CPU-side contracts: sharding, split, ETL semantics, ckpt layout.

SURVEY §4 tier 1/2: the reference relies on torch's DistributedSampler / random_split
(jobs/train_lightning_ddp.py:117-123, implicit sampler swap via DDPStrategy :136) and on Spark's
z-score with sample stddev and the std==0 guard (jobs/preprocess.py:32-41).  The example-based
tests pin fixed shapes; these draw them.  ``derandomize=True`` keeps every run identical.
"""
import math

import numpy as np
import pytest
import torch
from hypothesis import given, settings
from hypothesis import strategies as st

import dct_amd  # noqa: F401
from dct_amd.data.etl import column_stats, normalize_frame
from dct_amd.data.sampler import batches, distributed_indices, num_batches, seeded_random_split

SETTINGS = settings(max_examples=60, deadline=None, derandomize=True)


@SETTINGS
@given(n=st.integers(1, 400), world=st.integers(1, 8), shuffle=st.booleans(), drop_last=st.booleans(),
       epoch=st.integers(0, 5))
def test_distributed_indices_equal_torch_sampler(n, world, shuffle, drop_last, epoch):
    from torch.utils.data.distributed import DistributedSampler

    if drop_last and n < world:
        return  # torch yields empty shards here; nothing to compare
    shards = []
    for rank in range(world):
        s = DistributedSampler(range(n), num_replicas=world, rank=rank, shuffle=shuffle, seed=42,
                               drop_last=drop_last)
        s.set_epoch(epoch)
        got = distributed_indices(n, world, rank, shuffle=shuffle, seed=42, epoch=epoch, drop_last=drop_last)
        assert got.tolist() == list(iter(s))
        shards.append(got)
    # equal-length shards (DDP lock-step), and without drop_last every row is covered
    assert len({len(s) for s in shards}) == 1
    if not drop_last:
        assert set(torch.cat(shards).tolist()) == set(range(n))


@SETTINGS
@given(n=st.integers(2, 3000), frac=st.sampled_from([0.5, 0.8, 0.9]))
def test_seeded_split_matches_random_split(n, frac):
    from torch.utils.data import TensorDataset, random_split

    n_tr = int(frac * n)
    g = torch.Generator().manual_seed(42)
    tr, va = random_split(TensorDataset(torch.arange(n)), [n_tr, n - n_tr], generator=g)
    a, b = seeded_random_split(n, frac, 42)
    assert a.tolist() == list(tr.indices) and b.tolist() == list(va.indices)


@SETTINGS
@given(n_local=st.integers(0, 500), bs=st.integers(1, 64), drop_last=st.booleans())
def test_batches_cover_shard(n_local, bs, drop_last):
    idx = torch.arange(n_local)
    bl = batches(idx, bs, drop_last)
    assert len(bl) == num_batches(n_local, bs, drop_last)
    assert all(len(b) == bs for b in bl[:-1])
    if not drop_last and n_local:
        assert torch.cat(bl).tolist() == idx.tolist()


@SETTINGS
@given(vals=st.lists(st.one_of(st.floats(-1e4, 1e4, allow_nan=False), st.just(float("nan"))), min_size=0,
                     max_size=50))
def test_column_stats_spark_semantics(vals):
    a = np.asarray(vals, dtype=np.float64)
    mean, std = column_stats(a)
    v = a[~np.isnan(a)]
    if v.size == 0:
        assert mean is None and std is None
        return
    assert math.isclose(mean, float(v.mean()), rel_tol=1e-12, abs_tol=1e-9)
    if v.size < 2:
        assert std is None  # Spark stddev of one value is null
    else:
        assert math.isclose(std, float(v.std(ddof=1)), rel_tol=1e-9, abs_tol=1e-9)


@SETTINGS
@given(rows=st.integers(2, 60), const_col=st.integers(0, 4), seed=st.integers(0, 10_000))
def test_normalize_frame_zscore_and_guard(rows, const_col, seed):
    import pandas as pd

    from dct_amd.config import FEATURE_COLUMNS, LABEL_COLUMN, LABEL_SOURCE_COLUMN, NORM_SUFFIX

    rng = np.random.default_rng(seed)
    df = pd.DataFrame({c: rng.normal(size=rows) * 10 + 3 for c in FEATURE_COLUMNS})
    df[FEATURE_COLUMNS[const_col]] = 7.0  # std == 0 -> divide by 1.0 (preprocess.py:36)
    df[LABEL_SOURCE_COLUMN] = rng.choice(["rain", "no rain"], size=rows)
    out, stats = normalize_frame(df)
    assert list(out.columns) == [f"{c}{NORM_SUFFIX}" for c in FEATURE_COLUMNS] + [LABEL_COLUMN]
    for i, c in enumerate(FEATURE_COLUMNS):
        col = out[f"{c}{NORM_SUFFIX}"].to_numpy()
        if i == const_col:
            assert np.allclose(col, 0.0)
        else:
            assert abs(col.mean()) < 1e-9 and math.isclose(col.std(ddof=1), 1.0, rel_tol=1e-9)
    assert out[LABEL_COLUMN].tolist() == (df[LABEL_SOURCE_COLUMN] == "rain").astype(int).tolist()


@pytest.mark.parametrize("world", [1, 3])
def test_shards_disjoint_without_padding(world):
    n = 30 * world
    shards = [set(distributed_indices(n, world, r, epoch=1).tolist()) for r in range(world)]
    for i in range(world):
        for j in range(i + 1, world):
            assert not shards[i] & shards[j]
