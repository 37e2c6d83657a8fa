"""Training datasets.

``WeatherDataset`` keeps the reference's contract (jobs/train_lightning_ddp.py:16-49):
  * ``<data_path>/data.parquet`` must exist -> ``FileNotFoundError`` (:22-26);
  * read failure -> ``RuntimeError("Failed to read Parquet file: ...")`` (:30-33);
  * features = every column ending in ``_norm`` in file order (:37); none -> ``ValueError`` (:39-40);
  * fp32 features / int64 labels fully materialised (:45-46); ``__getitem__`` -> (x, y) (:49).

``DeviceTensorDataset`` is the MI355X side of the same data: the whole table is copied to HBM
once (pinned host buffer -> one H2D copy) and batches are gathered on the GPU from index
tensors, so the per-sample Python collate of the reference (:49 + default_collate) leaves the
hot loop entirely.
"""
from __future__ import annotations

import os
from typing import Optional, Sequence

import torch

from ..config import LABEL_COLUMN, NORM_SUFFIX


class WeatherDataset(torch.utils.data.Dataset):
    def __init__(self, data_path: str, parquet_name: str = "data.parquet", verbose: bool = True):
        parquet_path = os.path.join(data_path, parquet_name)
        if not os.path.exists(parquet_path):
            raise FileNotFoundError(
                f"CRITICAL ERROR: Data not found at {parquet_path}.\n"
                "Did the Spark preprocessing step finish successfully?"
            )
        if verbose:
            print(f"Loading data from: {parquet_path}")
        try:
            import pandas as pd

            df = pd.read_parquet(parquet_path)
        except Exception as e:  # noqa: BLE001 - reference wraps every read error
            raise RuntimeError(f"Failed to read Parquet file: {e}")
        feature_cols = [c for c in df.columns if c.endswith(NORM_SUFFIX)]
        if not feature_cols:
            raise ValueError("CRITICAL ERROR: No columns ending with '_norm' found. Check Spark logic.")
        if verbose:
            print(f"Loaded {len(df)} rows.")
            print(f"Training with {len(feature_cols)} features: {feature_cols}")
        self.feature_cols = feature_cols
        self.features = torch.tensor(df[feature_cols].to_numpy(), dtype=torch.float32)
        self.labels = torch.tensor(df[LABEL_COLUMN].to_numpy(), dtype=torch.int64)

    def __len__(self):
        return len(self.features)

    def __getitem__(self, idx):
        return self.features[idx], self.labels[idx]


class TensorPairDataset(torch.utils.data.Dataset):
    """(features, labels) already in memory (synthetic data, subsets)."""

    def __init__(self, features: torch.Tensor, labels: torch.Tensor):
        assert len(features) == len(labels)
        self.features = features
        self.labels = labels

    def __len__(self):
        return len(self.features)

    def __getitem__(self, idx):
        return self.features[idx], self.labels[idx]


def dataset_tensors(ds) -> "tuple[torch.Tensor, torch.Tensor]":
    """Materialise (features, labels) for a dataset or a ``torch.utils.data.Subset`` chain."""
    idx = None
    base = ds
    while isinstance(base, torch.utils.data.Subset):
        sub = torch.as_tensor(base.indices, dtype=torch.int64)
        idx = sub if idx is None else sub[idx]
        base = base.dataset
    if not hasattr(base, "features") or not hasattr(base, "labels"):
        xs, ys = zip(*[base[i] for i in range(len(base))])
        feats, labels = torch.stack(xs), torch.as_tensor(ys)
    else:
        feats, labels = base.features, base.labels
    if idx is not None:
        feats, labels = feats[idx], labels[idx]
    return feats, labels


class DeviceTensorDataset:
    """Whole dataset resident on a device; batches are gathered on-device by index."""

    def __init__(self, features: torch.Tensor, labels: torch.Tensor, device, feat_dtype=torch.float32):
        device = torch.device(device)
        if device.type == "cuda":
            f = features.to(feat_dtype).contiguous().pin_memory()
            l = labels.to(torch.int32).contiguous().pin_memory()
            self.features = f.to(device, non_blocking=True)
            self.labels = l.to(device, non_blocking=True)
        else:
            self.features = features.to(feat_dtype).contiguous()
            self.labels = labels.to(torch.int32).contiguous()
        self.device = device

    def __len__(self):
        return self.features.shape[0]

    @property
    def dim(self) -> int:
        return self.features.shape[1]
