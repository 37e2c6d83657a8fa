"""Typed configuration for the continuous-training pipeline.

The reference has no config system: constants are hard-coded across
``jobs/train_lightning_ddp.py`` (batch 4 :122, lr 0.01 :88, epochs 10 :132, split 0.8
:117, seed 42 :14, hidden 64 / dropout 0.2 :58-61, checkpoint template :103-110,
MLflow experiment :93, log cadence :139) and ``jobs/preprocess.py`` (paths :15,:44,
feature list :29), and the distributed topology comes from env vars set by
docker-compose (``MASTER_ADDR/MASTER_PORT/NODE_RANK/WORLD_SIZE/MLFLOW_TRACKING_URI``,
docker-compose.yml:120-125).  Here every one of those constants is a dataclass default
(so an un-configured run behaves exactly like the reference) and the reference's env
var names keep overriding them.  ``DCT_*`` env vars override the rest.
"""
from __future__ import annotations

import dataclasses
import json
import os
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence

# Column contract of the ETL output (preprocess.py:29,48).
FEATURE_COLUMNS: List[str] = ["Temperature", "Humidity", "Wind_Speed", "Cloud_Cover", "Pressure"]
LABEL_SOURCE_COLUMN = "Rain"
LABEL_COLUMN = "label_encoded"
NORM_SUFFIX = "_norm"


@dataclass
class DataConfig:
    raw_csv: str = "/opt/spark/data/raw/weather.csv"  # preprocess.py:15
    processed_out: str = "/opt/spark/data/processed/data.parquet"  # preprocess.py:44
    data_dir: str = "/workspace/data/processed"  # train_lightning_ddp.py:114
    parquet_name: str = "data.parquet"  # train_lightning_ddp.py:19
    train_fraction: float = 0.8  # train_lightning_ddp.py:117
    batch_size: int = 4  # per rank, train_lightning_ddp.py:122
    val_batch_size: int = 4
    shuffle: bool = True
    # where the dataset lives during training: "device" keeps it resident in HBM
    # (one H2D copy) and gathers batches on the GPU; "host" is the CPU/gloo plumbing path.
    residency: str = "device"


@dataclass
class ModelConfig:
    name: str = "weather"  # weather | mlp | tabtransformer
    input_dim: Optional[int] = None  # inferred from the data (#_norm columns) like :125
    hidden: Sequence[int] = (64,)  # train_lightning_ddp.py:58
    num_classes: int = 2  # :61
    dropout: float = 0.2  # :60
    loss: str = "ce"  # ce (reference :69) | mse (BASELINE.json north star)
    # TabTransformer-only knobs
    d_model: int = 64
    n_heads: int = 4
    n_layers: int = 4
    ffn_mult: int = 4


@dataclass
class OptimConfig:
    name: str = "adam"
    lr: float = 0.01  # :88
    betas: Sequence[float] = (0.9, 0.999)
    eps: float = 1e-8
    weight_decay: float = 0.0


@dataclass
class CheckpointConfig:
    dirpath: str = "/workspace/data/models"  # :99
    filename: str = "weather-best-{epoch:02d}-{val_loss:.2f}"  # :105
    monitor: str = "val_loss"  # :107
    mode: str = "min"  # :108
    save_top_k: int = 1  # :106
    save_last: bool = True  # :109
    resume: bool = False  # reference always starts from scratch (:143); opt-in resume


@dataclass
class TrackingConfig:
    experiment_name: str = "weather_forecasting"  # :93
    tracking_uri: str = "http://mlflow-server:5000"  # :94
    log_model: bool = True  # :95
    best_artifact_path: str = "best_checkpoints"  # :160


@dataclass
class DistConfig:
    backend: str = "auto"  # auto -> nccl (RCCL) on GPU, gloo on CPU
    world_size: int = 1
    rank: int = 0
    local_rank: int = 0
    node_rank: int = 0
    master_addr: str = "127.0.0.1"
    master_port: int = 29500  # docker-compose.yml:122
    timeout_s: int = 1800
    # gradient bucket cap for the bucketed reducer (bytes). xGMI rings are per-link bound
    # (7 links x ~153 GB/s); 8 MiB buckets keep each RCCL call in the bandwidth regime
    # while leaving >=2 buckets to overlap with backward on the 4-layer/1024h config.
    bucket_cap_bytes: int = 8 << 20
    first_bucket_bytes: int = 1 << 20


@dataclass
class TrainConfig:
    max_epochs: int = 10  # :132
    log_every_n_steps: int = 5  # :139
    seed: int = 42  # :14
    accelerator: str = "auto"  # auto | gpu | cpu
    precision: str = "fp32"  # fp32 | bf16 (compute dtype of the GEMM path; masters stay fp32)
    num_sanity_val_steps: int = 2
    engine: str = "auto"  # auto | fused | autograd
    steps_per_launch: int = 0  # fused engine: steps per persistent launch (0 = whole epoch)
    fault_inject_rank: int = -1  # kill this rank at fault_inject_step (tests; §5.3)
    fault_inject_step: int = -1


@dataclass
class PipelineConfig:
    data: DataConfig = field(default_factory=DataConfig)
    model: ModelConfig = field(default_factory=ModelConfig)
    optim: OptimConfig = field(default_factory=OptimConfig)
    ckpt: CheckpointConfig = field(default_factory=CheckpointConfig)
    tracking: TrackingConfig = field(default_factory=TrackingConfig)
    dist: DistConfig = field(default_factory=DistConfig)
    train: TrainConfig = field(default_factory=TrainConfig)

    # ------------------------------------------------------------------ env
    def apply_env(self, env: Optional[Dict[str, str]] = None) -> "PipelineConfig":
        """Apply the reference env var contract (docker-compose.yml:120-125) + DCT_* extras."""
        env = dict(os.environ if env is None else env)
        d = self.dist
        if "WORLD_SIZE" in env:
            d.world_size = int(env["WORLD_SIZE"])
        if "NODE_RANK" in env:
            d.node_rank = int(env["NODE_RANK"])
        if "RANK" in env:
            d.rank = int(env["RANK"])
        elif "NODE_RANK" in env and "LOCAL_WORLD_SIZE" not in env:
            # reference topology: one process per "node" (devices=1, num_nodes=W)
            d.rank = d.node_rank
        if "LOCAL_RANK" in env:
            d.local_rank = int(env["LOCAL_RANK"])
        if "MASTER_ADDR" in env:
            d.master_addr = env["MASTER_ADDR"]
        if "MASTER_PORT" in env:
            d.master_port = int(env["MASTER_PORT"])
        if "MLFLOW_TRACKING_URI" in env:
            self.tracking.tracking_uri = env["MLFLOW_TRACKING_URI"]
        simple = {
            "DCT_DATA_DIR": (self.data, "data_dir", str),
            "DCT_MODEL_DIR": (self.ckpt, "dirpath", str),
            "DCT_RAW_CSV": (self.data, "raw_csv", str),
            "DCT_PROCESSED_OUT": (self.data, "processed_out", str),
            "DCT_BATCH_SIZE": (self.data, "batch_size", int),
            "DCT_MAX_EPOCHS": (self.train, "max_epochs", int),
            "DCT_LR": (self.optim, "lr", float),
            "DCT_ACCELERATOR": (self.train, "accelerator", str),
            "DCT_PRECISION": (self.train, "precision", str),
            "DCT_ENGINE": (self.train, "engine", str),
            "DCT_BACKEND": (self.dist, "backend", str),
            "DCT_EXPERIMENT": (self.tracking, "experiment_name", str),
            "DCT_MODEL": (self.model, "name", str),
            "DCT_RESUME": (self.ckpt, "resume", lambda s: s.lower() in ("1", "true", "yes")),
            "DCT_FAULT_RANK": (self.train, "fault_inject_rank", int),
            "DCT_FAULT_STEP": (self.train, "fault_inject_step", int),
            "DCT_BUCKET_CAP_MB": (self.dist, "bucket_cap_bytes", lambda s: int(float(s) * (1 << 20))),
        }
        for key, (obj, attr, conv) in simple.items():
            if key in env and env[key] != "":
                setattr(obj, attr, conv(env[key]))
        if env.get("DCT_HIDDEN"):
            self.model.hidden = tuple(int(x) for x in env["DCT_HIDDEN"].split(","))
        return self

    # ------------------------------------------------------------------ io
    def to_dict(self) -> Dict[str, Any]:
        return dataclasses.asdict(self)

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "PipelineConfig":
        cfg = cls()
        for section, values in (d or {}).items():
            sub = getattr(cfg, section, None)
            if sub is None or not isinstance(values, dict):
                raise KeyError(f"unknown config section {section!r}")
            for k, v in values.items():
                if not hasattr(sub, k):
                    raise KeyError(f"unknown config key {section}.{k}")
                setattr(sub, k, tuple(v) if isinstance(v, list) else v)
        return cfg

    @classmethod
    def load(cls, path: str) -> "PipelineConfig":
        import yaml

        with open(path) as f:
            if path.endswith(".json"):
                d = json.load(f)
            else:
                d = yaml.safe_load(f)
        return cls.from_dict(d)


def default_config(env: Optional[Dict[str, str]] = None) -> PipelineConfig:
    """Reference-equivalent config with env overrides applied."""
    return PipelineConfig().apply_env(env)
