"""Distributed training job (reference: jobs/train_lightning_ddp.py:90-166).

Same contract as the reference job - reads ``<data_dir>/data.parquet`` (``*_norm`` features +
``label_encoded``), seeds 42, 80/20 ``random_split``, batch 4 per rank, WeatherClassifier,
Adam lr 0.01, 10 epochs, ``ModelCheckpoint(weather-best-{epoch:02d}-{val_loss:.2f}, top-1 on
val_loss, save_last)``, MLflow experiment ``weather_forecasting`` and an explicit
``best_checkpoints`` artifact upload from rank 0 - but launched one process per MI355X GPU:

    torchrun --nnodes=1 --nproc-per-node=8 --master-addr 127.0.0.1 jobs/train_ddp.py

The reference's env contract (``WORLD_SIZE``/``NODE_RANK``/``MASTER_ADDR``/``MASTER_PORT`` with one
process per node) still works unchanged.  Extra flags only exist for benchmarks / tests.
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import dct_amd  # noqa: E402
from dct_amd.ckpt import ModelCheckpoint, resume_checkpoint  # noqa: E402
from dct_amd.config import default_config  # noqa: E402
from dct_amd.data.dataset import TensorPairDataset, WeatherDataset  # noqa: E402
from dct_amd.models import build_model  # noqa: E402
from dct_amd.tracking import MLFlowLogger  # noqa: E402
from dct_amd.trainer import DDPStrategy, Trainer, seed_everything  # noqa: E402


def parse_args(argv=None):
    cfg = default_config()
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("--data-dir", default=cfg.data.data_dir)
    p.add_argument("--model-dir", default=cfg.ckpt.dirpath)
    p.add_argument("--epochs", type=int, default=cfg.train.max_epochs)
    p.add_argument("--batch-size", type=int, default=cfg.data.batch_size)
    p.add_argument("--lr", type=float, default=cfg.optim.lr)
    p.add_argument("--model", default=cfg.model.name)
    p.add_argument("--tracking-uri", default=cfg.tracking.tracking_uri)
    p.add_argument("--experiment", default=cfg.tracking.experiment_name)
    p.add_argument("--accelerator", default=cfg.train.accelerator)
    p.add_argument("--engine", default=cfg.train.engine)
    p.add_argument("--seed", type=int, default=cfg.train.seed)
    p.add_argument("--resume", action="store_true", default=cfg.ckpt.resume)
    p.add_argument("--synthetic-rows", type=int, default=0,
                   help="train on N synthetic weather rows instead of the parquet (no data on the box)")
    p.add_argument("--log-every-n-steps", type=int, default=cfg.train.log_every_n_steps)
    p.add_argument("--no-mlflow", action="store_true", help="disable tracking (smoke tests)")
    p.add_argument("--dump-params", default="",
                   help="directory: every rank writes its final flat parameters to params_rank<R>.json "
                        "(replica-consistency checks in tests)")
    return p.parse_args(argv)


def main(argv=None) -> int:
    a = parse_args(argv)
    seed_everything(a.seed)  # reference seeds at import time (:14)

    logger = None
    if not a.no_mlflow:
        logger = MLFlowLogger(experiment_name=a.experiment, tracking_uri=a.tracking_uri, log_model=True)
    os.makedirs(a.model_dir, exist_ok=True)
    checkpoint_callback = ModelCheckpoint(dirpath=a.model_dir, filename="weather-best-{epoch:02d}-{val_loss:.2f}",
                                          save_top_k=1, monitor="val_loss", mode="min", save_last=True)

    if a.synthetic_rows > 0:
        from dct_amd.data.synthetic import weather_tensors

        x, y = weather_tensors(a.synthetic_rows, seed=0)
        full_dataset = TensorPairDataset(x, y)
    else:
        full_dataset = WeatherDataset(a.data_dir)

    import torch
    from torch.utils.data import DataLoader, random_split

    train_size = int(0.8 * len(full_dataset))
    val_size = len(full_dataset) - train_size
    train_set, val_set = random_split(full_dataset, [train_size, val_size])
    train_loader = DataLoader(train_set, batch_size=a.batch_size, shuffle=True, num_workers=0)
    val_loader = DataLoader(val_set, batch_size=a.batch_size, shuffle=False, num_workers=0)

    input_dim = full_dataset.features.shape[1]
    model = build_model(a.model, input_dim, lr=a.lr)

    world_size = int(os.environ.get("WORLD_SIZE", 1))
    trainer = Trainer(
        max_epochs=a.epochs,
        accelerator=a.accelerator,
        devices=1,
        num_nodes=world_size,
        strategy=DDPStrategy(find_unused_parameters=False) if world_size > 1 else "auto",
        logger=logger,
        callbacks=[checkpoint_callback],
        log_every_n_steps=a.log_every_n_steps,
        engine=a.engine,
    )
    last = os.path.join(a.model_dir, "last.ckpt")
    # --resume, or a torchrun elastic restart after a failed rank: continue from last.ckpt
    ckpt_path = resume_checkpoint(a.model_dir, a.resume)
    trainer.fit(model, train_loader, val_loader, ckpt_path=ckpt_path)
    if a.dump_params:
        import json

        os.makedirs(a.dump_params, exist_ok=True)
        flat = torch.cat([p.detach().reshape(-1).cpu() for p in model.parameters()]).tolist()
        with open(os.path.join(a.dump_params, f"params_rank{trainer.global_rank}.json"), "w") as f:
            json.dump({"params": flat, "global_step": trainer.global_step, "world_size": trainer.world_size}, f)

    if trainer.global_rank == 0:
        best_path = checkpoint_callback.best_model_path
        if not best_path or not os.path.exists(best_path):
            print(f"Best model not found at {best_path!r}; falling back to last.ckpt")
            best_path = last
        print(f"Training finished. Saving model path: {best_path}")
        if os.path.exists(best_path):
            if logger is not None:
                logger.experiment.log_artifact(logger.run_id, best_path, "best_checkpoints")
                print("Model uploaded to MLflow")
        else:
            print("CRITICAL: No model file found to upload!")
            trainer.teardown()
            return 1
    trainer.teardown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
