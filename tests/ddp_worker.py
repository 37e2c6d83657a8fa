"""Worker for tests/test_ddp_cpu.py: a W-rank gloo DDP fit with the Trainer (autograd engine on
CPU: BASELINE config 1, the reference's own execution model).  Every rank dumps its final flat
parameters; rank 0 also writes checkpoints and an MLflow file-store run."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
from torch.utils.data import DataLoader, random_split  # noqa: E402

import dct_amd  # noqa: E402,F401
from dct_amd.ckpt import ModelCheckpoint, resume_checkpoint  # noqa: E402
from dct_amd.data.dataset import TensorPairDataset  # noqa: E402
from dct_amd.data.synthetic import weather_tensors  # noqa: E402
from dct_amd.models.mlp import MLPClassifier  # noqa: E402
from dct_amd.tracking import MLFlowLogger  # noqa: E402
from dct_amd.trainer import DDPStrategy, Trainer, seed_everything  # noqa: E402


def main():
    out_dir, epochs, rows = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    opts = sys.argv[4:]
    resume = "resume" in opts
    accel = "gpu" if "gpu" in opts else "cpu"  # gpu: fused engine (+ in-kernel exchange)
    # engine=<auto|autograd|fused|graph>, hidden=<a,b,..> (default 64), batch=<B>
    kv = dict(o.split("=", 1) for o in opts if "=" in o)
    engine = kv.get("engine", "autograd" if accel == "cpu" else "auto")
    hidden = tuple(int(h) for h in kv.get("hidden", "64").split(","))
    B = int(kv.get("batch", "4"))
    seed_everything(42)
    x, y = weather_tensors(rows, seed=0)
    ds = TensorPairDataset(x, y)
    n_tr = int(0.8 * rows)
    tr, va = random_split(ds, [n_tr, rows - n_tr])
    model = MLPClassifier(5, hidden=hidden, dropout=0.0)
    ck = ModelCheckpoint(dirpath=os.path.join(out_dir, "models"), filename="weather-best-{epoch:02d}-{val_loss:.2f}",
                         monitor="val_loss", mode="min", save_top_k=1, save_last=True)
    logger = MLFlowLogger(experiment_name="weather_forecasting", tracking_uri="file://" + os.path.join(out_dir, "mlruns"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    trainer = Trainer(max_epochs=epochs, accelerator=accel, num_nodes=world,
                      strategy=DDPStrategy(find_unused_parameters=False) if world > 1 else "auto", logger=logger,
                      callbacks=[ck], log_every_n_steps=5, engine=engine, verbose=False)
    ckpt_path = resume_checkpoint(os.path.join(out_dir, "models"), resume)  # --resume or an elastic restart
    trainer.fit(model, DataLoader(tr, batch_size=B, shuffle=True), DataLoader(va, batch_size=B), ckpt_path=ckpt_path)
    flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()]).tolist()
    rank = int(os.environ.get("RANK", "0"))
    with open(os.path.join(out_dir, f"params_rank{rank}.json"), "w") as f:
        json.dump({"params": flat, "global_step": trainer.global_step,
                   "restart": int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")), "val_loss": trainer.callback_metrics.get("val_loss"),
                   "best": ck.best_model_path, "engine": trainer.engine.name,
                   "xg": getattr(trainer.engine, "xg", None) is not None,
                   "gx": getattr(trainer.engine, "gx", None) is not None}, f)


if __name__ == "__main__":
    main()
