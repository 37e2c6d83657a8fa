"""``Trainer``: the fit loop (reference: ``pl.Trainer(...).fit(model, train_loader, val_loader)``,
jobs/train_lightning_ddp.py:128-143).

Semantics kept from the reference's Lightning 2.1 run [lib]:
  * ``num_sanity_val_steps`` validation batches before training (metrics discarded);
  * per epoch: all train steps, then a full validation pass; ``DistributedSampler``-equivalent
    sharding (``seed = PL_GLOBAL_SEED``, epoch-dependent shuffle, wrap-padding) for train and val;
  * ``self.log("train_loss", sync_dist=True)`` -> cross-rank mean, written to the logger every
    ``log_every_n_steps`` optimizer steps (step value = batches stepped before that batch);
  * ``val_loss``/``val_acc`` -> batch-size-weighted epoch means, cross-rank mean, logged with
    ``epoch`` at the end of validation; ``ModelCheckpoint`` decides on rank 0, all ranks barrier;
  * ``best_model_path`` / ``last.ckpt`` / ``callback_metrics`` like Lightning.
MI355X additions: the fused / autograd step engines (trainer/engines.py), per-epoch wall clock
and whole-job samples/sec as extra metrics, opt-in resume from a checkpoint, fault injection.
"""
from __future__ import annotations

import math
import os
import random
import sys
import time
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..ckpt.callbacks import ModelCheckpoint
from ..ckpt.lightning_io import build_checkpoint, load_checkpoint, save_checkpoint
from ..data.dataset import dataset_tensors
from ..data.sampler import distributed_indices
from ..parallel.dist import DistContext, init_distributed, shutdown
from .engines import AutogradEngine, FusedMLPEngine, adam_hparams_from
from .graph_engine import GraphMLPEngine
from ..utils.debug import assert_reducer_ordering
from ..utils.tracing import PhaseTimer, trace_range


def seed_everything(seed: int = 42) -> int:
    """``pl.seed_everything`` equivalent (python/numpy/torch RNGs + PL_GLOBAL_SEED)."""
    seed = int(seed)
    os.environ["PL_GLOBAL_SEED"] = str(seed)
    random.seed(seed)
    np.random.seed(seed % (2 ** 32))
    torch.manual_seed(seed)
    return seed


class DDPStrategy:
    """``pytorch_lightning.strategies.DDPStrategy`` stand-in (train_lightning_ddp.py:136)."""

    def __init__(self, find_unused_parameters: bool = False, bucket_cap_mb: float = 8.0, backend: str = "auto",
                 timeout_s: int = 1800, first_bucket_mb: float = 1.0):
        self.find_unused_parameters = find_unused_parameters
        self.bucket_cap_bytes = int(bucket_cap_mb * (1 << 20))
        self.first_bucket_bytes = int(first_bucket_mb * (1 << 20))
        self.backend = backend
        self.timeout_s = timeout_s


class _FaultInjected(RuntimeError):
    pass


class Trainer:
    def __init__(self, max_epochs: int = 10, accelerator: str = "auto", devices: int = 1, num_nodes: int = 1,
                 strategy: Any = "auto", logger=None, callbacks: Optional[Sequence] = None,
                 log_every_n_steps: int = 50, num_sanity_val_steps: int = 2, engine: str = "auto",
                 steps_per_launch: int = 0, enable_progress_bar: bool = True, default_root_dir: Optional[str] = None,
                 max_steps: int = -1, fault_inject: Optional[Tuple[int, int]] = None, verbose: bool = True):
        self.max_epochs = int(max_epochs)
        self.max_steps = int(max_steps)
        self.accelerator = accelerator
        self.devices = devices
        self.num_nodes = num_nodes
        self.strategy = strategy if isinstance(strategy, DDPStrategy) else DDPStrategy()
        self.logger = logger
        self.callbacks = list(callbacks or [])
        self.log_every_n_steps = int(log_every_n_steps)
        self.num_sanity_val_steps = int(num_sanity_val_steps)
        self.engine_choice = engine
        self.steps_per_launch = steps_per_launch
        self.enable_progress_bar = enable_progress_bar
        self.default_root_dir = default_root_dir or os.getcwd()
        self.fault_inject = fault_inject
        self.verbose = verbose
        env_fault = (os.environ.get("DCT_FAULT_RANK"), os.environ.get("DCT_FAULT_STEP"))
        if self.fault_inject is None and env_fault[0] and env_fault[1]:
            self.fault_inject = (int(env_fault[0]), int(env_fault[1]))
        self.ctx: Optional[DistContext] = None
        self.current_epoch = 0
        self.global_step = 0
        self.callback_metrics: Dict[str, float] = {}
        self.logged_metrics: Dict[str, float] = {}
        self.progress_bar_metrics: Dict[str, float] = {}
        self.epoch_times: List[float] = []
        self.phase_times = PhaseTimer(sync_device=False)  # host phases of an epoch -> time/<phase>_s
        self.engine = None
        self._stage = "idle"
        self._step_logs: Dict[str, Tuple[torch.Tensor, bool]] = {}
        self._epoch_logs: Dict[str, List] = {}
        self._cur_batch_size = 1
        self.should_stop = False

    # ------------------------------------------------------------------ properties
    @property
    def global_rank(self) -> int:
        return self.ctx.rank if self.ctx else int(os.environ.get("RANK", os.environ.get("NODE_RANK", 0)))

    @property
    def world_size(self) -> int:
        return self.ctx.world_size if self.ctx else 1

    @property
    def is_global_zero(self) -> bool:
        return self.global_rank == 0

    @property
    def checkpoint_callback(self) -> Optional[ModelCheckpoint]:
        for c in self.callbacks:
            if isinstance(c, ModelCheckpoint):
                return c
        return None

    # ------------------------------------------------------------------ logging from the module
    def _log_from_module(self, name, value, sync_dist=False, prog_bar=False, on_step=None, on_epoch=None,
                         batch_size=None):
        v = value.detach() if isinstance(value, torch.Tensor) else torch.tensor(float(value))
        if self._stage == "train":
            on_step = True if on_step is None else on_step
            on_epoch = False if on_epoch is None else on_epoch
            if on_step:
                self._step_logs[name] = (v, sync_dist)
            if on_epoch:
                acc = self._epoch_logs.setdefault(name, [0.0, 0, sync_dist, prog_bar])
                bs = batch_size or self._cur_batch_size
                acc[0] += float(v) * bs
                acc[1] += bs
        elif self._stage in ("val", "sanity"):
            bs = batch_size or self._cur_batch_size
            acc = self._epoch_logs.setdefault(name, [0.0, 0, sync_dist, prog_bar])
            acc[0] += float(v) * bs
            acc[1] += bs

    def _reduce_epoch_logs(self) -> Dict[str, float]:
        out = {}
        names = sorted(self._epoch_logs)
        if not names:
            return out
        vals = torch.tensor([self._epoch_logs[n][0] / max(1, self._epoch_logs[n][1]) for n in names],
                            dtype=torch.float64)
        if any(self._epoch_logs[n][2] for n in names):
            vals = self.ctx.all_reduce_mean(vals.to(torch.float32)).to(torch.float64)
        for n, v in zip(names, vals.tolist()):
            out[n] = v
        self._epoch_logs = {}
        return out

    def _log_series(self, key: str, points):
        """_log_metrics({key: v}, step) for every (step, v) in points, in one logger call."""
        if not points:
            return
        self.logged_metrics.update({key: points[-1][1], "epoch": self.current_epoch})
        if self.logger is not None and self.is_global_zero:
            if hasattr(self.logger, "log_metric_series"):
                self.logger.log_metric_series(key, points, extra={"epoch": self.current_epoch})
            else:
                for step, v in points:
                    self.logger.log_metrics({key: v, "epoch": self.current_epoch}, step)

    def _log_metrics(self, metrics: Dict[str, float], step: int):
        metrics = dict(metrics)
        metrics.setdefault("epoch", self.current_epoch)
        self.logged_metrics.update(metrics)
        if self.logger is not None and self.is_global_zero:
            self.logger.log_metrics(metrics, step)

    # ------------------------------------------------------------------ data plumbing
    @staticmethod
    def _loader_info(loader) -> Dict[str, Any]:
        if loader is None:
            return {}
        ds = loader.dataset if hasattr(loader, "dataset") else loader
        bs = getattr(loader, "batch_size", None) or 1
        sampler = getattr(loader, "sampler", None)
        shuffle = isinstance(sampler, torch.utils.data.RandomSampler)
        return dict(dataset=ds, batch_size=int(bs), shuffle=shuffle, drop_last=bool(getattr(loader, "drop_last", False)))

    @staticmethod
    def _split_tensors(train_ds, val_ds):
        """Return (X_all, Y_all, train_rows, val_rows) sharing one table when both splits come from
        the same base dataset (random_split Subsets), so the table is uploaded to HBM once."""
        def base_and_rows(ds):
            idx = None
            b = ds
            while isinstance(b, torch.utils.data.Subset):
                sub = torch.as_tensor(b.indices, dtype=torch.int64)
                idx = sub if idx is None else sub[idx]
                b = b.dataset
            return b, idx

        tb, tr = base_and_rows(train_ds)
        if val_ds is not None:
            vb, vr = base_and_rows(val_ds)
        else:
            vb, vr = tb, torch.zeros(0, dtype=torch.int64)
        if tb is vb and hasattr(tb, "features"):
            X, Y = tb.features, tb.labels
            n = len(X)
            tr = torch.arange(n) if tr is None else tr
            vr = torch.arange(n) if vr is None else vr
            return X, Y, tr, vr
        Xt, Yt = dataset_tensors(train_ds)
        if val_ds is None:
            return Xt, Yt, torch.arange(len(Xt)), torch.zeros(0, dtype=torch.int64)
        Xv, Yv = dataset_tensors(val_ds)
        X = torch.cat([Xt, Xv])
        Y = torch.cat([Yt, Yv])
        return X, Y, torch.arange(len(Xt)), torch.arange(len(Xt), len(Xt) + len(Xv))

    # ------------------------------------------------------------------ engine selection
    def _make_engine(self, model, batch_size: int, seed: int):
        ctx = self.ctx
        choice = self.engine_choice
        if choice == "auto":
            choice = os.environ.get("DCT_ENGINE", "auto")
        adam = adam_hparams_from(model.configure_optimizers())
        if choice in ("auto", "fused") and adam is not None and FusedMLPEngine.applicable(model, ctx.device, batch_size):
            return FusedMLPEngine(model, ctx, batch_size, seed, adam, steps_per_launch=self.steps_per_launch)
        if choice == "fused":
            raise RuntimeError("engine='fused' requested but the model/device/batch is not supported by it")
        if choice in ("auto", "graph") and adam is not None and GraphMLPEngine.applicable(model, ctx.device, batch_size):
            return GraphMLPEngine(model, ctx, batch_size, seed, adam, self.strategy.bucket_cap_bytes,
                                  self.strategy.first_bucket_bytes)
        if choice == "graph":
            raise RuntimeError("engine='graph' requested but the model/device is not supported by it")
        model.to(ctx.device)
        return AutogradEngine(model, ctx, batch_size, seed, self.strategy.bucket_cap_bytes,
                              self.strategy.first_bucket_bytes)

    # ------------------------------------------------------------------ checkpoints
    def _checkpoint_dict(self, batches_in_epoch: int = 0, val_batches: int = 0) -> Dict[str, Any]:
        model = self._model
        self.engine.sync_to_model()
        callbacks = {}
        for cb in self.callbacks:
            if isinstance(cb, ModelCheckpoint):
                callbacks[cb.state_key] = cb.state_dict()
        hp = dict(model.hparams) if getattr(model, "hparams", None) else None
        ckpt = build_checkpoint(model.state_dict(), epoch=self.current_epoch, global_step=self.global_step,
                                optimizer_states=[self.engine.optimizer_state_dict()], callbacks=callbacks,
                                hyper_parameters=hp, hparams_name=getattr(model, "_hparams_name", "kwargs"),
                                batches_in_epoch=batches_in_epoch, val_batches=val_batches)
        model.on_save_checkpoint(ckpt)
        return ckpt

    def save_checkpoint(self, filepath: str):
        ckpt = self._checkpoint_dict()
        if self.is_global_zero:
            save_checkpoint(ckpt, filepath)
        if self.ctx is not None:
            self.ctx.barrier()

    def _restore(self, ckpt_path: str):
        ckpt = load_checkpoint(ckpt_path)
        self._model.load_state_dict(ckpt["state_dict"])
        self.engine.load_from_model()
        if ckpt.get("optimizer_states"):
            self.engine.load_optimizer_state(ckpt["optimizer_states"][0], int(ckpt.get("global_step", 0)))
        for cb in self.callbacks:
            if isinstance(cb, ModelCheckpoint) and cb.state_key in ckpt.get("callbacks", {}):
                cb.load_state_dict(ckpt["callbacks"][cb.state_key])
        self.global_step = int(ckpt.get("global_step", 0))
        self.engine.global_step = self.global_step
        # Lightning resumes at the epoch after the saved one
        return int(ckpt.get("epoch", 0)) + 1

    # ------------------------------------------------------------------ fit
    def fit(self, model, train_dataloaders=None, val_dataloaders=None, ckpt_path: Optional[str] = None):
        self._model = model
        self._graph_step_logs = None
        self.ctx = init_distributed(self.accelerator, self.strategy.backend, self.strategy.timeout_s)
        object.__setattr__(model, "_trainer", self)
        seed = int(os.environ.get("PL_GLOBAL_SEED", "0"))
        tinfo = self._loader_info(train_dataloaders)
        vinfo = self._loader_info(val_dataloaders)
        B = tinfo.get("batch_size", 4)
        VB = vinfo.get("batch_size", B)
        X, Y, train_rows, val_rows = self._split_tensors(tinfo["dataset"], vinfo.get("dataset"))
        if self.logger is not None:
            self.logger.rank_zero = self.is_global_zero
        self.engine = self._make_engine(model, B, seed)
        self.engine.attach_data(X, Y, train_rows, val_rows)
        for cb in self.callbacks:
            if isinstance(cb, ModelCheckpoint) and cb.dirpath is None:
                cb.dirpath = os.path.join(self.default_root_dir, "checkpoints")
        start_epoch = 0
        if ckpt_path:
            start_epoch = self._restore(ckpt_path)
        if self.logger is not None and self.is_global_zero and getattr(model, "hparams", None):
            self.logger.log_hyperparams(dict(model.hparams))
        if self.verbose and self.is_global_zero:
            print(f"[dct] engine={self.engine.name} device={self.ctx.device} world={self.world_size} "
                  f"batch/rank={B} train_rows={len(train_rows)} val_rows={len(val_rows)}", flush=True)
        status = "success"
        try:
            if start_epoch == 0 and self.num_sanity_val_steps > 0 and len(val_rows):
                with trace_range("sanity_val"):
                    self._validate(VB, limit_batches=self.num_sanity_val_steps, sanity=True)
            for epoch in range(start_epoch, self.max_epochs):
                self.current_epoch = epoch
                t0 = time.perf_counter()
                with trace_range(f"epoch{epoch}/train"):
                    n_steps = self._train_epoch(epoch, B, tinfo.get("shuffle", True))
                train_t = time.perf_counter() - t0
                with self.phase_times.phase("validate"):
                    val_metrics = self._validate(VB) if len(val_rows) else {}
                epoch_t = time.perf_counter() - t0
                self.epoch_times.append(epoch_t)
                samples = len(train_rows)
                self.callback_metrics.update(val_metrics)
                if val_metrics:
                    self._log_metrics(val_metrics, self.global_step)
                extra = {"epoch_time_s": epoch_t, "train_time_s": train_t,
                         "samples_per_sec": samples / max(train_t, 1e-9),
                         "step_time_ms": 1e3 * train_t / max(n_steps, 1)}
                assert_reducer_ordering(getattr(self.engine, "reducer", None), f"epoch {epoch}")
                ar_ms = self._epoch_allreduce_ms()
                if ar_ms is not None:
                    extra["allreduce_ms"] = ar_ms
                pt = getattr(self.engine, "phase_timer", None)
                if pt is not None:  # GPU time of the step phases (DCT_PHASE_TIMING=1)
                    ph = pt.read()
                    extra.update({f"time/{k}_s": v for k, v in ph.items() if k != "steps"})
                extra.update(self.phase_times.metrics())
                self.phase_times = PhaseTimer(sync_device=False)
                self._log_metrics(extra, self.global_step)
                if self.logger is not None and self.is_global_zero:
                    self.logger.flush()  # the epoch's metrics reach the tracking store now
                with trace_range(f"epoch{epoch}/checkpoint"):
                    t_ck = time.perf_counter()
                    self._run_checkpoint_callbacks(n_steps)
                    t_ck = time.perf_counter() - t_ck
                if self.logger is not None and self.is_global_zero:
                    self._log_metrics({"time/checkpoint_s": t_ck}, self.global_step)
                if self.verbose and self.is_global_zero:
                    vm = " ".join(f"{k}={v:.4f}" for k, v in val_metrics.items())
                    print(f"[dct] epoch {epoch} steps={n_steps} {vm} epoch_time={epoch_t:.3f}s "
                          f"train_samples/s={extra['samples_per_sec']:.0f}", flush=True)
                if self.should_stop or (0 < self.max_steps <= self.global_step):
                    break
        except _FaultInjected:
            status = "failed"
            raise
        except BaseException:
            status = "failed"
            raise
        finally:
            if self.logger is not None and self.is_global_zero:
                try:
                    self.logger.finalize(status)
                except Exception as e:  # noqa: BLE001
                    print(f"[dct] logger finalize failed: {e!r}", file=sys.stderr)
        return self

    def teardown(self):
        if self.ctx is not None:
            shutdown(self.ctx)

    def _epoch_allreduce_ms(self) -> Optional[float]:
        """Gradient all-reduce time of the epoch (SURVEY 5.5 extra key): the in-kernel exchange's
        own clock on the fused engine, the exposed (not overlapped) wait of the torch reducer on
        the gloo path; None where it is not measured (the RCCL comm-stream reducers)."""
        eng = self.engine
        if getattr(eng, "last_allreduce_ms", None) is not None:
            return float(eng.last_allreduce_ms)
        red = getattr(eng, "reducer", None)
        if red is not None and hasattr(red, "wait_s"):
            ms = red.wait_s * 1e3
            red.wait_s = 0.0
            return ms
        return None

    # ------------------------------------------------------------------ loops
    def _maybe_fault(self, step: int):
        # an injected fault fires on the first attempt only: the workers torchrun restarts after it
        # (--max-restarts) are the recovery being tested, not new victims
        if self.fault_inject and int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0") or 0) > 0:
            return
        if self.fault_inject and self.global_rank == self.fault_inject[0] and step >= self.fault_inject[1]:
            print(f"[dct] fault injection: rank {self.global_rank} exits at step {step}", flush=True)
            sys.stdout.flush()
            os._exit(17)

    def _train_epoch(self, epoch: int, B: int, shuffle: bool) -> int:
        self._stage = "train"
        eng = self.engine
        if getattr(eng, "epoch_engine", False):
            losses = eng.train_epoch(epoch, shuffle)
            n = losses.numel()
            first = self.global_step
            self.global_step += n
            self._maybe_fault(self.global_step)
            lv = losses.cpu().tolist()
            # every log_every_n_steps-th step's loss, as ONE series call (a 20k-step epoch has 4k)
            ev = self.log_every_n_steps
            k0 = (-first) % ev or ev  # first k in 1..n with (first + k) % ev == 0
            self._log_series("train_loss", [(first + k - 1, lv[k - 1]) for k in range(k0, n + 1, ev)])
            if n:
                self.callback_metrics["train_loss"] = lv[-1]
            return n
        local = eng.epoch_local_indices(len(eng.train_rows), epoch, shuffle)
        rows_all = eng.train_rows[local]
        n_steps = math.ceil(len(rows_all) / B)
        for bi in range(n_steps):
            rows = rows_all[bi * B: (bi + 1) * B]
            self._cur_batch_size = len(rows)
            self._step_logs = {}
            loss = eng.train_step(rows, bi)
            mode = getattr(eng, "last_step_mode", "eager")
            if mode == "captured":
                # what training_step logged while it was traced into the step graph are the graph's
                # static outputs: every replay refreshes them, so they stand for later steps too
                self._graph_step_logs = dict(self._step_logs)
            elif mode == "replayed" and not self._step_logs:
                # a replay runs no Python: reuse the captured logs, else the step's loss
                self._step_logs = dict(getattr(self, "_graph_step_logs", None) or {"train_loss": (loss, True)})
            self.global_step += 1
            self._maybe_fault(self.global_step)
            if self.global_step % self.log_every_n_steps == 0 and self._step_logs:
                names = sorted(self._step_logs)
                vals = torch.stack([self._step_logs[n][0].float().reshape(()).cpu() for n in names])
                if any(self._step_logs[n][1] for n in names):
                    vals = self.ctx.all_reduce_mean(vals)
                m = dict(zip(names, vals.tolist()))
                self._log_metrics(m, self.global_step - 1)
                self.callback_metrics.update(m)
            if 0 < self.max_steps <= self.global_step:
                break
        return n_steps

    @torch.no_grad()
    def _validate(self, VB: int, limit_batches: Optional[int] = None, sanity: bool = False) -> Dict[str, float]:
        self._stage = "sanity" if sanity else "val"
        eng = self.engine
        try:
            if getattr(eng, "epoch_engine", False):
                limit = None if limit_batches is None else limit_batches * VB
                vl, va = eng.validate(limit=limit)
                return {} if sanity else {"val_loss": vl, "val_acc": va}
            model = self._model
            was_training = model.training
            model.eval()
            local = distributed_indices(len(eng.val_rows), self.world_size, self.global_rank, shuffle=False)
            rows_all = eng.val_rows[local]
            nb = math.ceil(len(rows_all) / VB)
            if limit_batches is not None:
                nb = min(nb, limit_batches)
            self._epoch_logs = {}
            for bi in range(nb):
                rows = rows_all[bi * VB: (bi + 1) * VB].to(eng.device)
                self._cur_batch_size = len(rows)
                model.validation_step((eng.X[rows], eng.Y[rows]), bi)
            out = self._reduce_epoch_logs()
            model.train(was_training)
            return {} if sanity else out
        finally:
            self._stage = "idle"

    def _run_checkpoint_callbacks(self, batches_in_epoch: int):
        metrics = dict(self.callback_metrics)
        metrics["epoch"] = self.current_epoch
        metrics["step"] = self.global_step
        for cb in self.callbacks:
            if not isinstance(cb, ModelCheckpoint):
                continue

            def save_fn(path, cb=cb):
                # the checkpoint embeds the callback state AFTER this epoch's decision
                ckpt = self._checkpoint_dict(batches_in_epoch)
                save_checkpoint(ckpt, path)
                if self.logger is not None:
                    self.logger.after_save_checkpoint(path)

            if self.is_global_zero:
                cb.on_validation_end(metrics, save_fn, True, self.current_epoch)
            else:
                cb.on_validation_end(metrics, lambda p: None, False, self.current_epoch)
                self.engine.sync_to_model()
        self.ctx.barrier()
