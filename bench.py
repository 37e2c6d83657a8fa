#!/usr/bin/env python3
"""Headline benchmark: whole-node training samples/sec of the weather-MLP DDP job.

BASELINE.json metric: "samples/sec (whole node) for weather-MLP DDP at 1/2/4/8 MI355X; epoch
wall-clock", on BASELINE.json's "Weather MLP (3-layer, 128-h)" (configs 0-2).  Default workload
(--model weather-mlp-3x128): 5 -> 128 -> 128 -> 2 with ReLU + Dropout(0.2) after each hidden
layer, cross-entropy, Adam(lr=0.01), batch 4 PER RANK (weak scaling) - the reference training step
(jobs/train_lightning_ddp.py:57-62,66-71,88,122) with BASELINE's 3-layer 128-h model -
DistributedSampler sharding, per-step gradient all-reduce across ranks plus the sync_dist
train_loss.  At one rank the reference-exact WeatherClassifier 5->64->2 is measured too, with the
same steps / warmup, and reported under extra.reference_model_*.  Other configs:
  --model weather              the reference-exact WeatherClassifier 5-64-2 as the headline
  --model tabular-mlp-4x1024   100M x 256 synthetic rows (bf16, HBM-resident), 256-1024-1024-1024-2
                               MLP, MSE, Adam(1e-3), batch 4096 per rank, graph-captured MFMA step
  --model tabtransformer       4-layer TabTransformer over 64 feature tokens (d 64, 4 heads), CE,
                               Adam(1e-3), batch 512 per rank, HIP GEMM/LayerNorm/attention kernels,
                               autograd step captured in a HIP graph
  --device cpu                 BASELINE config 1 (CPU plumbing: single process or gloo DDP, the
                               reference's own execution model) with the autograd engine
Data: synthetic rows (no network), random-init weights.

Timed region: exactly K optimizer steps, bracketed by barrier + device synchronize on both
sides, max over ranks.

    python bench.py --gpus 1 --steps 20000 --warmup 2000
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29511 bench.py --gpus 8
"""
from __future__ import annotations

import argparse
import gc
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

# BASELINE.md local probe (reference step shape, torch CPU, W=1): ~8,500 samples/s whole node.
# The reference publishes no number (BASELINE.json "published": {}); this probe is the only one.
# BASELINE.md local probes (reference step shape, plain torch on CPU, W=1, tools/cpu_reference_probe.py);
# the reference publishes no number (BASELINE.json "published": {}).  3x128: the 5-64-2 probe scaled by
# the measured 3x128 / 5-64-2 probe ratio (0.52), an optimistic CPU ceiling.
BASELINE_SAMPLES_PER_SEC = {"weather": 8500.0, "weather-mlp-3x128": 4400.0}
BASELINE_REF = {"weather": "BASELINE.md CPU probe (reference step shape, torch CPU, W=1): 8500 samples/s; the "
                           "reference publishes none",
                "weather-mlp-3x128": "BASELINE.md CPU probe of the 3-layer 128-h step (torch CPU, W=1): 4400 "
                                     "samples/s; the reference publishes none"}
MODELS = {"weather": "WeatherClassifier 5-64-2 (reference jobs/train_lightning_ddp.py)",
          "weather-mlp-3x128": "weather-mlp-3x128: Weather MLP (3-layer, 128-h) 5-128-128-2, ReLU+Dropout 0.2, CE "
                               "(BASELINE.json configs 0-2)",
          "tabular-mlp-4x1024": "tabular MLP 256-1024-1024-1024-2 (BASELINE config 4)",
          "tabtransformer": "TabTransformer 4 layers, 64 feature tokens, d 64, 4 heads (BASELINE config 5)"}
TABULAR = ("tabular-mlp-4x1024",)
TRANSFORMER = ("tabtransformer",)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=None, help="timed steps (default 20000; tabular 200)")
    p.add_argument("--warmup", type=int, default=None, help="untimed steps (default 2000; tabular 20)")
    p.add_argument("--model", default="weather-mlp-3x128",
                   help="weather-mlp-3x128 (BASELINE) | weather (reference 5-64-2) | tabular-mlp-4x1024 | tabtransformer")
    p.add_argument("--no-reference-model", action="store_true",
                   help="skip the extra 5-64-2 measurement of a single-rank weather-mlp-3x128 run")
    p.add_argument("--batch", type=int, default=None, help="per-rank batch (reference: 4; tabular: 4096)")
    p.add_argument("--rows", type=int, default=0,
                   help="synthetic dataset rows (0 = sized to the run; tabular: 100M per BASELINE config 4)")
    p.add_argument("--device", default="gpu", choices=("gpu", "cpu"),
                   help="cpu: BASELINE config 1 (autograd engine, gloo) - the plumbing path")
    p.add_argument("--epoch-rows", type=int, default=None,
                   help="dataset size used for the reported epoch wall-clock (weather 100k, tabular 100M)")
    p.add_argument("--reserve-cus", type=int, default=0,
                   help="A/B: run the step on a stream masked to all CUs but N, the DDP bucket reducer's "
                        "collectives on a stream masked to those N (hipExtStreamCreateWithCUMask)")
    p.add_argument("--reserve-pattern", default="spread", choices=("spread", "low", "high"),
                   help="which CU mask bits --reserve-cus takes: evenly spaced, the first N or the last N")
    p.add_argument("--no-epoch", action="store_true",
                   help="skip the measured epoch (weather models on GPU: one real epoch of --epoch-rows rows, "
                        "train + validation, timed after the step window)")
    a = p.parse_args()
    tab = a.model in TABULAR
    tt = a.model in TRANSFORMER
    a.steps = a.steps if a.steps is not None else (200 if (tab or tt) else 20000)
    a.warmup = a.warmup if a.warmup is not None else (20 if (tab or tt) else 2000)
    a.batch = a.batch if a.batch is not None else (4096 if tab else (512 if tt else 4))
    a.epoch_rows = a.epoch_rows if a.epoch_rows is not None else (
        100_000_000 if tab else (10_000_000 if tt else 100_000))
    return a


# this rank's split of its last timed window: host enqueue of the K steps, then the wait for them
WINDOW_SPLIT = {}


def _timed(ctx, fn, device_barrier=None):
    """Seconds for fn() (the K timed steps), max over ranks, bracketed by barrier + synchronize.

    End bracket on GPU ranks: with the in-kernel xGMI exchange active, ``device_barrier`` enqueues
    the exchange's own barrier (one wave per rank writes a tag into every peer's slot over xGMI
    and polls its own) right behind the steps, then the device is synchronized: no rank's clock
    stops before every rank finished its K steps.  Otherwise the process-group barrier (an RCCL
    4-byte all-reduce, or gloo on the host) brackets them."""
    import torch
    import torch.distributed as dist

    if ctx.device.type != "cuda":  # CPU plumbing config: steps are synchronous
        ctx.barrier()
        t0 = time.perf_counter()
        fn()
        ctx.barrier()
        dt_t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
        if ctx.is_distributed:
            dist.all_reduce(dt_t, op=dist.ReduceOp.MAX)
        return float(dt_t.item())
    # no cyclic-GC pass inside the window: the collector is paused for the K steps (the window
    # allocates almost nothing).  Measured on MI355X (profiles/bench_window_gc_r3.log): with it on,
    # the first window's completion wait was 0.34 ms instead of 0.10 ms in some processes; a
    # gc.collect() right before the window instead costs ~50 us of cold-cache enqueue.
    gc_paused = gc.isenabled()
    if gc_paused:
        gc.disable()
    torch.cuda.synchronize()
    ctx.barrier()
    torch.cuda.synchronize()
    _release_together(ctx)
    t0 = time.perf_counter()
    fn()
    t_enq = time.perf_counter()
    if device_barrier is not None and device_barrier():
        torch.cuda.synchronize()  # the xGMI barrier queued behind the steps on every rank
    elif ctx.backend == "nccl":
        ctx.barrier()  # an RCCL op queued behind the timed steps: the synchronize below covers both
        torch.cuda.synchronize()
    else:
        torch.cuda.synchronize()
        ctx.barrier()  # host-side (gloo) or a no-op at world size 1
    dt = time.perf_counter() - t0
    WINDOW_SPLIT["enqueue_us"] = round((t_enq - t0) * 1e6, 1)
    WINDOW_SPLIT["wait_us"] = round((dt - (t_enq - t0)) * 1e6, 1)
    if gc_paused:
        gc.enable()
    dt_t = torch.tensor([dt], dtype=torch.float64, device=ctx.device if ctx.backend == "nccl" else "cpu")
    if ctx.is_distributed:
        dist.all_reduce(dt_t, op=dist.ReduceOp.MAX)
    return float(dt_t.item())


def _release_together(ctx, margin_s: float = 0.002):
    """Leave the start barrier at one shared wall-clock instant on every rank.

    A barrier's release jitter (host wake-ups after the collective, a TCP round for gloo) puts
    ranks' first launches tens of microseconds apart, and the early ranks' first step then waits
    inside the timed window for the late one.  Rank 0 publishes a start time a couple of
    milliseconds ahead (longer than that jitter) and every rank spins on the node's shared clock
    until it: the window still contains all K steps of every rank, started together."""
    if not ctx.is_distributed:
        return
    t_go = ctx.broadcast_object(time.time() + margin_s if ctx.rank == 0 else None, src=0)
    while time.time() < t_go:
        pass


def _warmup(loop, n_items, warmup, loss):
    """The W untimed steps, issued as up to 8 launches through the same run_steps path the timed
    region uses, so its first launch finds the host launch path (Python, pybind, HIP runtime)
    warm: measured on MI355X, a single warmup launch leaves the first 20-step window ~25 us slower
    (tools/bench_window_probe.py).  Same steps, same data, same order as one launch."""
    calls = max(1, min(warmup, 8))
    first = 0
    exchange = getattr(loop, "xg", None) is not None or getattr(loop, "gx", None) is not None
    # replicas are identical before the first exchange launch: keep that state, so a timed-out
    # launch (the per-step peer all-reduce + Adam kernel can leave some blocks of a step applied)
    # is rolled back on every rank before the RCCL fallback re-syncs them
    snap = [t.clone() for t in (loop.p, loop.m, loop.v, loop.step_counter)] if exchange else None
    full_timeout = getattr(loop, "xg_timeout_s", None)
    if exchange:
        # the first exchange launch spins with the SHORT probe limit (a node whose peers cannot see
        # each other's writes then costs seconds, not the full training timeout, before the fallback)
        from dct_amd.parallel.xgmi import probe_timeout_s

        loop.xg_timeout_s, loop._bound, loop._fast_run = probe_timeout_s(), None, None
    for i in range(calls):
        k = warmup // calls + (1 if i < warmup % calls else 0)
        if k:
            loop.run_steps(n_items, k, loss, first_step=first)
            first += k
            if i == 0 and exchange:
                # the in-kernel exchange is checked after its FIRST launch: if peers cannot see
                # each other's writes, only that launch pays the spin timeout before the RCCL
                # fallback, not every warmup launch
                loop.xg_verify(fallback=True, snapshot=snap)
                snap = None
                # back to the full limit (launches rebound with it)
                loop.xg_timeout_s, loop._bound, loop._fast_run = full_timeout, None, None


def _params_in_sync(ctx, p):
    """DDP invariant: every rank holds the same parameters after the timed steps."""
    import torch
    import torch.distributed as dist

    if not ctx.is_distributed:
        return True
    ref = p.clone()
    ctx.broadcast_(ref, src=0)
    diff = torch.tensor([float((p - ref).abs().max())], device=ctx.device if ctx.backend == "nccl" else "cpu")
    dist.all_reduce(diff, op=dist.ReduceOp.MAX)
    return float(diff.item()) == 0.0


def setup_weather(a, ctx):
    import torch

    from dct_amd.data.synthetic import weather_tensors
    from dct_amd.models.mlp import build_mlp
    from dct_amd.trainer.engines import FusedMLPEngine, adam_hparams_from

    total_steps = a.warmup + a.steps
    rows = a.rows or int(math.ceil((total_steps + 8) * a.batch * ctx.world_size / 0.8)) + 1024
    X, Y = weather_tensors(rows, seed=0, dim=5)
    model = build_mlp(a.model, 5)
    adam = adam_hparams_from(model.configure_optimizers())
    if not FusedMLPEngine.applicable(model, ctx.device, a.batch):
        raise SystemExit("model/batch not supported by the fused engine")
    eng = FusedMLPEngine(model, ctx, a.batch, seed=42, adam=adam)
    n_train = int(0.8 * rows)
    perm = torch.randperm(rows, generator=torch.Generator().manual_seed(42))
    eng.attach_data(X, Y, perm[:n_train], perm[n_train:])
    return eng, 5


def setup_tabular(a, ctx):
    import torch

    from dct_amd.data.synthetic import make_tabular_device
    from dct_amd.models.mlp import build_mlp
    from dct_amd.trainer.engines import adam_hparams_from
    from dct_amd.trainer.graph_engine import GraphMLPEngine

    feats = 256
    rows = a.rows or 100_000_000
    X, Y = make_tabular_device(rows, feats, num_classes=2, device=ctx.device, dtype=torch.bfloat16, seed=0)
    model = build_mlp(a.model, feats)
    adam = adam_hparams_from(model.configure_optimizers())
    eng = GraphMLPEngine(model, ctx, a.batch, seed=42, adam=adam)
    n_train = int(0.8 * rows)
    perm = torch.randperm(rows, generator=torch.Generator().manual_seed(42))  # reference random_split
    eng.attach_data(X, Y, perm[:n_train], perm[n_train:])
    return eng, feats


class _StepLoop:
    """run_steps() over an AutogradEngine (one train_step per batch of the local shard)."""

    def __init__(self, eng, ctx):
        self.eng, self.ctx = eng, ctx

    def upload_epoch_indices(self, epoch, shuffle=True):
        local = self.eng.epoch_local_indices(len(self.eng.train_rows), epoch, shuffle)
        self.rows = self.eng.train_rows[local].to(self.eng.device)
        return self.rows.numel()

    def run_steps(self, n_items, steps, loss_out, first_step=0):
        # device-side batch loop: one captured graph per step, batch gather / loss record / cursor
        # on the device (trainer/engines.py AutogradEngine.run_device_steps)
        self.eng.run_device_steps(self.rows, first_step, steps, loss_out)

    def validate(self, limit=None):
        import torch

        eng = self.eng
        rows = eng.val_rows[: (limit or len(eng.val_rows))].to(eng.device)
        with torch.no_grad():
            eng.model.eval()
            logits = eng.model(eng.X[rows])
            loss = torch.nn.functional.cross_entropy(logits, eng.Y[rows])
            acc = (logits.argmax(1) == eng.Y[rows]).float().mean()
            eng.model.train()
        return float(loss), float(acc)


class _CpuLoop:
    """BASELINE config 1: the reference's execution model (CPU, batch 4, per-step autograd, gloo
    bucket all-reduce when distributed) on the AutogradEngine; batches sliced from the epoch's
    DistributedSampler shard like the Trainer does."""

    def __init__(self, eng):
        self.eng = eng

    def upload_epoch_indices(self, epoch, shuffle=True):
        self.rows = self.eng.train_rows[self.eng.epoch_local_indices(len(self.eng.train_rows), epoch, shuffle)]
        return self.rows.numel()

    def run_steps(self, n_items, steps, loss_out, first_step=0):
        B = self.eng.B
        for s in range(first_step, first_step + steps):
            loss_out[s] = self.eng.train_step(self.rows[s * B:(s + 1) * B], s)

    def validate(self, limit=None):
        import torch

        eng = self.eng
        rows = eng.val_rows[: (limit or len(eng.val_rows))]
        with torch.no_grad():
            eng.model.eval()
            logits = eng.model(eng.X[rows])
            loss = eng.model.compute_loss(logits, eng.Y[rows])
            acc = (logits.argmax(1) == eng.Y[rows]).float().mean()
            eng.model.train()
        return float(loss), float(acc)


def setup_cpu(a, ctx):
    import torch

    from dct_amd.data.synthetic import weather_tensors
    from dct_amd.models.mlp import build_mlp
    from dct_amd.trainer.engines import AutogradEngine

    rows = a.rows or int(math.ceil((a.warmup + a.steps + 8) * a.batch * ctx.world_size / 0.8)) + 1024
    X, Y = weather_tensors(rows, seed=0, dim=5)
    model = build_mlp(a.model, 5)
    eng = AutogradEngine(model, ctx, a.batch, seed=42)
    n_train = int(0.8 * rows)
    perm = torch.randperm(rows, generator=torch.Generator().manual_seed(42))
    eng.attach_data(X, Y, perm[:n_train], perm[n_train:])
    return eng, 5


def setup_transformer(a, ctx):
    import torch

    from dct_amd.data.synthetic import make_tabular_device
    from dct_amd.models import build_model
    from dct_amd.trainer.engines import AutogradEngine

    feats = 64
    rows = a.rows or 10_000_000
    X, Y = make_tabular_device(rows, feats, num_classes=2, device=ctx.device, dtype=torch.float32, seed=0)
    model = build_model("tabtransformer", feats, d_model=64, heads=4, layers=4, lr=1e-3)
    eng = AutogradEngine(model, ctx, a.batch, seed=42)
    n_train = int(0.8 * rows)
    perm = torch.randperm(rows, generator=torch.Generator().manual_seed(42))
    eng.attach_data(X, Y, perm[:n_train], perm[n_train:])
    return eng, feats


def _reserve_cus(a, eng):
    """--reserve-cus N: a compute stream masked to every CU but N and, if the engine has a native
    DDP bucket reducer, its comm stream masked to those N (the collectives then never share a CU with
    the step's kernels).  Returns the compute stream to run the measurement on."""
    import torch

    from dct_amd.ops._native import native

    nat = native()
    ncu = nat.device_cu_count()
    n = max(1, min(a.reserve_cus, ncu - 1))
    if a.reserve_pattern == "spread":
        cus = sorted({(i * ncu) // n for i in range(n)})
    elif a.reserve_pattern == "low":
        cus = list(range(n))
    else:
        cus = list(range(ncu - n, ncu))
    words = (ncu + 31) // 32
    comm = [0] * words
    for c in cus:
        comm[c // 32] |= 1 << (c % 32)
    full = [0xFFFFFFFF if 32 * (w + 1) <= ncu else (1 << (ncu - 32 * w)) - 1 for w in range(words)]
    compute = [f & ~c for f, c in zip(full, comm)]
    red = getattr(eng, "reducer", None)
    if red is not None and hasattr(red, "_r"):
        red._r.set_comm_cu_mask(comm)
    h = nat.cu_masked_stream(compute)
    return torch.cuda.ExternalStream(h, device=torch.cuda.current_device()), cus


def measure(a, ctx):
    """Set up a.model, run the W warmup steps, time exactly K steps; returns (result dict, ok)."""
    import contextlib

    import torch

    with contextlib.ExitStack() as stack:
        return _measure(a, ctx, stack)


def _measure(a, ctx, stack):
    import torch

    cpu = a.device == "cpu"
    tab = a.model in TABULAR
    tt = a.model in TRANSFORMER
    if cpu:
        if tab or tt:
            raise SystemExit("--device cpu runs the weather configs (BASELINE config 1)")
        eng, feats = setup_cpu(a, ctx)
        loop = _CpuLoop(eng)
    elif tt:
        eng, feats = setup_transformer(a, ctx)
        loop = _StepLoop(eng, ctx)
    else:
        eng, feats = (setup_tabular if tab else setup_weather)(a, ctx)
        loop = eng
    reserved = None
    if a.reserve_cus > 0 and not cpu:
        rs, reserved = _reserve_cus(a, eng)
        torch.cuda.synchronize()
        stack.enter_context(torch.cuda.stream(rs))
    total_steps = a.warmup + a.steps
    n_items = loop.upload_epoch_indices(0, shuffle=True)
    if total_steps * a.batch > n_items:
        raise SystemExit(f"dataset too small: {total_steps} steps x {a.batch} > {n_items} rows per rank")
    loss = torch.zeros(total_steps, dtype=torch.float32, device=ctx.device)

    # warmup (also builds / captures the step graphs outside the timed region)
    _warmup(loop, n_items, a.warmup, loss)
    if getattr(eng, "xg", None) is not None or getattr(eng, "gx", None) is not None:
        ok = eng.xg_verify(fallback=True)
        if ok and not _params_in_sync(ctx, eng.p):
            # the exchange completed but the replicas differ (should never happen): resync and
            # measure the RCCL path instead of reporting a broken DDP
            if ctx.rank == 0:
                print("[dct] replicas diverged under the in-kernel exchange; falling back to RCCL", flush=True)
            eng.xg_disable()
            ok = False
        if not ok:
            _warmup(eng, n_items, a.warmup, loss)  # re-warm on the RCCL path
    if not (tab or tt or cpu) and eng.ddp and eng.xg is None and eng.use_graph:
        eng._get_graph(n_items, min(eng.graph_chunk, a.steps), loss)
    dbar = getattr(eng, "device_barrier", None) if (ctx.is_distributed and not cpu) else None
    if dbar is not None and dbar():  # first launch of the barrier kernel (code-object load) untimed
        torch.cuda.synchronize()
    dt = _timed(ctx, lambda: loop.run_steps(n_items, a.steps, loss, first_step=a.warmup), device_barrier=dbar)

    xg_ok = (eng.xg_verify(fallback=True) if (getattr(eng, "xg", None) is not None
                                               or getattr(eng, "gx", None) is not None) else None)
    if cpu:
        engine_desc = "autograd(cpu)" + ("+gloo-bucket-allreduce" if ctx.is_distributed else "")
    elif tt:
        engine_desc = ("autograd(hip gemm/layernorm/attention)" + ("+rccl-bucket-allreduce" if ctx.is_distributed
                                                                    else "") + ("+hipgraph" if eng.graph_used else ""))
    elif tab:
        engine_desc = ("graph-mlp-executor(bf16 mfma gemm)" + ("+rccl-bucket-allreduce" if ctx.is_distributed else "")
                       + ("+hipgraph" if eng.graph_used else ""))
    elif eng.xg is not None or eng.ddp:
        engine_desc = eng.step_mode if (eng.xg is not None or eng.gx is not None) else (
            "fused+rccl-allreduce" + ("+update-then-grad" if eng.fused_update else "+adam")
            + ("+hipgraph" if eng.graph_used else ""))
    else:
        engine_desc = "fused-persistent"
    in_sync = _params_in_sync(ctx, eng.flat_p if (tt or cpu) else eng.p)
    losses = loss.cpu()
    finite = bool(torch.isfinite(losses).all())
    first_l = float(losses[: max(1, a.warmup // 10)].mean())
    last_l = float(losses[-max(1, a.steps // 10):].mean())
    eng.global_step = total_steps
    val_loss, val_acc = loop.validate(limit=(64 * a.batch) if (tab or tt) else None)

    samples = a.steps * a.batch * ctx.world_size
    sps = samples / dt
    ms_step = dt / a.steps * 1e3
    # epoch wall-clock for an --epoch-rows dataset at the measured step rate (train part)
    steps_per_epoch = math.ceil(math.ceil(int(0.8 * a.epoch_rows) / ctx.world_size) / a.batch)
    base = BASELINE_SAMPLES_PER_SEC.get(a.model)
    devices = _physical_devices(ctx)
    n_dev = len(set(devices)) if devices else 0
    out = {
        "metric": "samples/sec (whole node) for weather-MLP DDP",
        "value": round(sps, 1),
        "unit": "samples/s",
        "n_gpus": 0 if cpu else n_dev,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_step, 6),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": (round(sps / base, 2) if base else None),
        "dtype": "bf16" if (tab or tt) else "fp32",
        "data": "synthetic",
        "config": {
            "model": MODELS.get(a.model, a.model),
            "global_batch": a.batch * ctx.world_size,
            "per_rank_batch": a.batch,
            "seq_len": None,
            "parallelism": f"dp{ctx.world_size}" + ("-cpu-gloo" if cpu else ""),
            "optimizer": f"adam lr={(eng.optimizer.lr if (tt or cpu) else eng.adam['lr']):g}",
            "loss": "ce" if tt else (eng.model.loss_kind if cpu else eng.loss),
            "engine": engine_desc,
            "dataset_rows": int(eng.X.shape[0]),
            "seq_len_tokens": feats if tt else None,
            "features": feats,
            "baseline_ref": BASELINE_REF.get(a.model, "none (the reference publishes no number)"),
        },
        "extra": {
            "ranks": ctx.world_size,
            "ranks_per_device": (round(ctx.world_size / n_dev, 3) if n_dev else None),
            "us_per_step": round(ms_step * 1e3, 3),
            "window_rank0_us": dict(WINDOW_SPLIT),
            "epoch_wall_clock_s_train": round(steps_per_epoch * ms_step / 1e3, 6),  # derived
            "epoch_rows": a.epoch_rows,
            "loss_first": round(first_l, 4),
            "loss_last": round(last_l, 4),
            "val_loss": round(val_loss, 4),
            "val_acc": round(val_acc, 4),
            "losses_finite": finite,
            "params_in_sync": in_sync,
            "xgmi_exchange_ok": xg_ok,
            "reserved_cus": reserved,
            "device": torch.cuda.get_device_name(ctx.device) if not cpu else "cpu",
        },
    }
    if not (tab or tt or cpu) and not a.no_epoch and a.epoch_rows > 0:
        out["extra"].update(_measure_epoch(a, ctx, eng))
    if tab:
        flops = 6.0 * sum(eng.dims[i] * eng.dims[i + 1] for i in range(len(eng.dims) - 1)) * a.batch
        out["extra"]["model_tflops_per_gpu"] = round(flops / (ms_step * 1e-3) / 1e12, 1)
    if tt:
        out["extra"]["dtypes"] = {"gemm_and_attention_operands": "bf16", "accumulation": "fp32",
                                  "master_weights_and_adam": "fp32", "hbm_dataset": "fp32"}
    elif tab:
        out["extra"]["dtypes"] = {"gemm_operands": "bf16", "accumulation": "fp32",
                                  "master_weights_and_adam": "fp32", "hbm_dataset": "bf16"}
    return out, (finite and in_sync), eng


def _measure_epoch(a, ctx, eng):
    """One REAL epoch of the weather model after the step window (BASELINE metric "epoch
    wall-clock"; reference jobs/train_lightning_ddp.py:132 trains epochs of the 80 % split and
    validates after each): a fresh synthetic dataset of --epoch-rows rows (80/20 split) is attached,
    then the engine's own epoch path runs - host shuffle of this rank's DistributedSampler shard,
    index upload, every optimizer step of the shard (with the in-kernel exchange at W > 1), the
    loss read-back, and the full validation pass - bracketed by synchronize + barrier, max over
    ranks.  Reported next to the value derived from the timed window's step rate."""
    import torch
    import torch.distributed as dist

    from dct_amd.data.synthetic import weather_tensors

    X, Y = weather_tensors(a.epoch_rows, seed=1, dim=5)
    n_train = int(0.8 * a.epoch_rows)
    perm = torch.randperm(a.epoch_rows, generator=torch.Generator().manual_seed(7))
    eng.attach_data(X, Y, perm[:n_train], perm[n_train:])
    torch.cuda.synchronize()
    ctx.barrier()
    t0 = time.perf_counter()
    losses = eng.train_epoch(1, shuffle=True)
    l_host = losses.cpu()  # the trainer reads the epoch's losses back (epoch-end logging)
    t1 = time.perf_counter()
    val_loss, val_acc = eng.validate()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    ts = torch.tensor([t1 - t0, t2 - t0], dtype=torch.float64,
                      device=ctx.device if ctx.backend == "nccl" else "cpu")
    if ctx.is_distributed:
        dist.all_reduce(ts, op=dist.ReduceOp.MAX)
    tr, tot = (float(x) for x in ts.cpu())
    return {"epoch_wall_clock_s_measured": round(tot, 6), "epoch_train_s_measured": round(tr, 6),
            "epoch_steps_per_rank": int(l_host.numel()), "epoch_train_samples_per_s_measured":
            round(n_train / tr, 1), "epoch_loss_finite": bool(torch.isfinite(l_host).all()),
            "epoch_val_loss": round(val_loss, 4), "epoch_val_acc": round(val_acc, 4)}


def _physical_devices(ctx):
    """PCI bus id of every rank's GPU (rank order): n_gpus counts DISTINCT physical devices, so a
    rehearsal of several ranks on one GPU is never reported as a multi-GPU result."""
    if ctx.device.type != "cuda":
        return []
    from dct_amd.ops._native import native

    mine = native().pci_bus_id(ctx.device.index or 0)
    return ctx.all_gather_object(mine) if ctx.is_distributed else [mine]


def main():
    a = parse()
    # the DDP bucket reducer's device-side all-reduce timing (allreduce_ms in the trainer's logs) adds
    # two stamp kernels and two cross-stream edges per step: off for the timed step unless asked
    os.environ.setdefault("DCT_REDUCER_TIMING", "0")
    import copy

    import torch

    import dct_amd  # noqa: F401
    from dct_amd.parallel.dist import init_distributed, shutdown
    from dct_amd.trainer.trainer import seed_everything

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus and a.gpus > 1 and world == 1:
        raise SystemExit("--gpus > 1 must be launched with torch.distributed.run (one rank per GPU)")
    cpu = a.device == "cpu"
    ctx = init_distributed("cpu" if cpu else "gpu")
    seed_everything(42)
    out, ok, eng = measure(a, ctx)
    if not cpu and ctx.world_size > 1:
        from dct_amd.parallel.xgmi import peer_report

        bus, mat, peers_ok = peer_report(ctx)
        out["extra"]["xgmi_peers"] = {"rank_devices": bus, "can_access_peer": mat, "all_rank_pairs_ok": peers_ok}
    if (a.model == "weather-mlp-3x128" and not cpu and ctx.world_size == 1 and not a.no_reference_model):
        # the reference-exact model (jobs/train_lightning_ddp.py:57-62) with the same K / W
        del eng
        seed_everything(42)
        a_ref = copy.copy(a)
        a_ref.model = "weather"
        a_ref.no_epoch = True
        ref, ok_ref, _ = measure(a_ref, ctx)
        out["extra"].update({
            "reference_model": ref["config"]["model"],
            "reference_model_value": ref["value"],
            "reference_model_us_per_step": ref["extra"]["us_per_step"],
            "reference_model_vs_baseline": ref["vs_baseline"],
            "reference_model_engine": ref["config"]["engine"],
            "reference_model_loss_last": ref["extra"]["loss_last"],
        })
        ok = ok and ok_ref
    if ctx.rank == 0:
        print(json.dumps(out), flush=True)
    shutdown(ctx)
    return 0 if ok else 3


if __name__ == "__main__":
    sys.exit(main())
