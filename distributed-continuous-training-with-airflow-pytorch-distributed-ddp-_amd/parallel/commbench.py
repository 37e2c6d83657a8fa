"""All-reduce microbenchmark (``all_reduce_perf`` style) for sizing DDP gradient buckets.

Why: SURVEY §5.8 asks for busBW measured on the actual MI355X fabric before bucket sizes are
fixed.  The reference's traffic is one 2,056-byte gradient bucket + a 4-byte loss per step over
gloo/TCP (jobs/train_lightning_ddp.py:136 -> torch Reducer); here the same
collective runs on RCCL over xGMI, where the 8 GPUs are fully connected by 7 point-to-point links
(~153 GB/s each).  Small messages are latency bound (one LL-protocol hop), large ones are
link-bandwidth bound, and the knee between the two is where ``DistConfig.bucket_cap_mb`` belongs.

One rank per device (torchrun), three paths over the same buffers:
  * ``torch``  - ``torch.distributed.all_reduce`` on the process group (RCCL on GPU, gloo on CPU);
  * ``native`` - the C++ runtime's RCCL communicator (csrc/runtime.cpp ``Comm``) on the current
    HIP stream, the path ``NativeBucketReducer`` uses;
  * ``graph``  - ``native`` captured into a HIP graph (csrc/runtime.cpp ``StreamGraph``) and
    replayed, the launch-overhead-free path of the captured training steps.
Each size is checked once for correctness (rank r contributes r + 1; every element must equal
W (W + 1) / 2) before it is timed.  Times are the max over ranks; ``algbw = bytes / t`` and
``busbw = algbw * 2 (W - 1) / W`` (the ring all-reduce's per-link traffic, nccl-tests convention).
"""
from __future__ import annotations

import json
import os
import time
from typing import Dict, List, Optional, Sequence

import torch
import torch.distributed as dist

from .dist import DistContext

_DTYPES = {"fp32": torch.float32, "bf16": torch.bfloat16}


def sizes_pow2(min_bytes: int, max_bytes: int) -> List[int]:
    out, s = [], max(4, int(min_bytes))
    while s <= max_bytes:
        out.append(s)
        s *= 2
    return out


def bus_factor(world: int) -> float:
    return 2.0 * (world - 1) / world if world > 1 else 0.0


def _native_comm(ctx: DistContext):
    from ..ops._native import native
    from .dist import init_native_comm

    if ctx.is_distributed:
        return init_native_comm(ctx)
    nat = native()  # W = 1: a single-rank communicator still exercises the RCCL launch path
    # (the benchmark's point, so the Comm must not skip the identity collective - DCT_RCCL_ONE_RANK)
    prev = os.environ.get("DCT_RCCL_ONE_RANK")
    os.environ["DCT_RCCL_ONE_RANK"] = "1"
    try:
        return nat.Comm(nat.comm_unique_id(), 1, 0, ctx.device.index)
    finally:
        if prev is None:
            os.environ.pop("DCT_RCCL_ONE_RANK", None)
        else:
            os.environ["DCT_RCCL_ONE_RANK"] = prev
        nat.reload_knobs()


def _max_over_ranks(ctx: DistContext, x: float) -> float:
    if not ctx.is_distributed:
        return x
    dev = ctx.device if ctx.backend == "nccl" else torch.device("cpu")
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _sync(ctx: DistContext):
    if ctx.device.type == "cuda":
        torch.cuda.synchronize(ctx.device)


def run(ctx: DistContext, sizes: Sequence[int], dtype: str = "fp32", paths: Sequence[str] = ("torch",),
        iters: int = 20, warmup: int = 5, check: bool = True) -> List[Dict]:
    """Collective over all ranks; returns one record per (path, size) on every rank."""
    if ctx.device.type == "cuda":  # a capturable (non-legacy) stream for every path
        with torch.cuda.stream(torch.cuda.Stream(ctx.device)):
            return _run(ctx, sizes, dtype, paths, iters, warmup, check)
    return _run(ctx, sizes, dtype, paths, iters, warmup, check)


def _run(ctx, sizes, dtype, paths, iters, warmup, check):
    dt = _DTYPES[dtype]
    esize = torch.tensor([], dtype=dt).element_size()
    W = ctx.world_size
    records = []
    comm = None
    if any(p in ("native", "graph") for p in paths):
        if ctx.device.type != "cuda":
            raise RuntimeError("native / graph paths need a HIP device (RCCL)")
        comm = _native_comm(ctx)
    from ..ops._native import native as _nat

    for path in paths:
        for nbytes in sizes:
            count = max(1, nbytes // esize)
            buf = torch.full((count,), float(ctx.rank + 1), dtype=dt, device=ctx.device)
            stream = torch.cuda.current_stream(ctx.device).cuda_stream if ctx.device.type == "cuda" else 0
            code = _nat().DT_BF16 if (comm is not None and dt == torch.bfloat16) else (
                _nat().DT_F32 if comm is not None else None)

            def once():
                if path == "torch":
                    if ctx.is_distributed:
                        dist.all_reduce(buf)
                else:
                    comm.allreduce(buf.data_ptr(), count, code, _nat().OP_SUM, stream)

            ok = True
            if check:
                once()
                _sync(ctx)
                want = W * (W + 1) / 2
                ok = bool((buf.float() == want).all().item())
                ok = _max_over_ranks(ctx, 0.0 if ok else 1.0) == 0.0
            graph = None
            if path == "graph":
                graph = _nat().StreamGraph()
                graph.begin(stream)
                for _ in range(iters):
                    once()
                graph.end(stream)
            for _ in range(warmup):
                if graph is not None:
                    graph.replay(stream)
                else:
                    once()
            _sync(ctx)
            ctx.barrier()
            _sync(ctx)
            t0 = time.perf_counter()
            if graph is not None:
                graph.replay(stream)
            else:
                for _ in range(iters):
                    once()
            _sync(ctx)
            dt_s = _max_over_ranks(ctx, time.perf_counter() - t0) / iters
            bytes_ = count * esize
            algbw = bytes_ / dt_s / 1e9
            records.append({"path": path, "bytes": bytes_, "dtype": dtype, "world": W, "us": round(dt_s * 1e6, 3),
                            "algbw_GBps": round(algbw, 3), "busbw_GBps": round(algbw * bus_factor(W), 3),
                            "correct": ok})
            del graph
    return records


def bucket_knee(records: Sequence[Dict], path: str, fraction: float = 0.8) -> Optional[int]:
    """Smallest size reaching ``fraction`` of the path's best bus bandwidth: buckets at least this
    large are bandwidth bound; smaller ones pay latency per bucket.  None at W = 1 (no traffic)."""
    rs = [r for r in records if r["path"] == path]
    if not rs or rs[0]["world"] < 2:
        return None
    key = "busbw_GBps"
    best = max(r[key] for r in rs)
    if best <= 0:
        return None
    for r in sorted(rs, key=lambda r: r["bytes"]):
        if r[key] >= fraction * best:
            return r["bytes"]
    return None


def format_table(records: Sequence[Dict]) -> str:
    lines = [f"{'path':>7} {'bytes':>12} {'us':>10} {'algbw GB/s':>11} {'busbw GB/s':>11} ok"]
    for r in records:
        lines.append(f"{r['path']:>7} {r['bytes']:>12} {r['us']:>10.2f} {r['algbw_GBps']:>11.2f} "
                     f"{r['busbw_GBps']:>11.2f} {'y' if r['correct'] else 'N'}")
    return "\n".join(lines)


def main(argv=None) -> int:
    import argparse

    from .dist import init_distributed, shutdown

    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("--min-bytes", type=int, default=8)
    p.add_argument("--max-bytes", type=int, default=64 << 20)
    p.add_argument("--dtype", choices=sorted(_DTYPES), default="fp32")
    p.add_argument("--paths", default="torch,native,graph", help="comma list of torch | native | graph")
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--accelerator", default="auto", help="gpu | cpu | auto")
    p.add_argument("--json", action="store_true", help="one JSON line per record instead of a table")
    a = p.parse_args(argv)
    ctx = init_distributed(a.accelerator)
    paths = [s for s in a.paths.split(",") if s]
    if ctx.device.type != "cuda":
        paths = [s for s in paths if s == "torch"]
    recs = run(ctx, sizes_pow2(a.min_bytes, a.max_bytes), a.dtype, paths, a.iters, a.warmup)
    if ctx.rank == 0:
        if a.json:
            for r in recs:
                print(json.dumps(r), flush=True)
        else:
            print(format_table(recs), flush=True)
        if ctx.world_size == 1:
            print("# W = 1: no peer traffic (RCCL's single-rank in-place all-reduce is a no-op); the times are "
                  "per-call launch + enqueue latency", flush=True)
        for path in paths:
            k = bucket_knee(recs, path)
            if k is not None:
                print(f"# {path}: bandwidth knee (80% of best busbw) at {k} bytes", flush=True)
    bad = [r for r in recs if not r["correct"]]
    shutdown(ctx)
    return 1 if bad else 0
