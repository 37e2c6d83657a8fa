"""Bucketed gradient all-reduce (the DDP ``Reducer`` replacement).

Reference behaviour [lib]: ``DDPStrategy(find_unused_parameters=False)``
registers autograd hooks, packs gradients into buckets (first bucket 1 MiB, then 25 MiB) in
reverse parameter order and all-reduces each bucket as soon as all its gradients are ready,
overlapping communication with the rest of backward; gradients are averaged over ranks.

Here every parameter's ``.grad`` is a VIEW into one flat fp32 gradient buffer laid out in
parameter order, so a bucket (a run of consecutive parameters taken from the end) is a
contiguous slice of that buffer: there is no copy into / out of bucket storage.  Bucket
sizes default to 1 MiB first / 8 MiB after (``DistConfig``): on MI355X the ring all-reduce
runs per xGMI link (~153 GB/s x 7 links), 8 MiB buckets already sit in RCCL's bandwidth
regime while the 3.4 M-parameter 4x1024 config still gets 2 buckets to overlap.

Two executors with one interface:
  * ``NativeBucketReducer`` - the C++ ``BucketReducer`` (csrc/runtime.cpp): RCCL ``ncclAvg``
    all-reduces on a dedicated comm HIP stream, ordered after the producing backward kernels
    by HIP events, joined into the compute stream once at ``finalize``.
  * ``TorchBucketReducer`` - ``torch.distributed`` async all-reduces (gloo on CPU: the
    plumbing config of BASELINE.json; or nccl), averaged at ``finalize``.  With
    ``host_staging`` (gloo process group, gradients on the GPU: several ranks sharing one device,
    where RCCL refuses to run) each bucket goes through host memory.
"""
from __future__ import annotations

import time
from dataclasses import dataclass
from typing import List, Sequence, Tuple

import torch
import torch.distributed as dist


@dataclass
class BucketPlan:
    offsets: List[int]  # element offset of each bucket in the flat buffer
    counts: List[int]  # elements per bucket
    param_bucket: List[int]  # bucket index of each parameter (parameter order)
    param_offsets: List[int]  # element offset of each parameter


def plan_buckets(numels: Sequence[int], elem_bytes: int = 4, bucket_cap_bytes: int = 8 << 20,
                 first_bucket_bytes: int = 1 << 20, split_before: Sequence[int] = ()) -> BucketPlan:
    """Buckets of consecutive parameters filled in REVERSE parameter order (backward order).
    ``split_before``: parameter indices that close the bucket being filled before they are added
    (a model whose gradients become ready in groups - the TabTransformer's grouped dW launches -
    aligns buckets with those groups, so each bucket launches as its group finishes).  With
    ``split_before`` the byte caps are ignored: buckets close ONLY at group boundaries.  A group's
    weight gradients are written by one deferred grouped launch issued inside the backward of the
    group's lowest block, so a bucket holding only part of a group would complete (its hooks fire)
    and be all-reduced before those gradients exist."""
    splits = set(int(i) for i in split_before)
    offs, acc = [], 0
    for n in numels:
        offs.append(acc)
        acc += int(n)
    buckets: List[Tuple[int, int]] = []  # (first param idx, last param idx) in reverse fill order
    param_bucket = [0] * len(numels)
    cap = first_bucket_bytes
    cur_bytes = 0
    cur: List[int] = []
    for i in reversed(range(len(numels))):
        nb = int(numels[i]) * elem_bytes
        if cur and (i in splits or (not splits and cur_bytes + nb > cap)):
            buckets.append((cur[-1], cur[0]))
            cur, cur_bytes = [], 0
            cap = bucket_cap_bytes
        cur.append(i)
        cur_bytes += nb
    if cur:
        buckets.append((cur[-1], cur[0]))
    offsets, counts = [], []
    for b, (lo, hi) in enumerate(buckets):
        for i in range(lo, hi + 1):
            param_bucket[i] = b
        offsets.append(offs[lo])
        counts.append(offs[hi] + int(numels[hi]) - offs[lo])
    return BucketPlan(offsets, counts, param_bucket, offs)


class TorchBucketReducer:
    def __init__(self, flat_grad: torch.Tensor, plan: BucketPlan, world_size: int, host_staging: bool = False):
        self.flat = flat_grad
        self.plan = plan
        self.world = world_size
        self.host_staging = bool(host_staging)
        self.wait_s = 0.0  # exposed all-reduce wait, accumulated (the Trainer's allreduce_ms)
        self.expected = [0] * len(plan.offsets)
        for b in plan.param_bucket:
            self.expected[b] += 1
        self.prepare()

    def prepare(self):
        self.pending = [0] * len(self.plan.offsets)
        self.works = []
        self.next = 0

    def _launch(self, b: int):
        off, cnt = self.plan.offsets[b], self.plan.counts[b]
        view = self.flat[off: off + cnt]
        if self.world > 1:
            buf = view.cpu() if self.host_staging else view  # D2H copy waits for the producing kernels
            self.works.append((dist.all_reduce(buf, op=dist.ReduceOp.SUM, async_op=True), view, buf))

    def mark_ready(self, param_idx: int, stream=None) -> int:
        b = self.plan.param_bucket[param_idx]
        self.pending[b] += 1
        if self.pending[b] > self.expected[b]:
            raise RuntimeError("parameter marked ready twice in one step")
        n = 0
        while self.next < len(self.expected) and self.pending[self.next] == self.expected[self.next]:
            self._launch(self.next)
            self.next += 1
            n += 1
        return n

    def finalize(self, stream=None):
        while self.next < len(self.expected):
            self._launch(self.next)
            self.next += 1
        t0 = time.perf_counter()
        for w, view, buf in self.works:
            w.wait()
            buf.div_(self.world)
            if buf is not view:
                view.copy_(buf)
        self.works = []
        self.wait_s += time.perf_counter() - t0  # all-reduce time NOT hidden behind the backward

    @property
    def num_buckets(self):
        return len(self.plan.offsets)


class NativeBucketReducer:
    """The C++ ``BucketReducer`` (RCCL on a comm stream).  ``timing=True`` adds device-side stamps
    (one-thread kernels, so they survive HIP graph capture): per step the all-reduce SPAN (first
    bucket's start -> last bucket done, on the comm stream) and the EXPOSED part (end of backward
    on the compute stream -> last bucket done), read as ``allreduce_ms()``; ``check=True``
    (``DCT_DEBUG=1``) also verifies on the device that the compute stream joined the comm stream
    before the optimizer (``ordering_violations``).  ``defer_launch``: mark_ready only counts and
    every bucket launches at ``finalize`` - for backward passes whose weight gradients are issued
    after the hooks fire (the TabTransformer's grouped deferred dW GEMMs)."""

    def __init__(self, comm, flat_grad: torch.Tensor, plan: BucketPlan, timing: bool = False, check: bool = False):
        from ..ops._native import native

        nat = native()
        if flat_grad.dtype != torch.float32 or not flat_grad.is_cuda:
            raise ValueError("native reducer expects a cuda fp32 flat gradient buffer")
        self.flat = flat_grad
        self.plan = plan
        self._r = nat.BucketReducer(comm, flat_grad.data_ptr(), list(plan.offsets), list(plan.counts),
                                    list(plan.param_bucket), nat.DT_F32, nat.OP_AVG)
        self.timing = bool(timing or check)
        if self.timing:
            self._r.enable_timing(bool(check))
        self.defer_launch = False
        self._deferred: List[int] = []
        self.hook_launches = 0  # buckets launched from backward hooks (before finalize), cumulative

    def prepare(self):
        self._deferred = []
        self._r.prepare()

    def mark_ready(self, param_idx: int, stream=None) -> int:
        if self.defer_launch:
            self._deferred.append(param_idx)
            return 0
        s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        n = self._r.mark_ready(param_idx, s)
        self.hook_launches += n
        return n

    def finalize(self, stream=None):
        s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        for i in self._deferred:  # every gradient producer is enqueued by now (grouped dW included)
            self._r.mark_ready(i, s)
        self._deferred = []
        self._r.finalize(s)

    @property
    def launched(self) -> int:
        return self._r.launched

    @property
    def launched_before_finalize(self) -> int:
        return self._r.launched_before_finalize

    @property
    def num_buckets(self):
        return self._r.num_buckets

    def allreduce_ms(self, reset: bool = True):
        """(span_ms, exposed_ms, steps, ordering_violations) accumulated on the device since the
        last reset (synchronising read); None without timing."""
        if not self.timing:
            return None
        span, exposed, steps, bad = self._r.read_timing()
        if reset:
            self._r.reset_timing()
        return span, exposed, int(steps), int(bad)

    # the Trainer's allreduce_ms contract (seconds of exposed all-reduce wait, reset by assigning 0)
    @property
    def wait_s(self) -> float:
        t = self.allreduce_ms(reset=False)
        return 0.0 if t is None else t[1] / 1e3

    @wait_s.setter
    def wait_s(self, value: float):
        if value == 0.0 and self.timing:
            self._r.reset_timing()
