"""``GraphMLPEngine``: the wide-MLP data-parallel step issued by ONE native step executor.

For MLPs too wide for the single-CU fused kernels (the BASELINE "100M rows x 256 features,
4-layer MLP-1024h" config) the step is issued by the native ``MlpStepExecutor``
(csrc/mlp_executor.cpp): HBM-resident bf16 dataset -> device batch gather -> bf16 MFMA GEMMs
with fused bias/activation epilogues -> fused loss + dlogits -> backward GEMMs writing fp32
gradients straight into the flat DDP bucket buffer -> RCCL ncclAvg per bucket as soon as the
layer's dW is enqueued -> fused flat Adam with bf16 shadow weights.  The batch cursor, Adam step
and loss slot live in device memory, so the step needs no host round trip: by default the C++
executor simply enqueues it for every batch (11 launches from C++ stay ahead of the GPU: 171-173
us/step), and ``use_graph=True`` captures it once into a hipGraph replayed per full batch (175.5-
176.9 us/step on ROCm 7: every replay starts ~8 us after the previous one ends; 8 steps per graph
were slower still, profiles/tabular_graph_steps_ab_r2.log, profiles/mlp_graph_vs_eager_ab_r4.log).
The partial last batch (reference ``drop_last=False``) runs with its real row count.

Gradient buffer ``g`` (flat, parameter order + the loss slot): with a DDP reducer it holds every
averaged gradient after a step.  WITHOUT one (world size 1), up to three layers hand their
split-K dW slices straight to the Adam kernel (``exe.partial_layers``), so those layers' weight
ranges of ``g`` stay ZERO - read gradients through a reducer run (``DCT_FORCE_DDP=1``) or
``DCT_DW_INTO_ADAM=0`` for debugging / grad-norm checks.  A batch too short for the planned
slices (an epoch's partial last batch) falls back to ``g`` for that step
(``exe.part_fallbacks`` counts those steps).

Reference semantics kept: DistributedSampler sharding, batch-mean loss averaged over ranks
(``sync_dist``), Adam(lr) on fp32 master weights, checkpoints in the Lightning layout (the flat
buffers are copied back into the nn.Module for saving).
"""
from __future__ import annotations

import math
import os
from typing import Dict, Optional, Tuple

import torch

from ..data.sampler import distributed_indices
from ..ops._native import native
from ..ops.optim import FlatAdam
from ..parallel.dist import DistContext, init_native_comm
from ..parallel.reducer import NativeBucketReducer, plan_buckets
from ..utils.debug import enabled as debug_enabled
from ..utils.debug import reducer_timing_enabled

ACT_IDS = {"relu": 1, "gelu": 2}
LOSS_IDS = {"ce": 0, "mse": 1}


def layer_bucket_splits(numels, bucket_bytes: int, elem_bytes: int = 4):
    """Bucket boundaries of the executor's DDP reducer at LAYER boundaries (plan_buckets
    ``split_before``).  The executor marks a layer's weight and bias ready right after its dW GEMM,
    so a bucket that closes mid-layer gains nothing, and what matters for overlap is the size of the
    LAST bucket - its all-reduce runs after the whole backward.  Layers are taken from the top and
    a bucket closes once it holds >= min(bucket_bytes, 2 MiB): for 256-1024-1024-1024-2 that is
    {head + layer 2} (4 MB), {layer 1} (4 MB), {layer 0} (1 MB), instead of the byte-capped
    {head} / {layer 2} / {layer 1 + layer 0} whose last 5 MB all-reduce was fully exposed."""
    L = len(numels) // 2
    target = min(int(bucket_bytes), 2 << 20)
    splits, acc = [], 0
    for layer in range(L - 1, 0, -1):
        acc += (numels[2 * layer] + numels[2 * layer + 1]) * elem_bytes
        if acc >= target:
            splits.append(2 * (layer - 1) + 1)  # the next parameter down: bias of the layer below
            acc = 0
    return splits


class GraphMLPEngine:
    name = "graph"
    epoch_engine = True  # runs whole epochs on device; the Trainer reads back per-step losses

    @staticmethod
    def applicable(model, device: torch.device, batch_size: int) -> bool:
        if device.type != "cuda" or not hasattr(model, "fused_spec"):
            return False
        spec = model.fused_spec()
        return spec["dropout"] == 0.0 and spec["dims"][0] % 8 == 0 and batch_size >= 1

    def __init__(self, model, ctx: DistContext, batch_size: int, seed: int, adam: Dict,
                 bucket_cap_bytes: int = 8 << 20, first_bucket_bytes: int = 1 << 20, use_graph: Optional[bool] = None):
        native().reload_knobs()  # bind time: the native launchers' DCT_* knobs
        self.model = model
        self.ctx = ctx
        self.B = int(batch_size)
        self.seed = int(seed)
        self.global_step = 0
        spec = model.fused_spec()
        if spec["dropout"] != 0.0:
            raise ValueError("graph engine: dropout is not supported (use the autograd engine)")
        self.dims = list(spec["dims"])
        self.loss = spec["loss"]
        self.adam = adam
        self.device = dev = ctx.device
        if use_graph is None:
            use_graph = False  # (the eager C++ enqueue beats the replays; use_graph=True for A/Bs)
        self.use_graph = use_graph
        L = len(self.dims) - 1
        self.L = L
        self.numels = []
        for lin in model.linear_layers():
            self.numels += [lin.weight.numel(), lin.bias.numel()]
        self.P = sum(self.numels)
        self.p = torch.cat([t.detach().float().reshape(-1) for t in self._linear_params()]).to(dev)
        self.p_bf16 = self.p.to(torch.bfloat16)
        self.g = torch.zeros(self.P + 1, dtype=torch.float32, device=dev)
        self.m = torch.zeros_like(self.p)
        self.v = torch.zeros_like(self.p)
        self.step_counter = torch.zeros(1, dtype=torch.int32, device=dev)
        self.cursor = torch.zeros(1, dtype=torch.int32, device=dev)
        self.stats = torch.zeros(2, dtype=torch.float32, device=dev)
        B = self.B
        self.acts = [torch.empty(B, d, dtype=torch.bfloat16, device=dev) for d in self.dims]
        dmax = max(self.dims)
        self.dz = [torch.empty(B, dmax, dtype=torch.bfloat16, device=dev) for _ in range(2)]
        self.ybuf = torch.empty(B, dtype=torch.int32, device=dev)
        nat = native()
        self.comm = None
        self.reducer = None
        # DCT_FORCE_DDP=1 at world size 1: the DDP step (one-rank RCCL communicator, bucket reducer,
        # per-layer bucket launches, two-pass split-K dW into g) on one GPU - tested and measured
        # against the no-reducer step (split-K slices summed inside Adam)
        forced = not ctx.is_distributed and os.environ.get("DCT_FORCE_DDP", "0") == "1"
        if ctx.is_distributed or forced:
            if ctx.is_distributed and ctx.backend != "nccl":
                raise RuntimeError("graph engine needs the RCCL (nccl) backend for multi-rank runs")
            self.comm = init_native_comm(ctx) if ctx.is_distributed else nat.Comm(nat.comm_unique_id(), 1, 0,
                                                                                   dev.index or 0)
            s = torch.cuda.current_stream().cuda_stream
            self.comm.broadcast(self.p.data_ptr(), self.P, nat.DT_F32, 0, s)  # DDP _sync_module_states
            self.p_bf16.copy_(self.p)
            plan = plan_buckets(self.numels + [1], bucket_cap_bytes=bucket_cap_bytes,
                                first_bucket_bytes=first_bucket_bytes,
                                split_before=layer_bucket_splits(self.numels, bucket_cap_bytes))
            self.bucket_plan = plan
            self.reducer = NativeBucketReducer(self.comm, self.g, plan,
                                               timing=reducer_timing_enabled(),
                                               check=debug_enabled())
        self.exe = nat.MlpStepExecutor(self.dims, B, ACT_IDS["relu"], LOSS_IDS[self.loss], self.p.data_ptr(),
                                       self.p_bf16.data_ptr(), self.g.data_ptr(), self.m.data_ptr(),
                                       self.v.data_ptr(), [a.data_ptr() for a in self.acts], [],
                                       self.dz[0].data_ptr(), self.dz[1].data_ptr(), self.ybuf.data_ptr(),
                                       self.stats.data_ptr(), self.reducer._r if self.reducer is not None else None)
        a = adam
        self.exe.set_adam(a["lr"], a["betas"][0], a["betas"][1], a["eps"], a["weight_decay"], 0)
        self._graph = None
        self._graph_key = None
        self.graph_used = False

    # ------------------------------------------------------------------ params
    def _linear_params(self):
        out = []
        for lin in self.model.linear_layers():
            out += [lin.weight, lin.bias]
        return out

    def sync_to_model(self):
        flat = self.p.detach().cpu()
        off = 0
        with torch.no_grad():
            for t in self._linear_params():
                n = t.numel()
                t.copy_(flat[off: off + n].view_as(t))
                off += n

    def load_from_model(self):
        self.p.copy_(torch.cat([t.detach().float().reshape(-1) for t in self._linear_params()]).to(self.device))
        self.p_bf16.copy_(self.p)

    def optimizer_state_dict(self) -> Dict:
        shapes = [t.shape for t in self._linear_params()]
        fa = FlatAdam(self.p, self.p, shapes, lr=self.adam["lr"], betas=self.adam["betas"], eps=self.adam["eps"],
                      weight_decay=self.adam["weight_decay"])
        fa.m, fa.v = self.m, self.v
        fa.step_count = self.global_step
        return fa.state_dict()

    def load_optimizer_state(self, sd: Dict, global_step: int):
        shapes = [t.shape for t in self._linear_params()]
        fa = FlatAdam(self.p, self.p, shapes, **self.adam)
        fa.m, fa.v = self.m, self.v
        fa.load_state_dict(sd)
        self.global_step = global_step
        self.step_counter.fill_(int(fa.step_count))

    # ------------------------------------------------------------------ data
    def attach_data(self, X: torch.Tensor, Y: torch.Tensor, train_rows: torch.Tensor, val_rows: torch.Tensor):
        if X.shape[1] != self.dims[0]:
            raise ValueError(f"dataset has {X.shape[1]} features, model expects {self.dims[0]}")
        dev = self.device
        self.X = X if (X.is_cuda and X.dtype == torch.bfloat16 and X.is_contiguous()) else \
            X.to(dev, non_blocking=True).to(torch.bfloat16).contiguous()
        self.Y = Y if (Y.is_cuda and Y.dtype == torch.int32) else Y.to(dev).to(torch.int32).contiguous()
        n = X.shape[0]
        self.train_rows = train_rows.to(torch.int64)
        self.val_rows = val_rows.to(torch.int64)
        for rows in (self.train_rows, self.val_rows):
            if rows.numel() and (int(rows.min()) < 0 or int(rows.max()) >= n):
                raise ValueError("split indices out of range")
        n_local = math.ceil(len(self.train_rows) / self.ctx.world_size)
        self.idx = torch.zeros(max(1, n_local), dtype=torch.int32, device=dev)
        self.val_idx = torch.zeros(max(1, math.ceil(max(1, len(self.val_rows)) / self.ctx.world_size)),
                                   dtype=torch.int32, device=dev)
        self.row_bytes = self.dims[0] * 2

    def steps_per_epoch(self) -> int:
        n_local = math.ceil(len(self.train_rows) / self.ctx.world_size)
        return math.ceil(n_local / self.B)

    def upload_epoch_indices(self, epoch: int, shuffle: bool = True) -> int:
        local = distributed_indices(len(self.train_rows), self.ctx.world_size, self.ctx.rank, shuffle=shuffle,
                                    seed=self.seed, epoch=epoch)
        rows = self.train_rows[local].to(torch.int32)
        # pinned source + one stream sync per epoch: an async copy from PAGEABLE host memory is not
        # reliably ordered before the hipGraphLaunch replays that read idx (observed on ROCm 7:
        # replays of epoch >= 1 read a partly stale index list -> run-to-run divergence)
        self.idx[: rows.numel()].copy_(rows.pin_memory(), non_blocking=True)
        torch.cuda.current_stream(self.device).synchronize()
        return rows.numel()

    # ------------------------------------------------------------------ train
    def _step(self, n_items: int, loss_out: torch.Tensor, rows: int):
        self.exe.step(self.X.data_ptr(), self.row_bytes, self.Y.data_ptr(), self.idx.data_ptr(), int(n_items),
                      self.cursor.data_ptr(), self.step_counter.data_ptr(), loss_out.data_ptr(), loss_out.numel(),
                      int(rows), torch.cuda.current_stream().cuda_stream)

    def _get_graph(self, n_items: int, loss_out: torch.Tensor):
        key = (n_items, loss_out.data_ptr(), loss_out.numel())
        if self._graph_key == key:
            return self._graph
        # warm step (kernel attributes, RCCL channels) outside the capture, then roll back
        state = (self.p, self.p_bf16, self.m, self.v, self.g, self.step_counter, self.cursor, loss_out)
        saved = [t.clone() for t in state]
        self._step(n_items, loss_out, self.B)
        torch.cuda.synchronize(self.device)
        for t, sv in zip(state, saved):
            t.copy_(sv)
        g = torch.cuda.CUDAGraph()
        try:
            s = torch.cuda.Stream(self.device)
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                    self._step(n_items, loss_out, self.B)
            torch.cuda.current_stream().wait_stream(s)
        except Exception as e:  # noqa: BLE001 - eager steps stay correct
            print(f"[dct] graph capture of the MLP step failed ({e!r}); running eagerly", flush=True)
            g = None
        torch.cuda.synchronize(self.device)
        for t, sv in zip(state, saved):
            t.copy_(sv)
        self._graph, self._graph_key = g, key
        return g

    def run_steps(self, n_items: int, steps: int, loss_out: torch.Tensor, first_step: int = 0):
        """Steps [first_step, first_step+steps) of the epoch; loss_out[first_step + s] = reduced loss."""
        if steps <= 0:
            return
        n_full = n_items // self.B
        if first_step + steps > math.ceil(n_items / self.B) or loss_out.numel() < first_step + steps:
            raise ValueError("step range exceeds the epoch's batches / loss buffer")
        self.cursor.fill_(first_step)
        full_steps = max(0, min(first_step + steps, n_full) - first_step)
        g = self._get_graph(n_items, loss_out) if (self.use_graph and full_steps > 0) else None
        for _ in range(full_steps):
            if g is not None:
                g.replay()
            else:
                self._step(n_items, loss_out, self.B)
        if g is not None and full_steps:
            self.graph_used = True
        if first_step + steps > n_full:  # partial last batch, eager with its true row count
            self._step(n_items, loss_out, n_items - n_full * self.B)

    def train_epoch(self, epoch: int, shuffle: bool = True) -> torch.Tensor:
        n_items = self.upload_epoch_indices(epoch, shuffle)
        steps = math.ceil(n_items / self.B)
        buf = getattr(self, "_loss_buf", None)
        if buf is None or buf.numel() < steps:
            self._loss_buf = buf = torch.zeros(max(1, steps), dtype=torch.float32, device=self.device)
            self._graph_key = None
        self.run_steps(n_items, steps, buf)
        self.global_step += steps
        return buf[:steps]

    # ------------------------------------------------------------------ eval
    def validate(self, rows: Optional[torch.Tensor] = None, limit: Optional[int] = None) -> Tuple[float, float]:
        rows = self.val_rows if rows is None else rows
        local = distributed_indices(len(rows), self.ctx.world_size, self.ctx.rank, shuffle=False)
        if limit is not None:
            local = local[:limit]
        r = rows[local].to(torch.int32)
        n = r.numel()
        if n == 0:
            return float("nan"), float("nan")
        if n > self.val_idx.numel():
            self.val_idx = torch.zeros(n, dtype=torch.int32, device=self.device)
        self.val_idx[:n].copy_(r.to(self.device))
        cur = torch.zeros(1, dtype=torch.int32, device=self.device)
        acc = torch.zeros(2, dtype=torch.float32, device=self.device)
        stream = torch.cuda.current_stream().cuda_stream
        for b in range(math.ceil(n / self.B)):
            rows_b = min(self.B, n - b * self.B)
            self.exe.eval_batch(self.X.data_ptr(), self.row_bytes, self.Y.data_ptr(), self.val_idx.data_ptr(), n,
                                cur.data_ptr(), rows_b, acc.data_ptr(), stream)
        stats = self.ctx.all_reduce_mean(acc / float(n))
        vals = stats.cpu().tolist()
        return vals[0], vals[1]
