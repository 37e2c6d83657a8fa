"""Step engines: how one training epoch / one optimizer step is executed.

* ``FusedMLPEngine`` (GPU, MLP family with widths that fit one CU): the reference's whole
  per-step hot loop (collate -> forward -> CE -> backward -> DDP all-reduce -> Adam,
  jobs/train_lightning_ddp.py:66-71,88,136) runs in the fused HIP kernels of
  csrc/mlp_fused.hip with the dataset resident in HBM and batches gathered on device.
    - world size 1: ONE persistent launch runs every step of an epoch (weights in LDS, Adam
      moments in VGPRs, nothing but the batch rows touches HBM per step).
    - world size > 1, 2-layer nets of the single-wave kernel (the reference model): the same
      persistent launch, with the DDP gradient average done INSIDE the kernel over xGMI peer
      mappings (parallel/xgmi.py) - one launch per rank per epoch, no per-step collective.
    - other world size > 1 cases: per step {fused fwd+bwd (grads + loss -> one flat buffer), RCCL
      ncclAvg all-reduce of that buffer (gradients AND the sync_dist train_loss in ONE
      collective: X5+X6 of SURVEY §2.6), fused flat Adam}; the epoch's step loop is captured
      once into a HIP graph and replayed every epoch (the Adam step count and dropout stream
      are read from a device counter, so replays are exact).
* ``AutogradEngine`` (any TrainModule; CPU/gloo plumbing path and the large-model GPU path):
  ``training_step`` + autograd, parameters/gradients as views of flat buffers, the bucketed
  reducer hooked on ``post_accumulate_grad`` (overlap with backward), flat Adam.
"""
from __future__ import annotations

import contextlib
import math
import os
import time
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from ..data.sampler import distributed_indices
from ..ops._native import reload_knobs
from ..ops.fused_mlp import FusedMLPKernel, mlp_num_params
from ..ops.nn import BatchGather, bound_params, fold_batch_gather, join_side_work, unit_loss_seed
from ..ops.optim import FlatAdam, adam_flat_
from ..parallel.dist import DistContext, init_native_comm
from ..parallel.reducer import NativeBucketReducer, TorchBucketReducer, plan_buckets
from ..utils.debug import assert_reducer_complete, check_device
from ..utils.debug import enabled as debug_enabled
from ..utils.debug import reducer_timing_enabled


def adam_hparams_from(optimizer) -> Optional[Dict]:
    """Extract Adam hyper-parameters from a configure_optimizers() result (None if not Adam)."""
    opt = optimizer
    if isinstance(opt, (list, tuple)):
        if len(opt) != 1:
            return None
        opt = opt[0]
    if isinstance(opt, dict):
        opt = opt.get("optimizer")
    if type(opt) is not torch.optim.Adam:
        return None
    g = opt.param_groups[0]
    if g.get("amsgrad") or g.get("maximize"):
        return None
    return dict(lr=float(g["lr"]), betas=tuple(float(b) for b in g["betas"]), eps=float(g["eps"]),
                weight_decay=float(g["weight_decay"]))


class _EngineBase:
    name = "base"

    def __init__(self, model, ctx: DistContext, batch_size: int, seed: int):
        if ctx.device.type == "cuda":
            reload_knobs()  # bind time: the native launchers' DCT_* knobs
        self.model = model
        self.ctx = ctx
        self.B = int(batch_size)
        self.seed = int(seed)
        self.global_step = 0

    def epoch_local_indices(self, n_train: int, epoch: int, shuffle: bool) -> torch.Tensor:
        return distributed_indices(n_train, self.ctx.world_size, self.ctx.rank, shuffle=shuffle, seed=self.seed,
                                   epoch=epoch)


# ================================================================================ fused
class FusedMLPEngine(_EngineBase):
    name = "fused"
    epoch_engine = True  # runs whole epochs on device; the Trainer reads back per-step losses
    # DDP step path (the RCCL / peer-exchange fallback of the in-kernel exchange): steps per captured
    # graph chunk, and the update-then-grad single kernel where the wave kernel supports it (tests
    # override these on the class to exercise the other paths)
    GRAPH_CHUNK = 256
    FUSED_UPDATE = True

    @staticmethod
    def applicable(model, device: torch.device, batch_size: int) -> bool:
        if device.type != "cuda" or not hasattr(model, "fused_spec"):
            return False
        spec = model.fused_spec()
        return FusedMLPKernel.supported(spec["dims"], batch_size)

    def __init__(self, model, ctx: DistContext, batch_size: int, seed: int, adam: Dict,
                 steps_per_launch: int = 0, use_graph: Optional[bool] = None):
        super().__init__(model, ctx, batch_size, seed)
        spec = model.fused_spec()
        self.dims = spec["dims"]
        self.dropout = float(spec["dropout"])
        self.loss = spec["loss"]
        self.adam = adam
        self.kernel = FusedMLPKernel(self.dims, bmax=4 if self.B <= 4 else 16)
        self.P = mlp_num_params(self.dims)
        dev = ctx.device
        self.device = dev
        self.p = self._flat_from_model().to(dev)
        self.m = torch.zeros_like(self.p)
        self.v = torch.zeros_like(self.p)
        self.step_counter = torch.zeros(1, dtype=torch.int32, device=dev)
        self.steps_per_launch = int(steps_per_launch)
        self.use_graph = (os.environ.get("DCT_GRAPH", "1") != "0") if use_graph is None else use_graph
        self.rank_seed = (self.seed * 1000003 + ctx.rank * 7919 + 1) & 0xFFFFFFFF
        self.comm = None
        self.gbuf = None
        # DDP step path; DCT_FORCE_DDP=1 drives it at world size 1 (single-GPU test of the
        # RCCL communicator + graph capture + device cursors)
        self.ddp = ctx.is_distributed or os.environ.get("DCT_FORCE_DDP", "0") == "1"
        self.fused_update = self.kernel.fused_update_supported(self.B) and self.FUSED_UPDATE
        self.pending = torch.zeros(1, dtype=torch.int32, device=dev)
        self.stage = torch.zeros(64 * 4, dtype=torch.int32, device=dev)  # next-batch hand-off
        # (mlp_block5's grad mode takes no batch hand-off between DDP step launches: it measured 0.5 us
        # slower, profiles/block5_stage_ab_r3.log; the wave kernels' fused update uses self.stage)
        self._graphs = {}
        self.graph_chunk = int(self.GRAPH_CHUNK)
        self.cursor = torch.zeros(1, dtype=torch.int32, device=dev)
        self.graph_used = False
        if ctx.is_distributed:
            self.comm = init_native_comm(ctx) if ctx.backend == "nccl" else None
        elif self.ddp:
            from ..ops._native import native

            nat = native()
            self.comm = nat.Comm(nat.comm_unique_id(), 1, 0, dev.index or 0)
        if self.ddp:
            self.gbuf = torch.zeros(self.P + 1, dtype=torch.float32, device=dev)
            self._broadcast_params()
        self.xg = None  # in-kernel xGMI all-reduce (parallel/xgmi.py)
        self.gx = None  # DDP step path: fused peer all-reduce + Adam kernel over xGMI (csrc/xg_adam.hip)
        self._xg_probed = False
        if ctx.is_distributed:
            from ..parallel.xgmi import inkernel_enabled
            from ..parallel.xgmi import mode as xg_mode
            from ..parallel.xgmi import setup_grad_exchange, setup_peer_exchange, timeout_s

            # the persistent launch averages gradients itself when its kernel can (5-64-2 single-wave
            # kernel; the 3x128 block kernel at 2 .. 8 ranks) - the same answer on every rank, so
            # the collective setup below is entered by all or none
            if (self.kernel.xg_supported(self.B, ctx.world_size) and ctx.device.type == "cuda"
                    and inkernel_enabled()):
                self.xg = setup_peer_exchange(self.kernel, ctx, self.B)
            self.xg_timeout_s = timeout_s()
            # exchange time of the launches (s_memrealtime ticks, 100 MHz) -> allreduce_ms per epoch
            self.xg_ticks = torch.zeros(1, dtype=torch.int64, device=dev) if self.xg is not None else None
            if self.xg is None and not self.fused_update:
                self.gx = setup_grad_exchange(ctx, self.P + 1)
            if xg_mode() == "xgmi" and self.xg is None and self.gx is None:
                raise RuntimeError("DCT_ALLREDUCE=xgmi but neither the in-kernel exchange nor the peer "
                                   "all-reduce + Adam kernel is available for this model / world size")
            if self.xg is None and self.gx is None and self.comm is None:
                raise RuntimeError("distributed fused engine needs RCCL (backend nccl) or the in-kernel "
                                   "xGMI exchange; neither is available")
        elif self.ddp and not self.fused_update and os.environ.get("DCT_XG_GRAD") == "1":
            # single-GPU rehearsal (DCT_FORCE_DDP=1 DCT_XG_GRAD=1): the exchange kernel of one rank
            # (no pushes, no polls) in place of the one-rank RCCL all-reduce + flat Adam
            from ..ops._native import native
            from ..parallel.xgmi import timeout_s

            nat = native()
            self.gx = nat.PeerExchange(1, 0, nat.xg_adam_buffer_bytes(self.P + 1, 1))
            self.gx.set_peers([self.gx.recv])
            self.xg_timeout_s = timeout_s()
        self.last_allreduce_ms = None
        self._bound = None
        self._fast_run = None  # (loss_out, n_items, step limit, bound launch, loss ptr) of the last run

    # ------------------------------------------------------------------ params
    def _linear_params(self):
        out = []
        for lin in self.model.linear_layers():
            out += [lin.weight, lin.bias]
        return out

    def _flat_from_model(self) -> torch.Tensor:
        return torch.cat([t.detach().float().reshape(-1).cpu() for t in self._linear_params()])

    def _broadcast_params(self):
        if self.comm is None:  # gloo control plane (ranks sharing a device)
            self.ctx.broadcast_(self.p, src=0)
            return
        from ..ops._native import native

        nat = native()
        s = torch.cuda.current_stream().cuda_stream
        self.comm.broadcast(self.p.data_ptr(), self.P, nat.DT_F32, 0, s)  # X3 (DDP _sync_module_states)

    def sync_to_model(self):
        """Copy the flat device parameters back into the nn.Module (for checkpoints/serving)."""
        off = 0
        flat = self.p.detach().cpu()
        with torch.no_grad():
            for t in self._linear_params():
                n = t.numel()
                t.copy_(flat[off: off + n].view_as(t))
                off += n

    def load_from_model(self):
        self.p.copy_(self._flat_from_model().to(self.device))

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
        self._reset_exchanges()  # exchange tags derive from the step counter: drop stale granules

    def _reset_exchanges(self):
        """Collective: zero the exchanges' receive buffers (and status) once every rank is idle."""
        xs = [x for x in (self.xg, self.gx) if x is not None]
        if not xs:
            return
        torch.cuda.synchronize(self.device)
        self.ctx.barrier()
        for x in xs:
            x.reset(torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize(self.device)
        self.ctx.barrier()

    # ------------------------------------------------------------------ data
    def attach_data(self, X: torch.Tensor, Y: torch.Tensor, train_rows: torch.Tensor, val_rows: torch.Tensor):
        dev = self.device
        if X.shape[1] != self.dims[0]:
            raise ValueError(f"dataset has {X.shape[1]} features, model expects {self.dims[0]}")
        self.X = X.to(torch.float32).contiguous().pin_memory().to(dev, non_blocking=True)
        self.Y = Y.to(torch.int32).contiguous().pin_memory().to(dev, non_blocking=True)
        n = X.shape[0]
        for rows in (train_rows, val_rows):
            if rows.numel() and (int(rows.min()) < 0 or int(rows.max()) >= n):
                raise ValueError("split indices out of range")
        self.train_rows = train_rows.to(torch.int64)
        self.val_rows = val_rows.to(torch.int64)
        n_local = math.ceil(len(self.train_rows) / self.ctx.world_size)
        self.idx = torch.zeros(max(1, n_local), dtype=torch.int32, device=dev)
        vl = math.ceil(max(1, len(self.val_rows)) / self.ctx.world_size)
        self.val_idx = torch.zeros(max(1, vl), dtype=torch.int32, device=dev)
        self.eval_acc = torch.zeros(2, dtype=torch.float32, device=dev)
        self._bound = None  # launches bound to the previous tables

    def steps_per_epoch(self) -> int:
        n_local = math.ceil(len(self.train_rows) / self.ctx.world_size)
        return math.ceil(n_local / self.B)

    def upload_epoch_indices(self, epoch: int, shuffle: bool = True) -> int:
        self.stage.zero_()  # staged batches refer to the previous index list
        local = self.epoch_local_indices(len(self.train_rows), epoch, shuffle)
        rows = self.train_rows[local].to(torch.int32)
        self.idx[: rows.numel()].copy_(rows.pin_memory(), non_blocking=True)
        return rows.numel()

    # ------------------------------------------------------------------ train
    def _bound_launch(self, n_items: int, loss_out: torch.Tensor):
        """The persistent train launch bound to (index list, loss buffer, exchange): validated once,
        then every run_steps call is one short native call (ops/fused_mlp.py BoundTrain)."""
        key = (n_items, loss_out.data_ptr(), loss_out.numel())
        bl = getattr(self, "_bound", None)
        if bl is None or self._bound_key != key:
            a = self.adam
            bl = self.kernel.prepare_train(self.p, self.m, self.v, self.X, self.Y, self.idx, n_items=n_items,
                                           batch=self.B, lr=a["lr"], betas=a["betas"], eps=a["eps"],
                                           weight_decay=a["weight_decay"], dropout=self.dropout, seed=self.rank_seed,
                                           loss_out=loss_out, loss=self.loss, step_counter=self.step_counter,
                                           xg=self.xg, xg_timeout_s=getattr(self, "xg_timeout_s", 20.0),
                                           xg_ticks=getattr(self, "xg_ticks", None) if self.xg is not None else None)
            self._bound, self._bound_key = bl, key
        return bl

    @property
    def step_mode(self) -> str:
        if self.xg is not None:
            return "fused-persistent+xgmi-inkernel-allreduce"
        if not self.ddp:
            return "fused-persistent"
        if self.gx is not None:
            return "fused-step+xgmi-allreduce-adam" + ("+graph" if self.use_graph else "")
        return "fused-step+rccl" + ("+graph" if self.use_graph else "")

    def run_steps(self, n_items: int, steps: int, loss_out: torch.Tensor, first_step: int = 0):
        """Enqueue ``steps`` optimizer steps over batches [first_step, first_step+steps) of self.idx.

        loss_out is indexed by the absolute batch index (loss_out[first_step + s]) and must hold
        first_step + steps entries (with DDP: the cross-rank mean loss).  No host synchronisation."""
        fr = self._fast_run
        if (fr is not None and loss_out is fr[0] and n_items == fr[1] and 0 < steps and 0 <= first_step
                and first_step + steps <= fr[2] and fr[3] is self._bound and loss_out.data_ptr() == fr[4]):
            # repeat call on the same bound launch (the driver's timed window): checks already done
            fr[3].run(first_step, steps)
            return
        if steps <= 0:
            return
        if (first_step + steps - 1) * self.B >= n_items or loss_out.numel() < first_step + steps:
            raise ValueError("step range exceeds the epoch's batches / loss buffer")
        if not self.ddp or self.xg is not None:
            bl = self._bound_launch(n_items, loss_out)
            if not self.steps_per_launch:
                self._fast_run = (loss_out, n_items, min(loss_out.numel(), -(-n_items // self.B)), bl,
                                  loss_out.data_ptr())
            chunk = self.steps_per_launch or steps
            s = 0
            while s < steps:
                k = min(chunk, steps - s)
                bl.run(first_step + s, k)
                s += k
            return
        self.cursor.fill_(first_step)
        C = min(self.graph_chunk, steps)
        full, rem = divmod(steps, C)
        done = 0
        if self.use_graph:
            g = self._get_graph(n_items, C, loss_out)
            if g is not None:
                for _ in range(full):
                    g.replay()
                done = full * C
                self.graph_used = True
        for _ in range(steps - done):
            self._ddp_step(n_items, loss_out)
        if self.fused_update:  # the last step's update is still pending: apply it
            a = self.adam
            adam_flat_(self.p, self.gbuf[: self.P], self.m, self.v, 1, a["lr"], a["betas"], a["eps"],
                       a["weight_decay"], step_counter=self.step_counter)
            self.pending.zero_()
        # the last step's reduced loss is flushed by the next kernel; flush it here instead
        last = first_step + steps - 1
        loss_out[last: last + 1].copy_(self.gbuf[self.P: self.P + 1])

    def _ddp_step(self, n_items: int, loss_out: torch.Tensor):
        """One DDP step at the device cursor: fused fwd/bwd (grads + local loss -> gbuf) ->
        RCCL ncclAvg all-reduce of gbuf (X5 + X6 in one collective) -> fused flat Adam; with the
        peer exchange (self.gx) the last two are one kernel over the xGMI mappings."""
        from ..ops._native import native

        a = self.adam
        nat = native()
        stream = torch.cuda.current_stream().cuda_stream
        if self.fused_update:
            # one kernel: apply the previous step's (reduced) Adam update, then fwd/bwd
            self.kernel.train(self.p, self.m, self.v, self.X, self.Y, self.idx, n_items=n_items, batch=self.B,
                              steps=1, t0=0, lr=a["lr"], betas=a["betas"], eps=a["eps"],
                              weight_decay=a["weight_decay"], dropout=self.dropout, seed=self.rank_seed,
                              loss=self.loss, grad_out=self.gbuf, step_counter=self.step_counter,
                              cursor=self.cursor, loss_out=loss_out, pending=self.pending, stage=self.stage)
            self.comm.allreduce(self.gbuf.data_ptr(), self.P + 1, nat.DT_F32, nat.OP_AVG, stream)
            return
        self.kernel.train(self.p, None, None, self.X, self.Y, self.idx, n_items=n_items, batch=self.B, steps=1,
                          t0=0, lr=a["lr"], dropout=self.dropout, seed=self.rank_seed, loss=self.loss,
                          grad_out=self.gbuf, step_counter=self.step_counter, cursor=self.cursor,
                          loss_out=loss_out)
        if self.gx is not None:
            from ..parallel.xgmi import allreduce_adam_

            allreduce_adam_(self.gx, self.gbuf, self.p, self.m, self.v, self.P, self.step_counter, a["lr"],
                            a["betas"], a["eps"], a["weight_decay"], timeout=self.xg_timeout_s)
            return
        self.comm.allreduce(self.gbuf.data_ptr(), self.P + 1, nat.DT_F32, nat.OP_AVG, stream)
        adam_flat_(self.p, self.gbuf[: self.P], self.m, self.v, 1, a["lr"], a["betas"], a["eps"],
                   a["weight_decay"], step_counter=self.step_counter)

    def _get_graph(self, n_items: int, C: int, loss_out: torch.Tensor):
        key = (n_items, C, loss_out.data_ptr())
        if key in self._graphs:
            return self._graphs[key]
        from ..ops._native import native

        nat = native()
        # RCCL lazy init and kernel attribute setup must happen outside the capture
        if self.gx is None:
            scratch = torch.zeros(64, dtype=torch.float32, device=self.device)
            self.comm.allreduce(scratch.data_ptr(), 64, nat.DT_F32, nat.OP_SUM,
                                torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize(self.device)
        state = (self.p, self.m, self.v, self.step_counter, self.cursor, self.gbuf, loss_out, self.pending,
                 self.stage)
        saved = [t.clone() for t in state]
        # one eager step first (kernel attributes, RCCL channels), then roll the state back
        self._ddp_step(n_items, loss_out)
        torch.cuda.synchronize(self.device)
        for t, sv in zip(state, saved):
            t.copy_(sv)
        self._reset_exchanges()  # the rolled-back step counter re-issues the eager step's tags
        g = torch.cuda.CUDAGraph()
        try:
            s = torch.cuda.Stream(self.device)
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                    for _ in range(C):
                        self._ddp_step(n_items, loss_out)
            torch.cuda.current_stream().wait_stream(s)
        except Exception as e:  # noqa: BLE001 - eager fallback keeps training correct
            print(f"[dct] HIP graph capture failed ({e!r}); DDP steps run eagerly", flush=True)
            g = None
        torch.cuda.synchronize(self.device)
        for t, sv in zip(state, saved):
            t.copy_(sv)
        self._graphs[key] = g
        return g

    def train_epoch(self, epoch: int, shuffle: bool = True) -> torch.Tensor:
        n_items = self.upload_epoch_indices(epoch, shuffle)
        steps = math.ceil(n_items / self.B)
        loss_out = getattr(self, "_loss_buf", None)
        if loss_out is None or loss_out.numel() < steps:
            self._loss_buf = loss_out = torch.zeros(max(1, steps), dtype=torch.float32, device=self.device)
        first = 0
        if self.xg is not None or self.gx is not None:
            torch.cuda.synchronize(self.device)
            self.ctx.barrier()  # start the epoch's kernels together (the exchange spins are bounded)
            if not self._xg_probed:
                first = self._probe_exchange(n_items, steps, loss_out[:steps])
        if first < steps:
            self.run_steps(n_items, steps - first, loss_out[:steps], first_step=first)
        check_device("fused epoch")
        if self.gx is not None:
            self.xg_verify(fallback=False)
        elif self.xg is not None:
            self.xg_verify(fallback=False)
            # wave 0's exchange time over the epoch (the in-kernel all-reduce: X5 + X6 of SURVEY 2.6)
            self.last_allreduce_ms = float(self.xg_ticks.item()) / 1e5
            self.xg_ticks.zero_()
        self.global_step += steps
        return loss_out[:steps]

    def _probe_exchange(self, n_items: int, steps: int, loss_out: torch.Tensor) -> int:
        """First steps of a run through the peer exchange with a SHORT spin limit, then a
        collective check: if some rank cannot see its peers' writes (xGMI mapping, IPC mode), the
        job pays seconds, not the full timeout per launch, and continues on RCCL with every rank
        re-synced from rank 0.  Returns the steps of this epoch already applied."""
        from ..parallel.xgmi import probe_timeout_s

        self._xg_probed = True
        k = min(steps, 4)
        # a timed-out exchange may leave a step half applied (xg_adam: per block): every rank keeps
        # its pre-probe state to return to - replicas were identical before the probe
        snap = [t.clone() for t in (self.p, self.m, self.v, self.step_counter)]
        a = self.adam
        if self.xg is not None:
            self.kernel.train(self.p, self.m, self.v, self.X, self.Y, self.idx, n_items=n_items, batch=self.B,
                              steps=k, t0=0, lr=a["lr"], betas=a["betas"], eps=a["eps"],
                              weight_decay=a["weight_decay"], dropout=self.dropout, seed=self.rank_seed,
                              loss_out=loss_out, loss=self.loss, step_counter=self.step_counter, xg=self.xg,
                              xg_timeout_s=probe_timeout_s())
        else:
            full, self.xg_timeout_s = self.xg_timeout_s, probe_timeout_s()
            try:
                self.run_steps(n_items, k, loss_out, first_step=0)
            finally:
                self.xg_timeout_s = full
        if self.xg_verify(fallback=True, snapshot=snap):
            return k
        return 0  # every rank is back at its pre-probe state: the epoch runs whole on RCCL

    def xg_verify(self, fallback: bool, snapshot=None) -> bool:
        """Collective check of the in-kernel exchange.  On a timeout either raise (training: the
        steps of that launch are incomplete) or, with ``fallback``, re-sync every rank from rank 0
        and continue on the RCCL step path (benchmarks)."""
        x = self.xg if self.xg is not None else self.gx
        if x is None:
            return True
        from ..parallel.xgmi import check

        st = check(x, self.ctx)
        if st == 0:
            return True
        msg = f"in-kernel xGMI all-reduce timed out (step tag {st & 0x7FFFFFFF})"
        if not fallback:
            raise RuntimeError(msg)
        if self.ctx.rank == 0:
            print(f"[dct] {msg}; re-syncing from rank 0 and falling back to RCCL", flush=True)
        self.xg_disable(snapshot)
        return False

    def device_barrier(self) -> bool:
        """Enqueue the in-kernel exchange's device-side barrier on the current stream (collective).
        False when the exchange is not active (the caller then uses the process-group barrier)."""
        x = self.xg if self.xg is not None else self.gx
        if x is None:
            return False
        from ..parallel.xgmi import device_barrier

        device_barrier(x, torch.cuda.current_stream(self.device).cuda_stream, self.xg_timeout_s)
        return True

    def xg_disable(self, snapshot=None):
        """Leave the in-kernel exchange: replicas re-synced from rank 0, RCCL step path from now on.
        ``snapshot`` (p, m, v, step_counter taken while the replicas were in sync) is restored on
        every rank first, so no half-applied step of a timed-out exchange survives."""
        self.xg = None
        self.gx = None
        self._bound = None
        self._graphs = {}  # captured with the exchange's kernels
        if self.comm is None:
            raise RuntimeError("in-kernel exchange disabled and no RCCL communicator is available to fall back to")
        torch.cuda.synchronize(self.device)
        if snapshot is not None:
            for t, sv in zip((self.p, self.m, self.v, self.step_counter), snapshot):
                t.copy_(sv)
        for t in (self.p, self.m, self.v, self.step_counter):
            self.ctx.broadcast_(t, src=0)
        torch.cuda.synchronize(self.device)

    # ------------------------------------------------------------------ eval
    def validate(self, rows: Optional[torch.Tensor] = None, limit: Optional[int] = None) -> Tuple[float, float]:
        rows = self.val_rows if rows is None else rows
        local = distributed_indices(len(rows), self.ctx.world_size, self.ctx.rank, shuffle=False)
        if limit is not None:
            local = local[:limit]
        r = rows[local].to(torch.int32)
        if r.numel() == 0:
            return float("nan"), float("nan")
        if r.numel() > self.val_idx.numel():
            self.val_idx = torch.zeros(r.numel(), dtype=torch.int32, device=self.device)
        self.val_idx[: r.numel()].copy_(r)
        self.eval_acc.zero_()
        self.kernel.evaluate(self.p, self.X, self.Y, self.val_idx, r.numel(), self.eval_acc, loss=self.loss)
        stats = self.eval_acc / float(r.numel())
        stats = self.ctx.all_reduce_mean(stats)
        vals = stats.cpu().tolist()
        return vals[0], vals[1]


# ============================================================================= autograd
class AutogradEngine(_EngineBase):
    name = "autograd"

    def __init__(self, model, ctx: DistContext, batch_size: int, seed: int, bucket_cap_bytes: int = 8 << 20,
                 first_bucket_bytes: int = 1 << 20):
        super().__init__(model, ctx, batch_size, seed)
        dev = ctx.device
        self.device = dev
        model.to(dev)
        params = [p for p in model.parameters() if p.requires_grad]
        self.params = params
        numels = [p.numel() for p in params]
        total = sum(numels)
        self.flat_p = torch.zeros(total, dtype=torch.float32, device=dev)
        self.flat_g = torch.zeros(total, dtype=torch.float32, device=dev)
        off = 0
        with torch.no_grad():
            for p in params:
                n = p.numel()
                self.flat_p[off: off + n].copy_(p.detach().reshape(-1).float())
                p.data = self.flat_p[off: off + n].view_as(p)
                p.grad = self.flat_g[off: off + n].view_as(p)
                off += n
        if ctx.is_distributed:
            ctx.broadcast_(self.flat_p, 0) if ctx.backend != "nccl" else self._bcast_nccl()
        # models whose gradients become ready in block groups (the TabTransformer's grouped deferred
        # dW, model.ddp_block_groups) can get buckets aligned with the groups, each launched as its
        # group's dW launch is issued (DCT_TT_DDP_GROUPS=1).  Off by default: the step is graph-captured,
        # where the collectives run inline (runtime.cpp BucketReducer), so the split buys no overlap and
        # its second dW launch costs 7-14 us per step (forced-DDP TabTransformer 0.334-0.336 -> 0.322-0.327
        # ms, with the 60 us stand-in 0.397 -> 0.383-0.390; profiles/tt_ddp_groups_ab_r5.log)
        self._dw_groups, split_before = self._block_groups(model, params)
        self.plan = plan_buckets(numels, 4, bucket_cap_bytes, first_bucket_bytes, split_before=split_before)
        self.reducer = None
        # DCT_FORCE_DDP=1 at world size 1 on a GPU: the full DDP path (RCCL communicator of one
        # rank, bucket reducer on its comm stream, hooks, graph capture) - how its correctness,
        # overlap and cost are tested and measured on one GPU
        forced = (not ctx.is_distributed and dev.type == "cuda" and os.environ.get("DCT_FORCE_DDP", "0") == "1")
        if ctx.is_distributed or forced:
            if dev.type == "cuda" and (forced or ctx.backend == "nccl"):
                if forced:
                    from ..ops._native import native

                    nat = native()
                    self._own_comm = comm = nat.Comm(nat.comm_unique_id(), 1, 0, dev.index or 0)
                else:
                    comm = init_native_comm(ctx)
                # device-side all-reduce timing (allreduce_ms): opt-in (DCT_REDUCER_TIMING=1, or with
                # DCT_DEBUG=1) - its stamp kernels and the extra cross-stream edge cost every step,
                # so default training runs the same step the benchmark times; DCT_DEBUG=1 also adds
                # the stream-ordering check
                timing = reducer_timing_enabled()
                self.reducer = NativeBucketReducer(comm, self.flat_g, self.plan, timing=timing,
                                                   check=debug_enabled())
            else:
                # gloo: the CPU plumbing config, or GPU ranks sharing one device (init_distributed
                # falls back to gloo there because RCCL refuses it) - buckets staged through host
                # memory, which no HIP graph can capture
                staged = dev.type == "cuda"
                self.reducer = TorchBucketReducer(self.flat_g, self.plan, ctx.world_size, host_staging=staged)
                if staged:
                    self._graph_failed = True
            self._hooks = []
            for i, p in enumerate(params):
                self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(i)))
        self.graph_used = False
        # per-step GPU phase timing (device timestamps, works inside captured graphs): the Trainer
        # logs time/{fwd,bwd,allreduce,opt}_s per epoch
        self.phase_timer = None
        if dev.type == "cuda" and os.environ.get("DCT_PHASE_TIMING", "0") == "1":
            from ..utils.tracing import DevicePhaseTimer

            self.phase_timer = DevicePhaseTimer(["fwd", "bwd", "allreduce", "opt"], dev)
        opt = model.configure_optimizers()
        hp = adam_hparams_from(opt)
        if hp is not None:
            self.optimizer = FlatAdam(self.flat_p, self.flat_g, [p.shape for p in params], **hp)
            self.torch_optimizer = None
        else:
            self.optimizer = None
            self.torch_optimizer = opt[0] if isinstance(opt, (list, tuple)) else opt
        # native-op fast paths (ops/nn.py bound_params): weight-gradient accumulation straight into
        # the flat bucket buffer, and bf16 shadow weights maintained by the fused Adam
        self._shadows = None
        self.flat_p16 = None
        if dev.type == "cuda" and self.optimizer is not None:
            self.flat_p16 = self.flat_p.to(torch.bfloat16)
            self.optimizer.p_bf16 = self.flat_p16
            self._shadows = {}
            off = 0
            for p in params:
                n = p.numel()
                self._shadows[id(p)] = self.flat_p16[off: off + n].view(p.shape)
                off += n

    def _bcast_nccl(self):
        self.ctx.broadcast_(self.flat_p, 0)

    def _block_groups(self, model, params):
        """(deferred-dW group sizes, bucket split indices) of a model with ddp_block_groups(), else
        ((), ()).  Only for data-parallel runs (a reducer to overlap with)."""
        groups = model.ddp_block_groups() if hasattr(model, "ddp_block_groups") else None
        dp = self.ctx.is_distributed or os.environ.get("DCT_FORCE_DDP", "0") == "1"
        if not groups or len(groups) < 2 or not dp or os.environ.get("DCT_TT_DDP_GROUPS", "0") != "1":
            return (), ()
        index = {id(p): i for i, p in enumerate(params)}
        splits = []
        for g in groups[:-1]:
            lo = min(g)  # the group's lowest block: its first parameter opens the bucket
            first = min(index[id(p)] for p in model.blocks[lo].parameters())
            splits.append(first - 1)
        return tuple(len(g) for g in groups), tuple(splits)

    def _make_hook(self, i):
        def hook(_p):
            self.reducer.mark_ready(i)
        return hook

    def attach_data(self, X: torch.Tensor, Y: torch.Tensor, train_rows: torch.Tensor, val_rows: torch.Tensor):
        self.X = X.to(self.device, torch.float32)
        self.Y = Y.to(self.device, torch.int64)
        self.train_rows = train_rows.to(torch.int64)
        self.val_rows = val_rows.to(torch.int64)

    def steps_per_epoch(self) -> int:
        return math.ceil(math.ceil(len(self.train_rows) / self.ctx.world_size) / self.B)

    def _zero_grads(self):
        if self.flat_g.is_cuda:
            # a native kernel rather than zero_(): torch lowers it to a memset node, which replayed
            # graphs did not reliably order after the previous replay's Adam (csrc/step_kernels.hip)
            from ..ops._native import native

            native().zero_f32(self.flat_g.data_ptr(), self.flat_g.numel(), torch.cuda.current_stream().cuda_stream)
        else:
            self.flat_g.zero_()

    def _backward(self, loss: torch.Tensor):
        """loss.backward() with a persistent ones seed: autograd's implicit ones_like(loss) is a
        fill kernel per step (~4.5 us in the captured TabTransformer step on MI355X)."""
        one = getattr(self, "_one_seed", None)
        if one is None or one.device != loss.device or one.dtype != loss.dtype or one.shape != loss.shape:
            one = self._one_seed = torch.ones_like(loss)
        loss.backward(one)
        join_side_work()  # weight-gradient GEMMs issued on the side stream (ops/nn.py side_dw)

    def _pm(self, i: int):
        """Phase mark i of the step (DCT_PHASE_TIMING=1): 0 start, 1 forward done, 2 backward done,
        3 all-reduce joined, 4 optimizer done."""
        if self.phase_timer is not None:
            self.phase_timer.mark(i)
            if i == 4:
                self.phase_timer.close()

    def _step_body(self, x, y, batch_idx: int):
        self._zero_grads()
        if self.reducer is not None:
            self.reducer.prepare()
        self._pm(0)
        self.model.train()
        # the step's backward root is training_step's loss with a seed of exactly 1 (_backward): a fused
        # classifier head may compute its backward inside the forward launch (ops/nn.py unit_loss_seed)
        with self._bound(), unit_loss_seed():
            loss = self.model.training_step((x, y), batch_idx)
            if isinstance(loss, dict):
                loss = loss["loss"]
            self._pm(1)
            self._backward(loss)
        self._pm(2)
        if self.reducer is not None:
            self.reducer.finalize()
            assert_reducer_complete(self.reducer)
        self._pm(3)
        if self.optimizer is not None:
            self.optimizer.step()
        else:
            self.torch_optimizer.step()
        self._pm(4)
        return loss

    def train_step(self, rows: torch.Tensor, batch_idx: int):
        """One optimizer step.  ``last_step_mode`` tells the Trainer how training_step ran:
        ``eager``; ``captured`` (traced into the step graph, then replayed - the tensors it logged
        are the graph's static outputs); ``replayed`` (training_step and self.log did NOT run)."""
        rows_d = rows.to(self.device)
        self.last_step_mode = "eager"
        if self._graph_ok(rows_d.numel()):
            self.last_step_mode = "replayed" if getattr(self, "_graph", None) is not None else "captured"
            loss = self._graph_step(rows_d, batch_idx)
            if getattr(self, "_graph_failed", False):
                self.last_step_mode = "eager"
        elif getattr(self, "_warming", False):
            # graph warmup steps run on the capture stream (torch's capture recipe): autograd's
            # AccumulateGrad nodes then already live on that stream when the step is captured
            s = self._capture_stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                loss = self._step_body(self.X[rows_d], self.Y[rows_d], batch_idx).detach()
            torch.cuda.current_stream().wait_stream(s)
        else:
            loss = self._step_body(self.X[rows_d], self.Y[rows_d], batch_idx)
        self.global_step += 1
        return loss.detach()

    def _capture_stream(self):
        s = getattr(self, "_cap_stream", None)
        if s is None:
            self._cap_stream = s = torch.cuda.Stream(self.device)
        return s

    # ------------------------------------------------------------------ HIP graph of the step
    # GPU + flat Adam: after GRAPH_WARMUP eager steps the whole step (zero grads, forward,
    # backward with the bucket all-reduces issued from the grad hooks on the reducer's comm
    # stream, finalize, Adam with the device step counter) is captured once and replayed; the
    # batch is gathered into static input buffers by index_select on the device.
    GRAPH_WARMUP = 3

    def _graph_ok(self, n_rows: int) -> bool:
        self._warming = False
        if self.device.type != "cuda" or self.optimizer is None or n_rows != self.B:
            return False
        if os.environ.get("DCT_GRAPH", "1") == "0" or getattr(self, "_graph_failed", False):
            return False
        self._eager_full = getattr(self, "_eager_full", 0)
        if getattr(self, "_graph", None) is None and self._eager_full < self.GRAPH_WARMUP:
            self._eager_full += 1
            self._warming = True
            return False
        return True

    def _graph_step(self, rows_d: torch.Tensor, batch_idx: int):
        if getattr(self, "_graph", None) is None:
            self._x_static = self.X[rows_d].clone()
            self._y_static = self.Y[rows_d].clone()
            g = torch.cuda.CUDAGraph()
            try:
                s = self._capture_stream()
                s.wait_stream(torch.cuda.current_stream())
                torch.cuda.synchronize(self.device)
                with torch.cuda.stream(s):
                    with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                        self._loss_static = self._step_body(self._x_static, self._y_static, batch_idx).detach()
                torch.cuda.current_stream().wait_stream(s)
            except Exception as e:  # noqa: BLE001 - eager steps stay correct
                print(f"[dct] HIP graph capture of the autograd step failed ({e!r}); running eagerly", flush=True)
                self._graph_failed = True
                torch.cuda.synchronize(self.device)
                return self._step_body(self.X[rows_d], self.Y[rows_d], batch_idx)
            self._graph = g
            self.graph_used = True
            # capture records without executing: Adam's host count moved, the device one did not
            self.optimizer.step_count -= 1
        torch.index_select(self.X, 0, rows_d, out=self._x_static)
        torch.index_select(self.Y, 0, rows_d, out=self._y_static)
        self._graph.replay()
        self.optimizer.step_count += 1
        return self._loss_static

    # ------------------------------------------------------------------ device-side batch loop
    # Steps over a device-resident list of dataset rows with NO host work between replays: the
    # captured graph starts with ONE prologue kernel (batch gather at the device cursor, Adam
    # step counter += 1, gradient zeroing) and ends with the Adam kernel, which also records the
    # step's loss at loss_out[cursor] and advances the cursor (csrc/step_kernels.hip,
    # csrc/optim.hip).  Replaces, per step: host batch slicing, two index_selects, a counter add,
    # a zero kernel and the loss copy.
    def device_loop_ok(self) -> bool:
        return (self.device.type == "cuda" and self.optimizer is not None and self.X.dim() == 2
                and self.X.shape[1] % 4 == 0 and os.environ.get("DCT_GRAPH", "1") != "0"
                and not getattr(self, "_graph_failed", False))

    def run_device_steps(self, rows_dev: torch.Tensor, first_step: int, steps: int, loss_out: torch.Tensor):
        """Steps first_step .. first_step + steps - 1 over rows_dev (int64, device) batches of B;
        losses land in loss_out[step] (fp32, device)."""
        if not self.device_loop_ok():
            for s in range(first_step, first_step + steps):
                loss_out[s] = self.train_step(rows_dev[s * self.B:(s + 1) * self.B], s)
            return
        from ..ops._native import native

        nat = native()
        s = first_step
        end = first_step + steps
        while s < end and getattr(self, "_dgraph", None) is None and self._eager_full_dev() < self.GRAPH_WARMUP:
            loss_out[s] = self.train_step(rows_dev[s * self.B:(s + 1) * self.B], s)  # warm-up (capture stream)
            s += 1
        if s >= end:
            return
        key = (rows_dev.data_ptr(), rows_dev.numel(), loss_out.data_ptr(), loss_out.numel())
        if getattr(self, "_dgraph", None) is None or self._dgraph_key != key:
            try:
                self._capture_device_graph(nat, rows_dev, loss_out, s)
            except Exception as e:  # noqa: BLE001 - eager steps stay correct
                print(f"[dct] HIP graph capture of the device-loop step failed ({e!r}); running eagerly", flush=True)
                self._graph_failed = True
                self._dgraph = None
                torch.cuda.synchronize(self.device)
                for t in range(s, end):
                    loss_out[t] = self.train_step(rows_dev[t * self.B:(t + 1) * self.B], t)
                return
            self._dgraph_key = key
        self._dcursor.fill_(s)
        # one replay per step: a graph holding 8 steps measured the same 0.420 ms/step on the
        # TabTransformer (profiles/tt_device_loop_chunk_ab_r2.log), the replays are already queued
        # back to back
        for _ in range(end - s):
            self._dgraph.replay()
        self.optimizer.step_count += end - s
        self.global_step += end - s

    def _eager_full_dev(self) -> int:
        return getattr(self, "_eager_full", 0)

    def _prologue(self, nat, rows_dev):
        st = torch.cuda.current_stream().cuda_stream
        nat.ag_step_prologue(self.X.data_ptr(), self.X.shape[1] * 4, self.Y.data_ptr(), rows_dev.data_ptr(),
                             self._dcursor.data_ptr(), self.B, rows_dev.numel(), self._x_dev.data_ptr(),
                             self._y_dev.data_ptr(), self.optimizer._device_counter().data_ptr(),
                             self.flat_g.data_ptr(), self.flat_g.numel(), st)

    def _capture_device_graph(self, nat, rows_dev, loss_out, first):
        if not (self.X.is_contiguous() and self.Y.is_contiguous() and self.X.dtype == torch.float32):
            raise RuntimeError("device loop needs contiguous fp32 features / int64 labels")
        self._x_dev = torch.empty(self.B, self.X.shape[1], dtype=torch.float32, device=self.device)
        self._y_dev = torch.empty(self.B, dtype=torch.int64, device=self.device)
        self._dcursor = torch.full((1,), first, dtype=torch.int32, device=self.device)
        # a model whose first fused block can gather its own batch (models/tabtransformer.py
        # folds_batch_gather) takes the step prologue into that launch; if no block took it, the step is
        # captured again with the prologue kernel
        fold = bool(getattr(self.model, "folds_batch_gather", False))
        for folded in ((True, False) if fold else (False,)):
            spec = None
            if folded:
                spec = BatchGather(self.X, rows_dev, self._dcursor, self.B, rows_dev.numel(), self._x_dev, self.Y,
                                   self._y_dev, self.optimizer._device_counter(), self.flat_g)
            g, loss = self._capture_step(nat, rows_dev, loss_out, first, spec)
            self.optimizer.step_count -= 1  # capture recorded without executing
            if spec is None or spec.consumed:
                break
        self.gather_folded = spec is not None and spec.consumed
        self._dgraph = g
        self._dloss = loss
        self.graph_used = True

    def _capture_step(self, nat, rows_dev, loss_out, first, spec):
        g = torch.cuda.CUDAGraph()
        s = self._capture_stream()
        s.wait_stream(torch.cuda.current_stream())
        torch.cuda.synchronize(self.device)
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                if spec is None:
                    self._prologue(nat, rows_dev)
                if self.reducer is not None:
                    self.reducer.prepare()
                self._pm(0)
                self.model.train()
                with self._bound(), unit_loss_seed():  # (as _step_body: the backward seed is exactly 1)
                    with fold_batch_gather(spec) if spec is not None else contextlib.nullcontext():
                        loss = self.model.training_step((self._x_dev, self._y_dev), first)
                    if isinstance(loss, dict):
                        loss = loss["loss"]
                    self._pm(1)
                    self._backward(loss)
                self._pm(2)
                if self.reducer is not None:
                    self.reducer.finalize()
                self._pm(3)
                self.optimizer.step(bump_counter=False, epilogue=(self._dcursor, loss.detach(), loss_out))
                self._pm(4)
        torch.cuda.current_stream().wait_stream(s)
        return g, loss

    def optimizer_state_dict(self) -> Dict:
        if self.optimizer is not None:
            return self.optimizer.state_dict()
        return self.torch_optimizer.state_dict()

    def load_optimizer_state(self, sd: Dict, global_step: int):
        if self.optimizer is not None:
            self.optimizer.load_state_dict(sd)
        else:
            self.torch_optimizer.load_state_dict(sd)
        self.global_step = global_step

    def _bound(self):
        if self._shadows is None:
            return contextlib.nullcontext()
        # every transformer block's dW GEMMs as ONE grouped launch after backward (DCT_TT_DW_DEFER=0
        # keeps one launch per block): TabTransformer step 0.421-0.426 -> 0.407 ms
        # (profiles/tt_dw_defer_ab_r2.log).  With the native bucket reducer too: its hooks then only
        # count and every bucket launches at finalize, after the grouped launch - the model's
        # gradients fit ONE bucket (<= first_bucket_bytes), which could only start after the last
        # dW GEMM anyway, so deferring loses no overlap and keeps the grouped-dW win at W > 1
        defer_ok = self.reducer is None or isinstance(self.reducer, NativeBucketReducer)
        defer = defer_ok and os.environ.get("DCT_TT_DW_DEFER", "1") != "0"
        groups = self._dw_groups if (defer and self.reducer is not None) else ()
        if isinstance(self.reducer, NativeBucketReducer):
            # with block groups every group's dW launch is issued before its bucket's last hook
            # fires, so the hooks launch the buckets; otherwise they launch at finalize
            self.reducer.defer_launch = defer and self._has_deferrable_ops() and not groups
        return bound_params(self.params, self._shadows, defer_dw=defer, defer_groups=groups)

    def _has_deferrable_ops(self) -> bool:
        """True when the model routes weight gradients through the deferred grouped dW path
        (the fused transformer blocks); plain MLP/linear models keep hook-driven bucket launches."""
        return bool(getattr(self.model, "uses_fused_blocks", False))

    def sync_to_model(self):
        pass  # parameters ARE views of the flat buffer

    def load_from_model(self):
        # parameters ARE views of the flat buffer; only the bf16 shadow must follow external writes
        if self.flat_p16 is not None:
            self.flat_p16.copy_(self.flat_p)
