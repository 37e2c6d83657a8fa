"""In-kernel data-parallel gradient all-reduce over xGMI peer mappings.

Why: the reference's DDP step (jobs/train_lightning_ddp.py:136 -> torch Reducer -> one 2,056-byte
bucket all-reduce + the 4-byte ``sync_dist`` loss all-reduce per step) is pure
latency.  On MI355X a per-step RCCL collective costs more than the whole fused step itself (two
kernel boundaries + the collective's own launch and protocol), so for the models the single-wave
kernel trains (2-layer MLPs, widths <= 64) the gradient exchange moves INTO the persistent kernel:

* every rank allocates an uncached receive buffer ``[2 parity][W src][KX][64 lanes]`` of 8-byte
  granules and exports it with ``hipIpcGetMemHandle`` (dmabuf); the W handles are exchanged over
  the c10d process group and each rank maps its peers' buffers (``hipIpcOpenMemHandle``, xGMI
  peer access) - one node, up to 8 GPUs, fully connected by xGMI;
* per step each rank writes {tag = step + 1, fp32 gradient} granules straight into every peer's
  buffer (write-through system-scope stores), then polls its own buffer until all peers' tags
  match and sums the contributions in rank order (bit-identical on all ranks; the loss rides in
  the same granules, so the logged ``train_loss`` is the cross-rank mean like ``sync_dist``);
* no kernel boundary, no host round trip, no RCCL launch per step; RCCL remains the path for
  everything else (initial broadcast, validation metrics, the autograd engine's bucketed reducer).

Selection: ``DCT_ALLREDUCE=auto`` (default: use it when the model/batch qualify, all ranks are on
one node and every rank could map every peer), ``xgmi`` (required: raise if unavailable) or
``rccl`` (never).  Failures are detected collectively: a bounded spin records a timeout in the
status word; :func:`check` max-reduces it over ranks so every rank takes the same decision.
"""
from __future__ import annotations

import os
from typing import Optional

from .dist import DistContext


def mode() -> str:
    m = os.environ.get("DCT_ALLREDUCE", "auto").lower()
    if m not in ("auto", "xgmi", "rccl"):
        raise ValueError(f"DCT_ALLREDUCE must be auto|xgmi|rccl, got {m!r}")
    return m


def timeout_s() -> float:
    return float(os.environ.get("DCT_XG_TIMEOUT_S", "20"))


def inkernel_enabled() -> bool:
    """DCT_XG_INKERNEL=0 keeps the persistent launches out of the exchange (the per-step paths -
    peer all-reduce + Adam kernel or RCCL - take over); default on."""
    return os.environ.get("DCT_XG_INKERNEL", "1") != "0"


def probe_timeout_s() -> float:
    """Spin limit of the first exchange launch of a run (trainer/engines.py _probe_exchange)."""
    return 3.0


def peer_report(ctx: DistContext):
    """Collective: which physical GPU every rank drives and whether they can map each other.

    Returns ``(bus_ids, matrix, ok)``: the PCI bus id of each rank's device (rank order), the
    ``hipDeviceCanAccessPeer`` matrix over the devices visible to this process, and whether every
    pair of distinct rank devices that this process can see is peer-accessible (ranks sharing one
    GPU - a rehearsal - are trivially fine).  A peer outside this process's visible set cannot be
    checked here; the exchange's first-launch verification (``check``) still covers it."""
    from ..ops._native import native

    nat, mine = None, ""
    try:
        nat = native()
        mine = nat.pci_bus_id(ctx.device.index or 0) if ctx.device.type == "cuda" else ""
    except Exception:  # noqa: BLE001 - still take part in the collective below
        nat = None
    bus = ctx.all_gather_object(mine) if ctx.is_distributed else [mine]
    if ctx.device.type != "cuda" or nat is None or not mine:
        return bus, [], False
    mat = nat.peer_matrix()
    local = {nat.pci_bus_id(i).lower(): i for i in range(len(mat))}
    me = local.get(mine.lower(), ctx.device.index or 0)
    ok = True
    for b in bus:
        j = local.get(b.lower())
        if j is not None and j != me and not mat[me][j]:
            ok = False
    return bus, mat, ok


def setup_peer_exchange(kernel, ctx: DistContext, batch: int):
    """Collective: returns a native PeerExchange on every rank, or None on every rank.

    Before any buffer is exported every rank checks ``hipDeviceCanAccessPeer`` towards every
    other rank's device (:func:`peer_report`); one failing pair sends all ranks to RCCL."""
    return _open_exchange(ctx, kernel.xg_supported(batch, ctx.world_size),
                          lambda: kernel.xg_buffer_bytes(ctx.world_size, batch), f"dims {kernel.dims}, batch {batch}",
                          strict=True)


def setup_grad_exchange(ctx: DistContext, n: int):
    """Collective: a PeerExchange sized for the fused peer all-reduce + Adam kernel
    (csrc/xg_adam.hip) over ``n`` floats, or None on every rank.

    The DDP step path of the models the single-wave kernel does not train (the register-resident
    3x128 weather trainer in grad mode) uses it instead of RCCL all-reduce + flat Adam.  Selection
    follows ``DCT_ALLREDUCE`` (``rccl`` never; ``DCT_XG_GRAD=0`` turns this exchange off alone);
    under ``DCT_ALLREDUCE=xgmi`` an unavailable exchange is not an error here - the RCCL step path
    remains."""
    from ..ops._native import native

    on = os.environ.get("DCT_XG_GRAD", "1") != "0"
    return _open_exchange(ctx, on, lambda: native().xg_adam_buffer_bytes(n, ctx.world_size),
                          f"grad exchange of {n} floats", strict=False)


def _open_exchange(ctx: DistContext, supported: bool, nbytes, what: str, strict: bool):
    m = mode()
    W = ctx.world_size
    single_node = ctx.local_world_size == W
    peers_ok = True
    if m != "rccl" and ctx.device.type == "cuda" and 2 <= W <= 8 and single_node and supported:
        peers_ok = peer_report(ctx)[2]
        if not peers_ok and ctx.rank == 0:
            print("[dct] some rank pair is not peer-accessible (hipDeviceCanAccessPeer)", flush=True)
    eligible = (m != "rccl" and ctx.device.type == "cuda" and 2 <= W <= 8 and single_node and peers_ok
                and supported)
    # every rank must take the same decision before any collective below diverges
    if not ctx.all_reduce_bool_and(eligible):
        if m == "xgmi" and strict:
            raise RuntimeError("DCT_ALLREDUCE=xgmi but the in-kernel all-reduce is not applicable "
                               f"(world {W}, single node {single_node}, {what})")
        return None
    from ..ops._native import native

    xg, handle, err = None, b"", None
    try:
        xg = native().PeerExchange(W, ctx.rank, int(nbytes()))
        handle = xg.ipc_handle()
    except Exception as e:  # noqa: BLE001
        err = e
    handles = ctx.all_gather_object(handle)
    if err is None and all(handles):
        try:
            xg.open_peers(handles)
        except Exception as e:  # noqa: BLE001
            err = e
    ok = ctx.all_reduce_bool_and(err is None)
    if not ok:
        if m == "xgmi" and strict:
            raise RuntimeError(f"in-kernel all-reduce setup failed on some rank (this rank: {err!r})")
        if ctx.rank == 0:
            print(f"[dct] xGMI peer exchange unavailable ({err!r}); using RCCL per step", flush=True)
        return None
    return xg


def allreduce_adam_(xg, g, p, m, v, n_params: int, step_counter, lr: float, betas, eps: float,
                    weight_decay: float, timeout: Optional[float] = None):
    """Enqueue the fused peer all-reduce + Adam step (csrc/xg_adam.hip) on the current stream.

    ``g`` (fp32, the gradients then optionally the local loss) is replaced by the rank average -
    summed in rank order, so bit-identical on every rank - and Adam (L2 weight decay, step
    t = ``*step_counter``) updates ``p/m/v[:n_params]``.  Collective: every rank enqueues it once
    per step, after the kernel that advanced the step counter."""
    import torch

    from ..ops._native import native

    for t in (g, p, m, v):
        if not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()):
            raise ValueError("allreduce_adam_: g/p/m/v must be contiguous fp32 cuda tensors")
    if not (p.numel() == m.numel() == v.numel() == n_params <= g.numel()):
        raise ValueError("allreduce_adam_: p/m/v must hold n_params elements and g at least as many")
    if not (step_counter.is_cuda and step_counter.dtype == torch.int32):
        raise ValueError("allreduce_adam_: step_counter must be a cuda int32 tensor")
    native().xg_allreduce_adam(g.data_ptr(), p.data_ptr(), m.data_ptr(), v.data_ptr(), g.numel(), n_params,
                               step_counter.data_ptr(), float(lr), float(betas[0]), float(betas[1]), float(eps),
                               float(weight_decay), xg, timeout_s() if timeout is None else float(timeout),
                               torch.cuda.current_stream(p.device).cuda_stream)


def device_barrier(xg, stream: int, timeout: Optional[float] = None):
    """Enqueue a barrier over the peer mappings on ``stream`` (collective: every rank calls it).

    One wave writes a tag into every peer's barrier slot over xGMI and polls its own slots - no
    RCCL launch, no host round trip.  Followed by a device synchronize it is a full barrier: no
    rank's synchronize returns before every rank's stream reached the barrier.  A timeout is
    recorded in the status word (:func:`check` then reports the exchange as failed)."""
    xg.barrier(stream, timeout_s() if timeout is None else float(timeout))


def status(xg) -> int:
    """This rank's exchange status word (0 = ok, else the step + 1 that timed out); syncs."""
    return int(xg.read_status())


def check(xg, ctx: DistContext) -> int:
    """Collective: max over ranks of the status word (0 = every exchange completed)."""
    return ctx.all_reduce_max_int(status(xg))
