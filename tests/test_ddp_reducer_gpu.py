"""The DDP bucket-reducer paths of the wide models on ONE GPU (DCT_FORCE_DDP=1: a one-rank RCCL
communicator and the native BucketReducer - the path BASELINE configs 4/5 take at DDP=8,
reference jobs/train_lightning_ddp.py:136).  The correctness tests set DCT_RCCL_ONE_RANK=1, so
RCCL's one-rank all-reduce really runs (a one-rank communicator otherwise skips the identity) and
the auto placement puts it on the reducer's comm stream, as at W > 1:

(a) the trajectories equal the no-reducer path (ncclAvg over one rank is the identity);
(b) buckets are ENQUEUED from the backward hooks before finalize() (launch order only - that by
    itself proves no overlap); in the autograd engine the post-accumulate-grad hooks fire although
    the fused ops write the weight gradients straight into p.grad and return None;
(c) allreduce_ms is measured on the device (span and exposed time, also inside replayed graphs)
    and the debug-mode stream-ordering check stays clean;
(d) OVERLAP, with a stand-in collective (DCT_REDUCER_STANDIN_US: a busy kernel of fixed duration
    on the collective's stream, the footprint of a multi-rank all-reduce): on the comm stream the
    exposed all-reduce time is a fraction of its span, on the compute stream it is all of it.
"""
import json
import os
import subprocess
import sys

import pytest
import torch

import dct_amd  # noqa: F401
from dct_amd.models.mlp import MLPClassifier
from dct_amd.models.tabtransformer import TabTransformer
from dct_amd.parallel.dist import init_distributed
from dct_amd.trainer.engines import AutogradEngine, adam_hparams_from
from dct_amd.trainer.graph_engine import GraphMLPEngine
from dct_amd.trainer.trainer import seed_everything

pytestmark = pytest.mark.gpu


def _data(n, d, seed=0):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(n, d, generator=g)
    w = torch.randn(d, generator=g)
    return X, ((X @ w) > 0).long()


def _tabular(forced, monkeypatch, B=1024, epochs=2):
    monkeypatch.setenv("DCT_FORCE_DDP", "1" if forced else "0")
    monkeypatch.setenv("DCT_RCCL_ONE_RANK", "1")
    monkeypatch.setenv("DCT_DEBUG", "1")
    dims = [256, 1024, 1024, 1024, 2]
    torch.manual_seed(0)
    model = MLPClassifier(dims[0], hidden=tuple(dims[1:-1]), num_classes=2, dropout=0.0, loss="mse", lr=1e-3)
    ctx = init_distributed("gpu")
    eng = GraphMLPEngine(model, ctx, B, seed=42, adam=adam_hparams_from(model.configure_optimizers()))
    X, Y = _data(8 * B, dims[0], seed=5)
    rows = torch.arange(X.shape[0])
    eng.attach_data(X, Y, rows, rows[:B])
    losses = torch.cat([eng.train_epoch(ep).cpu() for ep in range(epochs)])
    torch.cuda.synchronize()
    return eng, losses


def test_tabular_forced_reducer_matches_no_reducer(cuda, monkeypatch):
    ref, l0 = _tabular(False, monkeypatch)
    assert ref.reducer is None
    eng, l1 = _tabular(True, monkeypatch)
    red = eng.reducer
    assert red is not None and red.num_buckets >= 2
    assert not red._r.inline_mode  # a real (one-rank) RCCL collective: auto placement = comm stream
    assert red._r.edge_timeouts() == 0  # every eager fork / join edge saw its producer
    # (a) same trajectory: the reducer path reduces the split-K dW slices into g before the bucket
    # launch, the no-reducer path sums the same slices in the same order inside Adam
    assert torch.isfinite(l1).all()
    assert torch.allclose(l0, l1, atol=1e-3), (l0 - l1).abs().max()
    assert (eng.p.cpu() - ref.p.cpu()).norm() / ref.p.cpu().norm() < 1e-2
    # (b) buckets were launched from the per-layer mark_ready calls during backward, before finalize
    # (every one of them, when the input layer's gradients complete the last bucket)
    assert 1 <= red.launched_before_finalize <= red.num_buckets, (red.launched_before_finalize, red.num_buckets)
    # (c) device-measured all-reduce time of every step (graph replays included), no ordering fault
    span, exposed, steps, bad = red.allreduce_ms(reset=False)
    assert steps >= len(l1) and span > 0 and 0 <= exposed <= span + 1e-3, (span, exposed, steps)
    assert bad == 0
    red.wait_s = 0.0  # the Trainer's reset
    assert red.allreduce_ms()[2] == 0


def test_tabular_reducer_on_reserved_cus(cuda, monkeypatch):
    """CU reservation (profiles/ddp_reducer_cu_reservation_r6.log): the step on a stream masked to every
    CU but 8, the reducer's collectives on a stream masked to those 8 (no collective kernel can share a
    CU with the backward's LDS-DMA GEMM tiles).  The masks round-trip, the reducer reports the
    reserved set, and training follows the no-reducer trajectory as in (a)."""
    from dct_amd.ops._native import native

    nat = native()
    ncu = nat.device_cu_count()
    assert ncu >= 64
    words = (ncu + 31) // 32
    full = [0xFFFFFFFF if 32 * (w + 1) <= ncu else (1 << (ncu - 32 * w)) - 1 for w in range(words)]
    comm = [0] * words
    for c in range(0, ncu, ncu // 8):
        comm[c // 32] |= 1 << (c % 32)
    compute = [f & ~c for f, c in zip(full, comm)]
    h = nat.cu_masked_stream(compute)
    try:
        assert list(nat.stream_cu_mask(h)) == compute
        ref, l0 = _tabular(False, monkeypatch)
        with torch.cuda.stream(torch.cuda.ExternalStream(h)):
            monkeypatch.setenv("DCT_FORCE_DDP", "1")
            monkeypatch.setenv("DCT_RCCL_ONE_RANK", "1")
            monkeypatch.setenv("DCT_DEBUG", "1")
            dims = [256, 1024, 1024, 1024, 2]
            torch.manual_seed(0)
            model = MLPClassifier(dims[0], hidden=tuple(dims[1:-1]), num_classes=2, dropout=0.0, loss="mse", lr=1e-3)
            ctx = init_distributed("gpu")
            eng = GraphMLPEngine(model, ctx, 1024, seed=42, adam=adam_hparams_from(model.configure_optimizers()))
            eng.reducer._r.set_comm_cu_mask(comm)
            assert list(eng.reducer._r.comm_cu_mask) == comm
            assert list(nat.stream_cu_mask(eng.reducer._r.comm_stream)) == comm
            X, Y = _data(8 * 1024, dims[0], seed=5)
            rows = torch.arange(X.shape[0])
            eng.attach_data(X, Y, rows, rows[:1024])
            l1 = torch.cat([eng.train_epoch(ep).cpu() for ep in range(2)])
        torch.cuda.synchronize()
        assert eng.reducer._r.edge_timeouts() == 0
        assert torch.isfinite(l1).all()
        assert torch.allclose(l0, l1, atol=1e-3), (l0 - l1).abs().max()
        assert (eng.p.cpu() - ref.p.cpu()).norm() / ref.p.cpu().norm() < 1e-2
    finally:
        torch.cuda.synchronize()
        nat.stream_destroy(h)


def _tt(forced, monkeypatch, defer="1", steps=10, B=128, groups="1"):
    monkeypatch.setenv("DCT_FORCE_DDP", "1" if forced else "0")
    monkeypatch.setenv("DCT_TT_DW_DEFER", defer)
    monkeypatch.setenv("DCT_TT_DDP_GROUPS", groups)
    monkeypatch.setenv("DCT_RCCL_ONE_RANK", "1")
    monkeypatch.setenv("DCT_DEBUG", "1")
    ctx = init_distributed("gpu")
    F_ = 64
    X, Y = _data(4096, F_, seed=4)
    rows = torch.randperm(4096, generator=torch.Generator().manual_seed(2))
    seed_everything(7)
    m = TabTransformer(num_features=F_, d_model=64, heads=4, layers=3, lr=3e-3)
    eng = AutogradEngine(m, ctx, B, seed=7)
    eng.attach_data(X.to(cuda_dev()), Y.to(cuda_dev()), rows[:3584], rows[3584:])
    rows_dev = eng.train_rows.to(cuda_dev())
    loss = torch.zeros(steps, device=cuda_dev())
    eng.run_device_steps(rows_dev, 0, steps, loss)  # eager warm-up steps, capture, replays
    torch.cuda.synchronize()
    return eng, loss.cpu(), eng.flat_p.detach().cpu().clone()


def cuda_dev():
    return torch.device("cuda", 0)


@pytest.mark.parametrize("defer,groups", [("1", "1"), ("1", "0"), ("0", "1")])
def test_tabtransformer_forced_reducer_matches_no_reducer(cuda, monkeypatch, defer, groups):
    ref, l0, p0 = _tt(False, monkeypatch, defer)
    _, lh, ph = _tt(False, monkeypatch, defer)  # run-to-run spread of the split-K atomics
    eng, l1, p1 = _tt(True, monkeypatch, defer, groups=groups)
    red = eng.reducer
    assert ref.reducer is None and red is not None and eng.graph_used
    assert torch.isfinite(l1).all() and (l1 != 0).all()
    assert torch.allclose(l0, l1, rtol=2e-3, atol=2e-4), (l0, l1)
    noise = float((p0 - ph).norm() / p0.norm())
    diff = float((p0 - p1).norm() / p0.norm())
    assert diff < max(3 * noise, 1e-4), (diff, noise)
    if defer == "0":
        # (b) the hooks fired during backward although the fused ops return None for the weight
        # gradients they accumulate in place, and they launched the bucket before finalize
        assert red.hook_launches >= 1 and not red.defer_launch
    elif groups == "1":
        # grouped deferred dW in two block groups (model.ddp_block_groups): buckets aligned with the
        # groups, each group's dW issued inside its last block's backward, so the first bucket
        # launches from the hooks before finalize and its all-reduce overlaps the lower blocks
        assert not red.defer_launch and red.num_buckets >= 2
        assert red.hook_launches >= 1 and red.launched_before_finalize >= 1, (red.hook_launches,
                                                                            red.launched_before_finalize)
    else:
        # grouped deferred dW for every block at once (DCT_TT_DDP_GROUPS=0): the hooks only count,
        # every bucket launches at finalize after the grouped launch (one bucket)
        assert red.defer_launch and red.num_buckets == 1
    span, exposed, steps, bad = red.allreduce_ms()
    assert steps >= 1 and span > 0 and bad == 0, (span, exposed, steps, bad)


def test_tabtransformer_comm_stream_in_graph_matches_no_reducer(cuda, monkeypatch):
    """DCT_REDUCER_INLINE=0 with the graph-replayed TabTransformer step: the captured collectives sit
    on a graph branch behind event edges (the auto placement runs them inline while capturing) -
    the same trajectory as without a reducer, and the eager warm-up steps' device-counter edges all
    saw their producers."""
    monkeypatch.setenv("DCT_REDUCER_INLINE", "0")
    ref, l0, p0 = _tt(False, monkeypatch)
    eng, l1, p1 = _tt(True, monkeypatch)
    red = eng.reducer
    assert eng.graph_used and not red._r.inline_mode
    assert red._r.edge_timeouts() == 0
    assert torch.isfinite(l1).all() and torch.allclose(l0, l1, rtol=2e-3, atol=2e-4), (l0, l1)
    span, exposed, steps, bad = red.allreduce_ms()
    assert steps >= 1 and span > 0 and bad == 0, (span, exposed, steps, bad)


def test_phase_timer_reports_step_phases(cuda, monkeypatch):
    """DCT_PHASE_TIMING=1: device timestamps of forward / backward / all-reduce / optimizer, also
    inside the captured step graphs."""
    monkeypatch.setenv("DCT_PHASE_TIMING", "1")
    eng, loss, _ = _tt(True, monkeypatch, "1", steps=8)
    ph = eng.phase_timer.read()
    assert ph["steps"] >= 8
    for k in ("fwd", "bwd", "allreduce", "opt"):
        assert ph[k] > 0, ph
    assert ph["bwd"] > ph["allreduce"]


def _tabular_step_us(standin_us, inline, out_path, steps=64, B=4096):
    """Forced-DDP tabular 4x1024 step time (us, CUDA events over `steps` eager steps) with a
    stand-in collective of `standin_us` per step; inline: "1" compute stream, "-2" auto.  Run in a
    fresh process (_spawn): a process's streams share GPU_MAX_HW_QUEUES (4) hardware queues round-
    robin, and once earlier tests' engines hold enough streams the comm stream lands on the compute
    stream's queue, where its collectives serialise with backward again."""
    os.environ.update({"DCT_REDUCER_STANDIN_US": str(standin_us), "DCT_REDUCER_INLINE": inline,
                       "DCT_REDUCER_TIMING": "1", "DCT_DEBUG": "0", "DCT_FORCE_DDP": "1"})
    os.environ.pop("DCT_RCCL_ONE_RANK", None)
    dims = [256, 1024, 1024, 1024, 2]
    torch.manual_seed(0)
    model = MLPClassifier(dims[0], hidden=tuple(dims[1:-1]), num_classes=2, dropout=0.0, loss="mse", lr=1e-3)
    ctx = init_distributed("gpu")
    eng = GraphMLPEngine(model, ctx, B, seed=42, adam=adam_hparams_from(model.configure_optimizers()))
    X, Y = _data(steps * B, dims[0], seed=5)
    rows = torch.arange(X.shape[0])
    eng.attach_data(X, Y, rows, rows[:B])
    eng.train_epoch(0)
    eng.reducer.allreduce_ms(reset=True)
    n = eng.upload_epoch_indices(1)
    loss = torch.zeros(steps, device="cuda")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    eng.run_steps(n, steps, loss)
    e1.record()
    torch.cuda.synchronize()
    span, exposed, k, bad = eng.reducer.allreduce_ms()
    res = {"step_us": e0.elapsed_time(e1) * 1e3 / steps, "span_us": span * 1e3 / max(k, 1),
           "exposed_us": exposed * 1e3 / max(k, 1), "inline": bool(eng.reducer._r.inline_mode), "steps": k,
           "bad": bad, "timeouts": eng.reducer._r.edge_timeouts()}
    json.dump(res, open(out_path, "w"))


def _spawn(fn, *args, timeout=300):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = (f"import sys; sys.path.insert(0, {root!r}); sys.path.insert(0, {os.path.join(root, 'tests')!r}); "
            f"import test_ddp_reducer_gpu as t; t.{fn}(*{args!r})")
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=timeout)


def test_tabular_standin_collective_overlaps_backward(cuda, tmp_path):
    """(d) A 60 us stand-in all-reduce per step (split over the buckets by size, 16 one-wave busy
    workgroups; about an 8-rank all-reduce of the 13.6 MB of fp32 gradients over xGMI).  With the
    auto placement (comm stream) most of it runs under the remaining backward: the step grows by
    well under the stand-in's 60 us and the exposed time (end of backward -> last bucket done) is a
    fraction of the span.  Forced onto the compute stream it serialises: the step grows by ~60 us."""
    res = {}
    for name, us, inline in (("base", 0, "-2"), ("comm", 60, "-2"), ("inline", 60, "1")):
        out = tmp_path / f"{name}.json"
        r = _spawn("_tabular_step_us", us, inline, str(out))
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        res[name] = json.loads(out.read_text())
        assert res[name]["steps"] == 64 and res[name]["bad"] == 0 and res[name]["timeouts"] == 0, res[name]
    base, comm, inl = res["base"]["step_us"], res["comm"]["step_us"], res["inline"]["step_us"]
    span_c, exp_c = res["comm"]["span_us"], res["comm"]["exposed_us"]
    print(f"forced-DDP tabular step: no stand-in {base:.1f} us, 60 us stand-in on the comm stream {comm:.1f} us "
          f"(span {span_c:.1f}, exposed {exp_c:.1f}), on the compute stream {inl:.1f} us")
    assert not res["comm"]["inline"] and res["inline"]["inline"]
    assert span_c >= 55.0, span_c  # the stand-in ran
    assert inl - base > 45.0, (inl, base)  # serialised on the compute stream
    assert exp_c < 0.5 * span_c, (span_c, exp_c)
    assert comm - base < 0.5 * (inl - base), (base, comm, inl)
