"""Tracing / debug utilities (CPU)."""
import time

import pytest

import dct_amd  # noqa: F401
from dct_amd.utils import debug
from dct_amd.utils.tracing import PhaseTimer, mark, trace_range


def test_trace_range_and_phase_timer_are_safe_without_gpu():
    t = PhaseTimer(sync_device=False)
    with t.phase("a"):
        time.sleep(0.01)
    with t.phase("a"):
        pass
    with trace_range("outer"):
        mark("hello")
    m = t.metrics()
    assert m["time/a_s"] >= 0.01 and t.counts["a"] == 2


def test_debug_reducer_assertion(monkeypatch):
    class R:
        num_buckets = 3
        launched = 2

    debug.assert_reducer_complete(R())  # disabled: no-op
    monkeypatch.setenv("DCT_DEBUG", "1")
    with pytest.raises(AssertionError):
        debug.assert_reducer_complete(R())
    R.launched = 3
    debug.assert_reducer_complete(R())


def test_native_build_relinks_when_the_object_set_changes(tmp_path, monkeypatch):
    """_build.build() links when the object list differs from the one recorded next to the .so,
    not only when something was recompiled: reverting a source finds its cached object, and the
    previously linked .so (built from the other version) must not survive.  hipcc is faked."""
    import subprocess

    from dct_amd import _build

    pkg, csrc, obj = tmp_path / "pkg", tmp_path / "pkg" / "csrc", tmp_path / "build" / "obj"
    csrc.mkdir(parents=True)
    (csrc / "a.hip").write_text("v1")
    monkeypatch.setattr(_build, "PKG_DIR", str(pkg))
    monkeypatch.setattr(_build, "CSRC", str(csrc))
    monkeypatch.setattr(_build, "BUILD", str(obj))
    monkeypatch.setattr(_build, "_flags", lambda debug=False: ["-O3"])
    links = []

    def fake_run(cmd, capture_output=True, text=True):
        out = cmd[cmd.index("-o") + 1]
        with open(out, "w") as f:
            f.write(" ".join(cmd))
        if "-shared" in cmd:
            links.append([c for c in cmd if c.endswith(".o")])
        return subprocess.CompletedProcess(cmd, 0, "", "")

    monkeypatch.setattr(_build.subprocess, "run", fake_run)
    _build.build()
    assert len(links) == 1 and not _build.is_stale()
    _build.build()
    assert len(links) == 1  # nothing changed: no relink
    (csrc / "a.hip").write_text("v2")
    _build.build()
    assert len(links) == 2  # recompiled -> relinked
    (csrc / "a.hip").write_text("v1")  # revert: the v1 object is cached, no compile ...
    _build.build()
    assert len(links) == 3 and links[2] == links[0]  # ... but the .so is relinked from it
    assert not _build.is_stale()


class _StubCtx:
    """Just what parallel/xgmi.py's exchange setup asks of a DistContext (one process stands for
    every rank: the collective AND of a decision is the local value)."""

    def __init__(self, world, device="cpu", local_world=None):
        import torch

        self.world_size, self.rank = world, 0
        self.local_world_size = world if local_world is None else local_world
        self.device = torch.device(device)
        self.calls = []

    def all_reduce_bool_and(self, v):
        self.calls.append(bool(v))
        return bool(v)


@pytest.mark.parametrize("env,world,local,dev", [({}, 2, None, "cpu"), ({}, 1, None, "cpu"),
                                                 ({"DCT_XG_GRAD": "0"}, 2, None, "cpu"),
                                                 ({"DCT_ALLREDUCE": "rccl"}, 8, None, "cpu"),
                                                 ({}, 16, 8, "cpu")])
def test_grad_exchange_setup_declines_collectively(env, world, local, dev, monkeypatch):
    """setup_grad_exchange (the 3x128 DDP step's peer all-reduce + Adam kernel) is only taken with
    every rank on one node, on GPUs, 2..8 ranks and not turned off; otherwise every rank gets None
    after one collective decision (so no rank goes on to export IPC handles alone), and
    DCT_ALLREDUCE=xgmi does not make its absence an error (RCCL remains the step path)."""
    from dct_amd.parallel.xgmi import setup_grad_exchange

    for k in ("DCT_XG_GRAD", "DCT_ALLREDUCE"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    ctx = _StubCtx(world, dev, local)
    assert setup_grad_exchange(ctx, 17539) is None
    assert ctx.calls == [False]
    monkeypatch.setenv("DCT_ALLREDUCE", "xgmi")
    ctx = _StubCtx(world, dev, local)
    assert setup_grad_exchange(ctx, 17539) is None


def test_xg_adam_buffer_size_matches_the_kernel_layout():
    """[2 parities][W ranks][ceil(n / 2) element pairs] x 16-B granules (csrc/xg_adam.hip)."""
    from dct_amd.ops._native import native

    nat = native()
    assert nat.xg_adam_buffer_bytes(17539, 8) == 2 * 8 * 8770 * 16
    assert nat.xg_adam_buffer_bytes(4, 2) == 2 * 2 * 2 * 16
