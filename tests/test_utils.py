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
