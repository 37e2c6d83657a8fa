"""Debug run mode (SURVEY §5.2 race detection; the reference has none).

``DCT_DEBUG=1`` turns on:
  * device-synchronised error checks after every engine phase (``check_device``), so an
    asynchronous HIP fault is reported at the phase that caused it (the HIP_LAUNCH_BLOCKING idea
    without serialising every launch of the runtime);
  * stream-ordering assertions of the bucketed reducer: every bucket must have been launched
    before the optimizer reads the gradients (``assert_reducer_complete``), and - on the native
    RCCL reducer - a device-side check that the optimizer's stream really waited for the comm
    stream's done event: a one-thread kernel on the compute stream, right after the join,
    compares the comm stream's per-step close counter with its own step count and latches a
    violation flag (csrc/step_kernels.hip reducer_check_kernel; it runs inside replayed HIP
    graphs too), read by ``assert_reducer_ordering`` at the end of every epoch.
Host-side C++ can additionally be built with ASan (``DCT_SANITIZE=1 python -m dct_amd._build``,
host code only: ``-Xarch_host -fsanitize=address``).
"""
from __future__ import annotations

import os


def enabled() -> bool:
    return os.environ.get("DCT_DEBUG", "0") == "1"


def reducer_timing_enabled() -> bool:
    """Device-side all-reduce timing of the bucket reducers (allreduce_ms): opt-in with
    DCT_REDUCER_TIMING=1 or DCT_DEBUG=1 (it costs every step two stamp kernels and a
    cross-stream edge, so the default training step is the one bench.py times)."""
    return os.environ.get("DCT_REDUCER_TIMING", "0") == "1" or enabled()


def check_device(what: str):
    if not enabled():
        return
    import torch

    if torch.cuda.is_available() and torch.cuda.is_initialized():
        try:
            torch.cuda.synchronize()
        except Exception as e:  # noqa: BLE001
            raise RuntimeError(f"[dct debug] device error after {what}: {e}") from e


def assert_reducer_complete(reducer):
    if not enabled() or reducer is None:
        return
    launched = getattr(reducer, "launched", None)
    if callable(launched):
        launched = launched()
    if launched is None and hasattr(reducer, "_r"):
        launched = reducer._r.launched
    n = reducer.num_buckets
    if launched is not None and launched != n:
        raise AssertionError(f"[dct debug] optimizer step with {launched}/{n} gradient buckets all-reduced")


def assert_reducer_ordering(reducer, where: str = "epoch end"):
    """Debug mode: raise if the device-side ordering check of the native reducer latched a
    violation (the compute stream ran the optimizer before the comm stream finished)."""
    if not enabled() or reducer is None or not hasattr(reducer, "allreduce_ms"):
        return
    t = reducer.allreduce_ms(reset=False)
    if t is not None and t[3] > 0:
        raise AssertionError(f"[dct debug] {where}: the optimizer stream did not wait for the gradient "
                             f"all-reduce ({t[3]} ordering violation(s) over {t[2]} steps)")
