"""Debug run mode (SURVEY §5.2 race detection; the reference has none).

``DCT_DEBUG=1`` turns on:
  * device-synchronised error checks after every engine phase (``check_device``), so an
    asynchronous HIP fault is reported at the phase that caused it (the HIP_LAUNCH_BLOCKING idea
    without serialising every launch of the runtime);
  * stream-ordering assertions of the bucketed reducer: every bucket must have been launched
    before the optimizer reads the gradients (``assert_reducer_complete``).
Host-side C++ can additionally be built with ASan (``DCT_SANITIZE=1 python -m dct_amd._build``,
host code only: ``-Xarch_host -fsanitize=address``).
"""
from __future__ import annotations

import os


def enabled() -> bool:
    return os.environ.get("DCT_DEBUG", "0") == "1"


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
