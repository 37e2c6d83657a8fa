"""Tracing / timing (the reference has none).

* ``trace_range(name)`` - a roctx range (rocprofiler-sdk's roctx) around a phase, so rocprofv3
  ``--marker-trace`` timelines show epoch / train / validate / checkpoint / all-reduce phases
  next to the kernels; a no-op when the library is missing or ``DCT_ROCTX=0``.
* ``PhaseTimer`` - wall-clock accumulation per phase (device-synchronised on demand), reported
  by the Trainer as extra metrics (``time/<phase>_s``).
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import time
from collections import defaultdict
from typing import Dict, Optional

_roctx = None
_roctx_tried = False


def _lib():
    global _roctx, _roctx_tried
    if _roctx_tried:
        return _roctx
    _roctx_tried = True
    if os.environ.get("DCT_ROCTX", "1") == "0":
        return None
    rocm_lib = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib")
    # rocprofiler-sdk's roctx first: rocprofv3 (--marker-trace) intercepts that one; the legacy
    # roctracer libroctx64 is only seen by the old rocprof
    for name in ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so",
                 os.path.join(rocm_lib, "librocprofiler-sdk-roctx.so"), "libroctx64.so", "libroctx64.so.4",
                 os.path.join(rocm_lib, "libroctx64.so")):
        try:
            lib = ctypes.CDLL(name)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.restype = ctypes.c_int
            lib.roctxMarkA.argtypes = [ctypes.c_char_p]
            _roctx = lib
            break
        except OSError:
            continue
    return _roctx


def mark(msg: str):
    lib = _lib()
    if lib is not None:
        lib.roctxMarkA(msg.encode())


@contextlib.contextmanager
def trace_range(name: str):
    lib = _lib()
    if lib is None:
        yield
        return
    lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        lib.roctxRangePop()


class PhaseTimer:
    def __init__(self, sync_device: Optional[bool] = None):
        self.totals: Dict[str, float] = defaultdict(float)
        self.counts: Dict[str, int] = defaultdict(int)
        self.sync = sync_device

    def _sync(self):
        if self.sync:
            import torch

            if torch.cuda.is_available() and torch.cuda.is_initialized():
                torch.cuda.synchronize()

    @contextlib.contextmanager
    def phase(self, name: str):
        self._sync()
        t0 = time.perf_counter()
        with trace_range(name):
            yield
        self._sync()
        self.totals[name] += time.perf_counter() - t0
        self.counts[name] += 1

    def metrics(self, prefix: str = "time/") -> Dict[str, float]:
        return {f"{prefix}{k}_s": v for k, v in self.totals.items()}
