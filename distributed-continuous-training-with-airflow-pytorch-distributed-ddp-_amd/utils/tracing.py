"""Tracing / timing (the reference has none).

* ``trace_range(name)`` - a roctx range (rocprofiler-sdk's roctx) around a phase, so rocprofv3
  ``--marker-trace`` timelines show epoch / train / validate / checkpoint / all-reduce phases
  next to the kernels; a no-op when the library is missing or ``DCT_ROCTX=0``.
* ``PhaseTimer`` - wall-clock accumulation per host phase (device-synchronised on demand): the
  Trainer reports its epoch phases (train / validate / checkpoint / tracking flush) as
  ``time/<phase>_s`` metrics.
* ``DevicePhaseTimer`` - GPU time of the phases INSIDE a training step (forward, backward,
  all-reduce, optimizer): one-thread kernels write ``s_memrealtime`` at each phase mark on the
  compute stream and one more accumulates the deltas on the device, so it also works inside
  captured / replayed HIP graphs (host timers and event pairs do not); ``DCT_PHASE_TIMING=1``
  turns it on in the autograd engine and the Trainer logs ``time/<phase>_s`` per epoch.
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


class DevicePhaseTimer:
    """Per-step GPU phase timing with device timestamps (see the module docstring).

    ``mark(i)`` for i = 0 .. len(phases) on the current stream delimit the phases of one step,
    ``close()`` after the last mark accumulates them; ``read()`` synchronises and returns seconds
    per phase summed over the steps since the last reset."""

    def __init__(self, phases, device):
        import torch

        self.phases = list(phases)
        self.n = len(self.phases) + 1  # marks
        self.buf = torch.zeros(2 * self.n, dtype=torch.int64, device=device)

    def _nat(self):
        from ..ops._native import native

        return native()

    def mark(self, i: int):
        import torch

        self._nat().phase_stamp(self.buf.data_ptr(), int(i), torch.cuda.current_stream().cuda_stream)

    def close(self):
        import torch

        self._nat().phase_accum(self.buf.data_ptr(), self.n, torch.cuda.current_stream().cuda_stream)

    def read(self, reset: bool = True) -> Dict[str, float]:
        import torch

        torch.cuda.synchronize(self.buf.device)
        v = self.buf.cpu().tolist()
        out = {name: v[self.n + i] / 1e8 for i, name in enumerate(self.phases)}  # 100 MHz ticks -> s
        out["steps"] = v[2 * self.n - 1]
        if reset:
            self.buf[self.n:].zero_()
        return out
