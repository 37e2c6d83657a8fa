"""Loader for the in-tree native extension ``_dct_native``.

GPU code paths call :func:`native` which returns the module or RAISES - there is no silent
eager fallback on a GPU box (a missing or stale extension is a build error, not a slow path).
CPU-only code paths (the gloo plumbing config, unit tests) never touch it.
"""
from __future__ import annotations

import importlib
import os
import threading

import torch  # noqa: F401  - load torch's HIP runtime / RCCL before ours (same sonames)

_lock = threading.Lock()
_mod = None
_err = None


def _pkg_name() -> str:
    return __name__.rsplit(".", 2)[0]


def load(build_if_missing: bool = True):
    """Import the extension, (re)building it with hipcc if it is missing or stale."""
    global _mod, _err
    with _lock:
        if _mod is not None:
            return _mod
        from .. import _build

        try:
            if build_if_missing and os.environ.get("DCT_NO_BUILD", "0") != "1" and _build.is_stale():
                _build.build()
            _mod = importlib.import_module(_pkg_name() + "._dct_native")
        except Exception as e:  # noqa: BLE001
            _err = e
            raise
        return _mod


def native():
    if _mod is not None:
        return _mod
    try:
        return load()
    except Exception as e:  # noqa: BLE001
        raise RuntimeError(
            "dct_amd native extension (_dct_native, HIP/gfx950) is not available: "
            f"{e!r}. Build it with `python -m dct_amd._build` (hipcc --offload-arch=gfx950)."
        ) from e


def reload_knobs() -> None:
    """Re-read the native launchers' DCT_* knobs (csrc/knobs.h).  Plan / bind time only: the
    launch paths read the struct, never the environment."""
    native().reload_knobs()


def available() -> bool:
    try:
        native()
        return True
    except Exception:  # noqa: BLE001
        return False


def stream_handle(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()
