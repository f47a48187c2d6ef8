"""Native operator library.

``native()`` returns the compiled gfx950 extension (``fedmi/ops/_fedmi_hip*.so``: the
fused FL round kernels, the RCCL communicator, HIP-graph capture).  On a machine with a
GPU the extension is REQUIRED: every device code path goes through it and there is no
silent eager fallback -- if it is missing or fails to load, ``native()`` raises.  On a
CPU-only host, ``fedmi.fl.engine.TorchRoundEngine`` implements the same round math with
eager torch ops (used as the CPU plumbing path and as the numerics oracle in tests).
"""
from __future__ import annotations

import importlib
import os

_NATIVE = None
_NATIVE_ERR = None


def native(build_if_missing: bool = True):
    """Import (building in-tree first if needed) the native extension."""
    global _NATIVE, _NATIVE_ERR
    if _NATIVE is not None:
        return _NATIVE
    import torch  # noqa: F401  -- must load torch's libamdhip64/librccl before the extension
    alt = os.environ.get("FEDMI_NATIVE_SO")  # A/B measurements of alternative builds
    if alt:
        from importlib import util as _ilu
        spec = _ilu.spec_from_file_location("fedmi.ops._fedmi_hip", alt)
        mod = _ilu.module_from_spec(spec)
        spec.loader.exec_module(mod)
        _NATIVE = mod
        return _NATIVE
    try:
        _NATIVE = importlib.import_module("fedmi.ops._fedmi_hip")
        return _NATIVE
    except ImportError as e:  # not built yet
        _NATIVE_ERR = e
    if build_if_missing and os.environ.get("FEDMI_NO_BUILD", "0") != "1":
        from . import build as _b
        _b.build()
        _NATIVE = importlib.import_module("fedmi.ops._fedmi_hip")
        return _NATIVE
    raise ImportError(f"fedmi native extension unavailable: {_NATIVE_ERR}")


def native_available() -> bool:
    try:
        native(build_if_missing=False)
        return True
    except Exception:
        return False
