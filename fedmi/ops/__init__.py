"""Native operator library.

``native()`` returns the compiled gfx950 extension (``fedmi/ops/_fedmi_hip*.so``: the
fused FL round kernels, the RCCL communicator, HIP-graph capture).  On a machine with a
GPU the extension is REQUIRED: every device code path goes through it and there is no
silent eager fallback -- if it is missing or fails to load, ``native()`` raises.  A binary
is only loaded if the source digest compiled into it matches this tree's sources
(``build.so_digest`` / ``build.build_digest``): a stale ``.so`` is rebuilt (under a file
lock, so concurrent ranks build once) or, with ``FEDMI_NO_BUILD=1``, refused.  On a
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
    from . import build as _b
    if not _b.is_fresh():
        have = _b.so_digest(_b.TARGET)
        why = ("not built" if not os.path.isfile(_b.TARGET) else
               f"stale (built from sources {have}, tree is {_b.build_digest()})")
        if not build_if_missing or os.environ.get("FEDMI_NO_BUILD", "0") == "1":
            raise ImportError(f"fedmi native extension {why}: run `python -m fedmi.ops.build`")
        import sys
        print(f"[fedmi] native extension {why}; building", file=sys.stderr, flush=True)
        _b.build()
    try:
        _NATIVE = importlib.import_module("fedmi.ops._fedmi_hip")
    except ImportError as e:
        _NATIVE_ERR = e
        raise ImportError(f"fedmi native extension unavailable: {_NATIVE_ERR}") from e
    return _NATIVE


def native_available() -> bool:
    try:
        native(build_if_missing=False)
        return True
    except Exception:
        return False
