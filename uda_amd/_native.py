"""Loader for the in-tree native runtime (uda_amd/_uda_native*.so + uda_amd/lib/libuda.so).

torch is imported first on purpose: torch ships its own libamdhip64/librccl, and loading them
before libuda.so makes the dynamic loader resolve libuda's HIP/RCCL dependencies (same sonames)
to those copies, so the process has exactly one HIP runtime.
"""
from __future__ import annotations

import importlib
import os

import torch  # noqa: F401  (must precede the native import, see module docstring)

_native = None
_error: Exception | None = None


def native():
    """Return the native module, raising a clear error if the extension was not built."""
    global _native, _error
    if _native is not None:
        return _native
    try:
        _native = importlib.import_module("uda_amd._uda_native")
    except ImportError as e:  # pragma: no cover - exercised only on a broken build
        _error = e
        raise ImportError(
            "uda_amd native extension is missing; build it with `python tools/build.py` "
            f"(original error: {e})") from e
    return _native


def available() -> bool:
    try:
        native()
        return True
    except ImportError:
        return False


def lib_path() -> str:
    return os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libuda.so")
