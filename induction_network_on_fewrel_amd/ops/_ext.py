"""Loader for the in-tree gfx950 kernel library (``_ina_kernels.so``).

The GPU execution path has NO silent fallback: if a CUDA(HIP) device is used and the library is
missing or fails to load, ``ops()`` raises. Build it with ``python csrc/build.py`` (or
``__graft_entry__.build()``).
"""
from __future__ import annotations

import os
import threading

import torch

# INA_KERNEL_LIB selects an experiment build (csrc/build.py with INA_BUILD_TAG); default: in-tree.
_LIB = os.environ.get("INA_KERNEL_LIB") or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                        "_ina_kernels.so")
_lock = threading.Lock()
_loaded = False
_error = None


def library_path() -> str:
    return _LIB


def load(build_if_missing: bool = False) -> bool:
    global _loaded, _error
    with _lock:
        if _loaded:
            return True
        if not os.path.exists(_LIB) and build_if_missing:
            import importlib.util
            spec = importlib.util.spec_from_file_location(
                "ina_build", os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(_LIB))), "csrc", "build.py"))
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
            mod.build()
        try:
            torch.ops.load_library(_LIB)
            _loaded = True
        except Exception as e:  # pragma: no cover - surfaced loudly by ops()
            _error = e
            return False
        return True


def available() -> bool:
    return load()


def ops():
    """``torch.ops.ina`` -- raises if the native library cannot be loaded."""
    if not load():
        raise RuntimeError(f"Induction-Network HIP kernel library not available at {_LIB}: {_error!r}. "
                           "Build it with `python csrc/build.py`.")
    return torch.ops.ina
