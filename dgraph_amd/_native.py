"""Loader for the native op library ``dgraph_amd/_C.so``.

GPU tensors always go through the hand-written HIP kernels; if the library is missing
on a machine with a GPU, every native op raises (no silent eager fallback). CPU tensors
use the pure-PyTorch reference implementations in :mod:`dgraph_amd.ops.reference`, which
double as the numerics oracle in the tests.
"""
from __future__ import annotations

import os
import threading
from pathlib import Path

import torch

_LIB_PATH = Path(__file__).resolve().parent / "_C.so"
_lock = threading.Lock()
_loaded = False
_load_error: Exception | None = None


def library_path() -> Path:
    return _LIB_PATH


def load(build_if_missing: bool | None = None) -> bool:
    """Load ``_C.so`` into the torch dispatcher. Returns True when available."""
    global _loaded, _load_error
    with _lock:
        if _loaded:
            return True
        if build_if_missing is None:
            build_if_missing = os.environ.get("DGRAPH_AUTOBUILD", "1") == "1"
        if not _LIB_PATH.exists() and build_if_missing:
            try:
                from . import _build

                _build.build(verbose=False)
            except Exception as e:  # pragma: no cover - build env problems
                _load_error = e
                return False
        if not _LIB_PATH.exists():
            _load_error = FileNotFoundError(str(_LIB_PATH))
            return False
        try:
            torch.ops.load_library(str(_LIB_PATH))
            _loaded = True
        except Exception as e:  # pragma: no cover
            _load_error = e
            return False
        return True


def available() -> bool:
    return load()


def ops():
    """Return ``torch.ops.dgraph_amd`` or raise loudly."""
    if not load():
        raise RuntimeError(
            f"dgraph_amd native library unavailable ({_load_error}); "
            "run `python -m dgraph_amd._build` — GPU ops never fall back to eager PyTorch"
        )
    return torch.ops.dgraph_amd
