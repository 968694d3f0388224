"""Loader for the in-tree native extension ``multidisttorch_amd/_C.so``.

Policy (no silent fallbacks on the GPU): when a GPU is present every HIP op
*requires* the extension and raises if it is missing or fails to load. On a
CPU-only host the pure-torch reference implementations are used instead and
are clearly labelled as such (``backend == "torch"``).
"""

from __future__ import annotations

import importlib
import importlib.util
import os
import sys

import torch

_MOD = None
_ERR = None


def _load():
    global _MOD, _ERR
    if _MOD is not None or _ERR is not None:
        return _MOD
    try:
        alt = os.getenv("MDT_NATIVE_SO")  # e.g. the host-sanitized build (_build.py, MDT_SANITIZE=1)
        if alt:
            spec = importlib.util.spec_from_file_location("multidisttorch_amd._C", alt)
            _MOD = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(_MOD)
            sys.modules["multidisttorch_amd._C"] = _MOD
        else:
            _MOD = importlib.import_module("multidisttorch_amd._C")
    except Exception as e:  # pragma: no cover - exercised when the .so is absent
        _ERR = e
        _MOD = None
    return _MOD


def available() -> bool:
    return _load() is not None


def load_error():
    _load()
    return _ERR


def require():
    """Return the extension module or raise a loud, actionable error."""
    m = _load()
    if m is None:
        raise RuntimeError(
            "multidisttorch_amd native extension (_C.so) is not available: "
            f"{_ERR!r}. Build it with `python -m multidisttorch_amd._build` "
            "(hipcc --offload-arch=gfx950).")
    return m


def so_path() -> str:
    return os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_C.so")


def ensure_built(jobs: int = 8):
    """Build the extension in-tree if it is missing (used by tests / build())."""
    global _MOD, _ERR
    if not os.path.exists(so_path()):
        from .. import _build

        _build.build(jobs=jobs)
        _MOD, _ERR = None, None
    return require()


def gpu_backend_default() -> str:
    """'hip' when a GPU is visible (extension mandatory), else 'torch'."""
    return "hip" if torch.cuda.is_available() else "torch"


def upload_graph(g) -> None:
    """hipGraphUpload a captured torch CUDAGraph (its one-time upload then
    happens here, not inside the first -- possibly timed -- replay)."""
    exec_ptr = int(g.raw_cuda_graph_exec())
    if exec_ptr:
        require().graph_upload(exec_ptr)
