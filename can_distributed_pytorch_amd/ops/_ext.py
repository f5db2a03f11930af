"""Loader of the in-tree native extension (``_C``, built by build_native.py).

No silent fallback: on a machine with a GPU, a missing or stale extension is
an error (``require()`` raises), so GPU tests can never pass on an eager
PyTorch path by accident.
"""
from __future__ import annotations

import importlib
import os

import torch  # noqa: F401  — must be loaded first: _C resolves libamdhip64/librccl to torch's copies

_mod = None
_err = None


def load(build_if_missing: bool = False):
    global _mod, _err
    if _mod is not None:
        return _mod
    name = "_C_asan" if os.environ.get("CANNET_ASAN", "0") == "1" else "_C"   # host-ASan build (build_native --asan)
    try:
        _mod = importlib.import_module("can_distributed_pytorch_amd." + name)
    except ImportError as e:  # pragma: no cover - depends on build state
        _err = e
        if build_if_missing or os.environ.get("CANNET_AUTOBUILD", "0") == "1":
            from .. import build_native
            build_native.build()
            _mod = importlib.import_module("can_distributed_pytorch_amd._C")
            _err = None
    return _mod


def available() -> bool:
    return load() is not None


def require():
    m = load()
    if m is None:
        raise RuntimeError(
            "can_distributed_pytorch_amd native extension (_C) is not built: run "
            "`python -m can_distributed_pytorch_amd.build_native` (hipcc --offload-arch=gfx950). "
            f"Import error: {_err}")
    return m


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream
