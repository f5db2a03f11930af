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


_checked = False


def check_source_hash(m) -> None:
    """Refuse a binary that was not built from the csrc/ sources in this tree (a stale or foreign _C)."""
    from .. import build_native
    files = build_native.source_files()
    if not files:                      # installed without sources: nothing to compare against
        return
    want = build_native.source_hash(files)
    got = m.src_hash()
    if got != want:
        raise RuntimeError(
            f"stale native extension: {m.__file__} was built from csrc/ sources with sha256 {got[:16]}..., the tree's "
            f"sources hash to {want[:16]}...; rebuild with `python -m can_distributed_pytorch_amd.build_native`")


def require():
    global _checked
    m = load()
    if m is None:
        raise RuntimeError(
            "can_distributed_pytorch_amd native extension (_C) is not built: run "
            "`python -m can_distributed_pytorch_amd.build_native` (hipcc --offload-arch=gfx950). "
            f"Import error: {_err}")
    if not _checked:
        check_source_hash(m)
        from . import dispatch
        dispatch.apply(dispatch.current())    # the validated $CANNET_DISPATCH config, pushed once
        _checked = True
    return m


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream
