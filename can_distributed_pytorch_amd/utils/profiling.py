"""Tracing: roctx ranges + a device-timed step profiler.

The reference has no tracing at all.  Here:
  * ``trace_range(name)`` emits a roctx range (visible in rocprofv3
    ``--marker-trace`` timelines) around forward / backward / all-reduce /
    optimizer phases when ``CANNET_ROCTX=1``; otherwise it is free;
  * ``CudaEventTimer`` measures device time of code regions with hipEvents
    (no host sync until ``summary()``).
Kernel-level analysis uses rocprofv3 directly (scripts/gpu/*.sh, profiles/).
"""
from __future__ import annotations

import contextlib
import ctypes
import glob
import os

import torch

_roctx = None
_enabled = os.environ.get("CANNET_ROCTX", "0") == "1"


def _load_roctx():
    global _roctx
    if _roctx is not None:
        return _roctx
    cands = glob.glob(os.path.join(os.path.dirname(torch.__file__), "lib", "libroctx64.so*")) + \
        ["libroctx64.so", "/opt/rocm/lib/libroctx64.so"]
    for c in cands:
        try:
            lib = ctypes.CDLL(c)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxMarkA.argtypes = [ctypes.c_char_p]
            _roctx = lib
            return lib
        except OSError:
            continue
    _roctx = False
    return _roctx


def enable(flag: bool = True):
    global _enabled
    _enabled = flag


@contextlib.contextmanager
def trace_range(name: str):
    lib = _load_roctx() if _enabled else None
    if lib:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib:
            lib.roctxRangePop()


def mark(name: str):
    lib = _load_roctx() if _enabled else None
    if lib:
        lib.roctxMarkA(name.encode())
