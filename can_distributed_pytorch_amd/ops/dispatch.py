"""Kernel / schedule dispatch configuration: ONE validated config, read once.

The production step is fully determined by the defaults below.  The only way to change it is the single opt-in
string ``CANNET_DISPATCH="key=value,key=value"`` (parsed and validated once per process: an unknown key or an
out-of-range value is an error, never silently ignored) or, in tests and A/B scripts, ``override(**kw)``.  No other
environment variable is read on the launch path, so a stray variable cannot change the default training step.

Native fields are pushed into the extension (csrc/dispatch.h, ``set_dispatch``); the others are read by the executor
(ops/executor.py) and the conv front-end (ops/conv.py) from ``current()``.
"""
from __future__ import annotations

import contextlib
import dataclasses
import os
from typing import Dict, Iterator

ENV = "CANNET_DISPATCH"


@dataclasses.dataclass(frozen=True)
class DispatchConfig:
    # ---- native (csrc/dispatch.h)
    rring: int = 2            # row-ring 3x3 kernels: 0 off, 1 dilation-1 layers, 2 every dilation
    rring64: int = 1          # cfg 28: 64-channel 4-row row-ring tiles
    rring128: int = 1         # cfg 29: 0 off, 1 K > 1152 dil 1, 2 + K <= 1152, 3 + dilation 2
    ws64: int = 1             # weight-stationary Cin = Cout = 64 kernel (0: halo kernel)
    ctx_tile_f: int = 256     # linearised context GEMM tiles (256 / 128)
    ctx_tile_b: int = 256
    wgrad_halo_ring: int = 1  # full-resolution weight gradient: row-ring kernel (0: 2-row halo tiles)
    ring_fast: int = 1        # row-ring weight gradient: fast in-image addressing where the shape allows
    ring_skew: int = 1        # row-ring weight gradient: skewed DMA issue
    reduce_tiled: int = 1     # slab reduction: tiled kernel where it applies
    wgrad_tap: int = 3        # tap-ring weight gradient (cfg 12): 0 off, 1 v2-GEMM layers, 2 + Cout-128 ring layers,
    #                           3 + Cout-64 layers
    wgrad_tap_adb: int = 1    # tap ring: double-buffered dY fragments
    first_pf: int = 1        # conv1_1: persistent, next tile's halo loaded under the current stores
    rring_pool: int = 1       # conv + 2x2 max-pool on the row ring (Cout % 256 layers)
    # ---- executor / front-end (Python)
    w1g: int = 1              # conv1_1's weight gradient fused into conv1_2's data gradient
    pool_fwd_fused: int = 1   # 2x2 max-pool in the conv epilogue
    poolbwd_fused: int = 1    # max-pool backward in the data-gradient epilogue
    ctx_linear: int = 1       # context module as one GEMM each way (0: direct per-scale form)
    ctx_batched: int = 1      # direct form: the four conv{S}_2 convs in one launch
    bias_fused: int = 1       # bias gradients from the data-gradient epilogue partials
    wgrad_stream: int = 1     # weight gradients on a second stream
    ctx_wgrad_cus: int = 224  # CUs the batched context 1x1 weight gradient is planned for

    NATIVE = ("rring", "rring64", "rring128", "ws64", "ctx_tile_f", "ctx_tile_b", "wgrad_halo_ring", "ring_fast",
              "ring_skew", "reduce_tiled", "wgrad_tap", "wgrad_tap_adb", "rring_pool", "first_pf")

    def native(self) -> Dict[str, int]:
        return {k: getattr(self, k) for k in self.NATIVE}


_ALLOWED = {
    "rring": (0, 1, 2), "rring64": (0, 1), "rring128": (0, 1, 2, 3), "ws64": (0, 1), "ctx_tile_f": (128, 256),
    "ctx_tile_b": (128, 256), "wgrad_halo_ring": (0, 1), "ring_fast": (0, 1), "ring_skew": (0, 1),
    "reduce_tiled": (0, 1), "wgrad_tap": (0, 1, 2, 3), "wgrad_tap_adb": (0, 1), "rring_pool": (0, 1), "first_pf": (0, 1),
    "w1g": (0, 1), "pool_fwd_fused": (0, 1), "poolbwd_fused": (0, 1), "ctx_linear": (0, 1),
    "ctx_batched": (0, 1), "bias_fused": (0, 1), "wgrad_stream": (0, 1),
}


def validate(cfg: DispatchConfig) -> DispatchConfig:
    for f in dataclasses.fields(DispatchConfig):
        v = getattr(cfg, f.name)
        if not isinstance(v, int) or isinstance(v, bool):
            raise ValueError(f"dispatch {f.name}={v!r}: integer expected")
        allowed = _ALLOWED.get(f.name)
        if allowed is not None and v not in allowed:
            raise ValueError(f"dispatch {f.name}={v}: allowed {allowed}")
    if not 1 <= cfg.ctx_wgrad_cus <= 4096:
        raise ValueError(f"dispatch ctx_wgrad_cus={cfg.ctx_wgrad_cus}: 1..4096")
    return cfg


def parse(text: str) -> DispatchConfig:
    """``"key=value,key=value"`` -> a validated config (unknown keys are errors)."""
    names = {f.name for f in dataclasses.fields(DispatchConfig)}
    kw = {}
    for item in (text or "").replace(";", ",").split(","):
        item = item.strip()
        if not item:
            continue
        if "=" not in item:
            raise ValueError(f"{ENV}: {item!r} is not key=value")
        k, v = (t.strip() for t in item.split("=", 1))
        if k not in names:
            raise ValueError(f"{ENV}: unknown key {k!r} (known: {sorted(names)})")
        kw[k] = int(v)
    return validate(DispatchConfig(**kw))


_current = None


def current() -> DispatchConfig:
    """The process's dispatch config ($CANNET_DISPATCH parsed and validated on first use)."""
    global _current
    if _current is None:
        _current = parse(os.environ.get(ENV, ""))
    return _current


def apply(cfg: DispatchConfig) -> None:
    """Make ``cfg`` the process's config and push its native fields into the extension (if it is loaded)."""
    global _current
    _current = validate(cfg)
    from . import _ext
    m = _ext.load()
    if m is not None and hasattr(m, "set_dispatch"):
        m.set_dispatch(cfg.native())


@contextlib.contextmanager
def override(**kw) -> Iterator[DispatchConfig]:
    """Temporarily switch dispatch fields (tests / A/B scripts): ``with dispatch.override(rring=0): ...``."""
    prev = current()
    cfg = validate(dataclasses.replace(prev, **kw))
    apply(cfg)
    try:
        yield cfg
    finally:
        apply(prev)
