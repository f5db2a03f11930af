"""Checkpoints.

* ``save_checkpoint(model, path)`` writes a plain CANNet state_dict (the
  reference's test.py layout, no ``module.`` prefix — SURVEY Appendix A Q1);
  ``load_checkpoint`` accepts both layouts and reports missing/unexpected keys
  (the reference's strict=False load of its own DDP checkpoint silently loads
  nothing).  Loading uses ``weights_only=True``: nothing in the file executes.
* ``save_train_state`` / ``load_train_state``: full resume (weights, SGD
  momentum arena, epoch, min_mae, RNG states) — the reference has no resume.
"""
from __future__ import annotations

import os
import random
from typing import Optional

import numpy as np
import torch

from ..models.cannet import strip_module_prefix


def _unwrap(model):
    return model.module if hasattr(model, "module") else model


def save_checkpoint(model, path: str) -> None:
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    sd = {k: v.detach().cpu().contiguous() for k, v in _unwrap(model).state_dict().items()}
    tmp = path + ".tmp"
    torch.save(sd, tmp)
    os.replace(tmp, path)


def load_checkpoint(model, path: str, strict: bool = True, map_location="cpu"):
    sd = torch.load(path, map_location=map_location, weights_only=True)
    if isinstance(sd, dict) and "model" in sd and isinstance(sd["model"], dict):
        sd = sd["model"]
    sd = strip_module_prefix(sd)
    m = _unwrap(model)
    with torch.no_grad():
        res = m.load_state_dict(sd, strict=strict)
    return res


def save_train_state(path: str, model, momentum: Optional[torch.Tensor], epoch: int, min_mae: float,
                     extra: Optional[dict] = None) -> None:
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    state = {
        "model": {k: v.detach().cpu() for k, v in _unwrap(model).state_dict().items()},
        "momentum": None if momentum is None else momentum.detach().cpu(),
        "epoch": int(epoch),
        "min_mae": float(min_mae),
        "torch_rng": torch.get_rng_state(),
        "numpy_rng": torch.from_numpy(np.frombuffer(np.random.bytes(8), dtype=np.uint8).copy()),
        "py_rng_seed": random.getrandbits(63),
    }
    if extra:
        state["extra"] = extra
    tmp = path + ".tmp"
    torch.save(state, tmp)
    os.replace(tmp, path)


def load_train_state(path: str, model, momentum: Optional[torch.Tensor] = None):
    st = torch.load(path, map_location="cpu", weights_only=True)
    load_checkpoint_dict(model, st["model"])
    if momentum is not None and st.get("momentum") is not None:
        momentum.copy_(st["momentum"].to(momentum.device))
    torch.set_rng_state(st["torch_rng"])
    random.seed(int(st["py_rng_seed"]))
    return int(st["epoch"]), float(st["min_mae"])


def load_checkpoint_dict(model, sd, strict: bool = True):
    sd = strip_module_prefix(sd)
    with torch.no_grad():
        return _unwrap(model).load_state_dict(sd, strict=strict)
