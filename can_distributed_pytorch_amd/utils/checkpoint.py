"""Checkpoints.

* ``save_checkpoint(model, path)`` writes a plain CANNet state_dict (the
  reference's test.py layout, no ``module.`` prefix — SURVEY Appendix A Q1);
  ``load_checkpoint`` accepts both layouts and reports missing/unexpected keys
  (the reference's strict=False load of its own DDP checkpoint silently loads
  nothing).  Loading uses ``weights_only=True``: nothing in the file executes.
* ``save_train_state`` / ``load_train_state``: exact resume (weights, SGD
  momentum — native arena or torch optimizer state —, epoch, min_mae,
  min_epoch, the native stepper's loss scale / lr / step count, and the
  torch CPU+CUDA, numpy and Python RNG streams) — the reference has none.
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


def _rng_state() -> dict:
    """Every host/device RNG stream as weights_only-loadable values (tensors, ints, floats, lists)."""
    kind, keys, pos, has_gauss, cached = np.random.get_state()
    ver, py_state, gauss_next = random.getstate()
    st = {
        "torch_cpu": torch.get_rng_state(),
        "numpy": {"kind": str(kind), "keys": torch.from_numpy(np.asarray(keys, dtype=np.int64)), "pos": int(pos),
                  "has_gauss": int(has_gauss), "cached_gaussian": float(cached)},
        "python": {"version": int(ver), "state": torch.tensor(py_state, dtype=torch.int64),
                   "gauss_next": None if gauss_next is None else float(gauss_next)},
    }
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        st["torch_cuda"] = torch.cuda.get_rng_state_all()
    return st


def _set_rng_state(st: dict) -> None:
    torch.set_rng_state(st["torch_cpu"])
    n = st["numpy"]
    np.random.set_state((n["kind"], n["keys"].numpy().astype(np.uint32), n["pos"], n["has_gauss"],
                         n["cached_gaussian"]))
    p = st["python"]
    random.setstate((p["version"], tuple(int(v) for v in p["state"].tolist()), p["gauss_next"]))
    if "torch_cuda" in st and torch.cuda.is_available():
        torch.cuda.set_rng_state_all(st["torch_cuda"])


def save_train_state(path: str, model, momentum: Optional[torch.Tensor], epoch: int, min_mae: float,
                     extra: Optional[dict] = None, optimizer=None, min_epoch: int = 0,
                     stepper_state: Optional[dict] = None) -> None:
    """Everything an uninterrupted run carries into the next epoch: weights, the momentum (native arena, or
    the torch optimizer's state_dict), epoch / min_mae / min_epoch, the native stepper's device state (fp16 loss
    scale, lr, step count) and every RNG stream.  The data order needs no state: DistributedSampler is a
    function of (seed, epoch) and the flip of CrowdDataset one of (seed, epoch, index)."""
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    state = {
        "model": {k: v.detach().cpu() for k, v in _unwrap(model).state_dict().items()},
        "momentum": None if momentum is None else momentum.detach().cpu(),
        "optimizer": None if optimizer is None else optimizer.state_dict(),
        "stepper": None if stepper_state is None else {k: (v.detach().cpu() if torch.is_tensor(v) else v)
                                                       for k, v in stepper_state.items()},
        "epoch": int(epoch),
        "min_mae": float(min_mae),
        "min_epoch": int(min_epoch),
        "rng": _rng_state(),
    }
    if extra:
        state["extra"] = extra
    tmp = path + ".tmp"
    torch.save(state, tmp)
    os.replace(tmp, path)


def load_train_state(path: str, model, momentum: Optional[torch.Tensor] = None, optimizer=None,
                     restore_rng: bool = True) -> dict:
    """Restores what save_train_state wrote (weights_only load: nothing in the file executes).  Returns
    {"epoch", "min_mae", "min_epoch", "stepper"}."""
    st = torch.load(path, map_location="cpu", weights_only=True)
    load_checkpoint_dict(model, st["model"])
    if momentum is not None and st.get("momentum") is not None:
        momentum.copy_(st["momentum"].to(momentum.device))
    if optimizer is not None and st.get("optimizer") is not None:
        optimizer.load_state_dict(st["optimizer"])
    if restore_rng and st.get("rng") is not None:
        _set_rng_state(st["rng"])
    return {"epoch": int(st["epoch"]), "min_mae": float(st["min_mae"]), "min_epoch": int(st.get("min_epoch", 0)),
            "stepper": st.get("stepper")}


def load_checkpoint_dict(model, sd, strict: bool = True):
    sd = strip_module_prefix(sd)
    with torch.no_grad():
        return _unwrap(model).load_state_dict(sd, strict=strict)
