"""Experiment logging: JSONL metrics (rank 0), optional wandb (lazy; not installed here).

Reference: wandb.init/log (train.py:40-46,167-171), tqdm bars and prints
(utils/train_eval_utils.py:25-26,44-46).  Here every record is one JSON line
(loss, mae, lr, img/s, step time, ...), and wandb is used only if importable.
"""
from __future__ import annotations

import json
import os
import time
from typing import Optional


class JsonlLogger:
    def __init__(self, path: Optional[str], enabled: bool = True):
        self.path = path
        self.enabled = enabled and path is not None
        if self.enabled:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)

    def log(self, **kv):
        if not self.enabled:
            return
        kv.setdefault("ts", time.time())
        with open(self.path, "a") as f:
            f.write(json.dumps(kv, default=float) + "\n")


_wandb = None


def wandb_init(enabled: bool, **kw) -> bool:
    global _wandb
    if not enabled:
        return False
    try:
        import wandb  # noqa: F401
    except Exception:
        print("[wandb not installed: metrics go to the JSONL log only]")
        return False
    import wandb
    _wandb = wandb
    wandb.init(**kw)
    return True


def wandb_log(**kv):
    if _wandb is not None:
        _wandb.log(kv)


def wandb_log_images(paths, epoch):
    if _wandb is not None:
        _wandb.log({"examples": [_wandb.Image(p, caption=f"{os.path.basename(p)} {epoch}") for p in paths]})


class StepTimer:
    """Wall-clock img/s over a window (host side; call after a device sync point)."""

    def __init__(self):
        self.t0 = time.perf_counter()
        self.n = 0

    def add(self, n_imgs: int):
        self.n += n_imgs

    def rate(self) -> float:
        return self.n / max(time.perf_counter() - self.t0, 1e-9)
