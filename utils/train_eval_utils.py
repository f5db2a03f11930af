"""Compatibility module for ``from utils.train_eval_utils import train_one_epoch, evaluate``."""
from can_distributed_pytorch_amd.engine.train_eval import train_one_epoch, evaluate  # noqa: F401

__all__ = ["train_one_epoch", "evaluate"]
