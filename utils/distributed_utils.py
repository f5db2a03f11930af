"""Compatibility module for ``from utils.distributed_utils import ...`` (reference layout)."""
from can_distributed_pytorch_amd.parallel.distributed import (init_distributed_mode, cleanup,  # noqa: F401
                                                              is_dist_avail_and_initialized, get_world_size, get_rank,
                                                              is_main_process, reduce_value)
import torch.distributed as dist  # noqa: F401

__all__ = ["init_distributed_mode", "cleanup", "is_dist_avail_and_initialized", "get_world_size", "get_rank",
           "is_main_process", "reduce_value", "dist"]
