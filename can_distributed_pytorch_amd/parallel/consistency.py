"""Replica-consistency and failure checks for data-parallel training.

The reference relies on DDP and has no desync detection.  Here:
  * ``replica_fingerprint`` — two fp64 reductions of the flat parameter arena
    (sum and an index-weighted sum); ``check_replicas_consistent`` all-reduces
    MIN and MAX of the fingerprint and raises if any rank differs: catches a
    missed/duplicated gradient bucket, a non-deterministic kernel or a stale
    weight pack diverging across ranks;
  * ``check_comm_health`` — surfaces RCCL asynchronous errors of the native
    communicator (instead of hanging at the next collective).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def replica_fingerprint(flat: torch.Tensor) -> torch.Tensor:
    x = flat.detach().double()
    idx = torch.arange(1, x.numel() + 1, device=x.device, dtype=torch.float64)
    return torch.stack([x.sum(), (x * (idx % 9973)).sum()])


def check_replicas_consistent(flat: torch.Tensor, rtol: float = 0.0) -> bool:
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() < 2:
        return True
    fp = replica_fingerprint(flat)
    lo, hi = fp.clone(), fp.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    ok = bool(torch.all((hi - lo).abs() <= rtol * hi.abs()))
    if not ok:
        raise RuntimeError(f"replica desync detected: fingerprint min {lo.tolist()} max {hi.tolist()}")
    return ok


def check_comm_health(reducer) -> None:
    comm = getattr(reducer, "comm", None)
    if comm is not None and hasattr(comm, "async_error"):
        err = comm.async_error()
        if err:
            raise RuntimeError(f"RCCL asynchronous error: {err}")
