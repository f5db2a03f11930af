"""Process-group bootstrap and rank helpers.

Parity: utils/distributed_utils.py:7-70 of the reference (init_distributed_mode,
cleanup, is_dist_avail_and_initialized, get_world_size, get_rank,
is_main_process, reduce_value).

Differences by design:
  * Q4: with no launcher env the world-size-1 path works without a process
    group (the reference crashes at its first barrier).
  * Q5: the SLURM branch reads SLURM_NTASKS / SLURM_LOCALID.
  * One process per GPU; backend "nccl" is RCCL on ROCm (xGMI intra-node).
    On CPU (tests, fake clusters) the backend is gloo.
  * The native RCCL communicator (csrc/rccl_reducer.cpp) gets its
    ncclUniqueId through this process group (parallel/reducer.py:
    make_rccl_comm, one broadcast_object_list).
"""
from __future__ import annotations

import datetime
import os
from typing import Optional

import torch
import torch.distributed as dist


def init_distributed_mode(args) -> None:
    """Fill args.{rank, world_size, gpu, distributed} and init the process group."""
    env = os.environ
    if "RANK" in env and "WORLD_SIZE" in env:
        args.rank = int(env["RANK"])
        args.world_size = int(env["WORLD_SIZE"])
        args.gpu = int(env.get("LOCAL_RANK", 0))
    elif "SLURM_PROCID" in env:
        args.rank = int(env["SLURM_PROCID"])
        args.world_size = int(env.get("SLURM_NTASKS", getattr(args, "world_size", 1)))
        ndev = max(torch.cuda.device_count(), 1)
        args.gpu = int(env.get("SLURM_LOCALID", args.rank % ndev))
    else:
        args.rank, args.world_size, args.gpu = 0, 1, 0
        args.distributed = False
        return

    args.distributed = args.world_size > 1 or dist.is_available()
    use_gpu = str(getattr(args, "device", "cuda")).startswith("cuda") and torch.cuda.is_available()
    if use_gpu:
        torch.cuda.set_device(args.gpu)
    args.dist_backend = "nccl" if use_gpu else "gloo"
    url = getattr(args, "dist_url", "env://")
    timeout = datetime.timedelta(seconds=int(env.get("CANNET_PG_TIMEOUT", "1800")))
    kwargs = dict(backend=args.dist_backend, init_method=url, world_size=args.world_size,
                  rank=args.rank, timeout=timeout)
    if use_gpu:
        kwargs["device_id"] = torch.device("cuda", args.gpu)
    if not dist.is_initialized():
        dist.init_process_group(**kwargs)
    if args.rank == 0:
        print(f"| distributed init: world {args.world_size} backend {args.dist_backend} url {url}", flush=True)
    barrier()


def cleanup() -> None:
    if is_dist_avail_and_initialized():
        dist.destroy_process_group()


def is_dist_avail_and_initialized() -> bool:
    return dist.is_available() and dist.is_initialized()


def get_world_size() -> int:
    return dist.get_world_size() if is_dist_avail_and_initialized() else 1


def get_rank() -> int:
    return dist.get_rank() if is_dist_avail_and_initialized() else 0


def is_main_process() -> bool:
    return get_rank() == 0


def barrier() -> None:
    if is_dist_avail_and_initialized():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def reduce_value(value: torch.Tensor, average: bool = True) -> torch.Tensor:
    """In-place SUM all-reduce of a (scalar) tensor, optionally /world.  (utils/distributed_utils.py:60-70)"""
    world = get_world_size()
    if world < 2:
        return value
    with torch.no_grad():
        dist.all_reduce(value)
        if average:
            value /= world
    return value


def reduce_scalars(*values: torch.Tensor, average: bool = True) -> torch.Tensor:
    """Fuse several device scalars (loss, mae, non-finite flag, ...) into ONE all-reduce.

    The reference issues one 4-byte all-reduce per scalar;
    here they travel together.  Returns the stacked reduced vector.
    """
    vec = torch.stack([v.reshape(()).float() for v in values])
    world = get_world_size()
    if world >= 2:
        dist.all_reduce(vec)
        if average:
            vec /= world
    return vec


def get_store() -> Optional[dist.Store]:
    """The default process group's TCPStore (used to exchange the RCCL unique id)."""
    if not is_dist_avail_and_initialized():
        return None
    try:
        from torch.distributed.distributed_c10d import _get_default_store
        return _get_default_store()
    except Exception:  # pragma: no cover - older torch
        return None
