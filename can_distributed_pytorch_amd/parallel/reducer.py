"""Bucketed gradient reducer (this framework's DistributedDataParallel).

Reference: torch DDP as used at train.py:121-122 (1 MiB first
bucket, 25 MiB buckets, built in gradient-ready order, all-reduce overlapped
with backward, averaged by world size).  Re-designed for MI355X:

* the fp32 gradient arena (utils/flat.py) is laid out in gradient-READY
  order, so each bucket is one contiguous slice and the all-reduce runs in
  place — no copy-in / copy-out;
* ``mark_ready(param_indices)`` is called by the native executor right after
  a layer's weight-gradient kernel (or by post-accumulate-grad hooks on the
  autograd path); when a bucket is complete it is launched — strictly in
  bucket order so that every rank issues identical collective sequences;
* transport "rccl": the C++ BucketReducer (csrc/rccl_reducer.cpp) — own
  RCCL communicator, comm stream at high priority, one hipEvent per bucket,
  graph-capturable;  transport "torch": torch.distributed (gloo on CPU for the
  fake-cluster tests, or NCCL) with async work handles;
* averaging (1/world) is folded into the fused SGD kernel, not done here.
"""
from __future__ import annotations

import time
from dataclasses import dataclass
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist

from ..utils.flat import FlatArena

MIB = 1 << 20


@dataclass
class Bucket:
    start: int          # element offset into the arena
    end: int
    params: List[int]   # parameter indices (model.parameters() order)

    @property
    def numel(self):
        return self.end - self.start


def plan_buckets(arena: FlatArena, ready_order: Sequence[int], bucket_mb: float = 25.0,
                 first_bucket_mb: float = 1.0, last_bucket_mb: Optional[float] = 1.0) -> List[Bucket]:
    """Greedy bucketing over the arena in ready order (arena must follow that order).

    Like DDP: a small first bucket (its all-reduce starts early) and ``bucket_mb`` caps.  Unlike DDP the
    TAIL is split too: the trailing parameters (conv1_2 / conv1_1, whose weight gradients finish last)
    form their own bucket of at most ``last_bucket_mb``, so the ~11 MiB of frontend gradients before them
    are all-reduced while those last weight gradients still run, and only a ~150 KiB all-reduce is
    exposed after the backward (None: DDP's greedy tail)."""
    slots = [arena.slot(i) for i in ready_order]
    for (s0, e0), (s1, _) in zip(slots, slots[1:]):
        if s1 != e0:
            raise ValueError("arena is not laid out in gradient-ready order")
    buckets: List[Bucket] = []
    cur: List[int] = []
    cur_start = None
    cap = first_bucket_mb * MIB
    for i, (s, e) in zip(ready_order, slots):
        if cur_start is None:
            cur_start = s
        cur.append(i)
        if (e - cur_start) * 4 >= cap:
            buckets.append(Bucket(cur_start, e, cur))
            cur, cur_start = [], None
            cap = bucket_mb * MIB
    if cur:
        buckets.append(Bucket(cur_start, slots[-1][1], cur))
    last = buckets[-1]
    if last_bucket_mb is not None and len(last.params) > 1 and last.numel * 4 > last_bucket_mb * MIB:
        k = len(last.params) - 1            # first index of the tail: at least one parameter
        while k > 1:
            s0 = arena.slot(last.params[k - 1])[0]
            if (last.end - s0) * 4 > last_bucket_mb * MIB:
                break
            k -= 1
        split = arena.slot(last.params[k])[0]
        buckets[-1] = Bucket(last.start, split, last.params[:k])
        buckets.append(Bucket(split, last.end, last.params[k:]))
    return buckets


class BucketedReducer:
    def __init__(self, arena: FlatArena, ready_order: Sequence[int], bucket_mb: float = 25.0,
                 first_bucket_mb: float = 1.0, transport: str = "auto", group=None, comm=None,
                 last_bucket_mb: Optional[float] = 1.0):
        self.arena = arena
        self.buckets = plan_buckets(arena, ready_order, bucket_mb, first_bucket_mb, last_bucket_mb)
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        dev = arena.grad.device
        if transport == "auto":
            transport = "rccl" if dev.type == "cuda" else "torch"
        self.transport = transport
        self.param_bucket = [-1] * len(arena.params)
        for b, bk in enumerate(self.buckets):
            for i in bk.params:
                self.param_bucket[i] = b
        self._native = None
        self.comm = None
        if transport == "rccl":
            from ..ops import _ext
            C = _ext.require()
            self.comm = comm or self._make_comm_agreed(dev, group)
            if self.comm is None:
                self.transport = transport = "torch"      # every rank falls back together (see below)
            else:
                self._native = C.BucketReducer(self.comm, arena.grad.data_ptr(),
                                               [b.start for b in self.buckets], [b.numel for b in self.buckets],
                                               self.param_bucket, 1)
        self._pending = None
        self._next = 0
        self._works = []
        self._timing = False
        self._host_t = None          # torch transport timing: host clock per launched bucket

    def _make_comm_agreed(self, dev, group):
        """This rank's RCCL communicator, or None on EVERY rank if any rank failed to create one.  Every step
        that can fail is bounded and followed by a step every rank reaches, so a failure on one rank cannot strand
        the others in a blocking call:
          1. rank 0 broadcasts (ok, unique id | error) — a failed ncclGetUniqueId is seen by every rank;
          2. the communicator is initialised NON-blocking with a deadline (csrc/rccl_reducer.cpp: RcclComm), so
             ranks whose peer died before or inside its init time out and return instead of waiting forever;
          3. one all-reduce of a failure flag on the torch process group: if any rank failed, every rank aborts
             its communicator and the reducer runs its buckets through torch.distributed (the same RCCL
             underneath, without the owned communicator) instead of training with mismatched transports."""
        comm, err = None, None
        try:
            comm = make_rccl_comm(dev, group)
        except Exception as e:                    # any failure, not only RCCL's RuntimeError
            err = e
        if self.world > 1:
            ok = torch.tensor([0.0 if err is None else 1.0], device=dev)
            dist.all_reduce(ok, group=group)
            failed = ok.item() > 0
        else:
            failed = err is not None
        if failed:
            if comm is not None:
                comm.abort()
            import warnings
            warnings.warn(f"owned RCCL communicator unavailable ({err or 'failed on another rank'}); "
                          "gradient buckets go through torch.distributed")
            return None
        return comm

    # --------------------------------------------------------------- step API
    def begin(self):
        if self._native is not None:
            from ..ops import _ext
            self._native.begin(_ext.stream_ptr(self.arena.grad.device))
            return
        self._pending = [len(b.params) for b in self.buckets]
        self._next = 0
        self._works = []
        if self._timing:
            self._host_t = {"t0": time.perf_counter(), "launch": {}, "end": {}, "bwd": None}

    # ------------------------------------------------------------- diagnostics
    def set_timing(self, on: bool):
        """Per-bucket all-reduce timing for the next steps (diagnostics; not inside a captured step).
        rccl: hipEvents on the producer / comm streams; torch: host clock around the async works."""
        self._timing = bool(on)
        if self._native is not None:
            self._native.set_timing(self._timing)

    def timings(self) -> Optional[dict]:
        """The last timed step: per bucket {bucket, mib, ready_ms, start_ms, end_ms} (ms after begin(); ready =
        its last gradient written, start / end = its all-reduce) and ``backward_end_ms`` (every gradient written);
        ``exposed_ms`` = how long the last all-reduce ran past the backward (the part not hidden by compute)."""
        if self._native is not None:
            rows, bwd = self._native.timings()
            if bwd < 0:
                return None
            bk = [dict(bucket=b, mib=round(self.buckets[b].numel * 4 / MIB, 3), ready_ms=round(r, 4),
                       start_ms=round(s0, 4), end_ms=round(e, 4)) for b, r, s0, e in rows]
        else:
            ht = self._host_t
            if not ht or ht["bwd"] is None:
                return None
            t0 = ht["t0"]
            bk = [dict(bucket=b, mib=round(self.buckets[b].numel * 4 / MIB, 3),
                       ready_ms=round(1e3 * (ht["launch"][b] - t0), 4), start_ms=round(1e3 * (ht["launch"][b] - t0), 4),
                       end_ms=round(1e3 * (ht["end"].get(b, ht["launch"][b]) - t0), 4)) for b in sorted(ht["launch"])]
            bwd = 1e3 * (ht["bwd"] - t0)
        last_end = max((r["end_ms"] for r in bk), default=bwd)
        return {"buckets": bk, "backward_end_ms": round(bwd, 4), "exposed_ms": round(max(0.0, last_end - bwd), 4)}

    def mark_ready(self, params: Sequence[int]):
        if self._native is not None:
            from ..ops import _ext
            self._native.mark_ready(list(params), _ext.stream_ptr(self.arena.grad.device))
            return
        for p in params:
            b = self.param_bucket[p]
            if b < 0:
                continue
            self._pending[b] -= 1
            if self._pending[b] < 0:
                raise RuntimeError(f"parameter {p} marked ready twice in one step")
        while self._next < len(self.buckets) and self._pending[self._next] == 0:
            self._launch(self._next)
            self._next += 1

    def _launch(self, b: int):
        if self._timing and self._host_t is not None:
            self._host_t["launch"][b] = time.perf_counter()
        if self.world < 2:                        # a 1-rank all-reduce is the identity
            return
        bk = self.buckets[b]
        view = self.arena.grad[bk.start:bk.end]
        self._works.append((b, dist.all_reduce(view, group=self.group, async_op=True)))

    def finish(self):
        if self._native is not None:
            from ..ops import _ext
            self._native.finish(_ext.stream_ptr(self.arena.grad.device))
            return
        if self._timing and self._host_t is not None:
            self._host_t["bwd"] = time.perf_counter()
        while self._next < len(self.buckets):
            self._launch(self._next)
            self._next += 1
        for b, w in self._works:
            w.wait()
            if self._timing and self._host_t is not None:
                self._host_t["end"][b] = time.perf_counter()
        self._works = []

    def allreduce_scalars(self, t: torch.Tensor):
        """In-place SUM of a small device vector (loss, non-finite flag) on the compute stream."""
        if self.world < 2:
            return t
        if self._native is not None:
            from ..ops import _ext
            self.comm.allreduce(t.data_ptr(), t.numel(), 0, 0, _ext.stream_ptr(t.device))
        else:
            dist.all_reduce(t, group=self.group)
        return t

    def broadcast_arena(self, src: int = 0):
        """One collective for the whole parameter arena (DDP ctor broadcast, train.py:98-122)."""
        if self.world < 2:
            return
        if self._native is not None:
            from ..ops import _ext
            self.comm.broadcast(self.arena.data.data_ptr(), self.arena.numel, 0, src,
                                _ext.stream_ptr(self.arena.data.device))
        else:
            dist.broadcast(self.arena.data, src=src, group=self.group)

    # ------------------------------------------------------- autograd hooks
    def attach_hooks(self):
        """Generic autograd path: post-accumulate-grad hooks -> mark_ready (like DDP's reducer hooks)."""
        handles = []
        for i, p in enumerate(self.arena.params):
            def hook(_p, i=i):
                self.mark_ready([i])
            handles.append(p.register_post_accumulate_grad_hook(hook))
        return handles


def make_rccl_comm(device, group=None, init_timeout_s: Optional[float] = None):
    """Create this process's RCCL communicator; the 128-byte unique id travels through the existing torch process
    group (one broadcast_object_list) together with rank 0's ok flag, so a rank-0 failure to make the id raises on
    every rank.  The init itself is bounded by ``init_timeout_s`` (env CANNET_RCCL_INIT_TIMEOUT, default 300 s)."""
    import os
    from ..ops import _ext
    C = _ext.require()
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if init_timeout_s is None:
        init_timeout_s = float(os.environ.get("CANNET_RCCL_INIT_TIMEOUT", "300"))
    msg = None
    if rank == 0:
        try:
            msg = (True, C.rccl_unique_id())
        except Exception as e:
            msg = (False, f"rank 0: ncclGetUniqueId failed: {e}")
    obj = [msg]
    if world > 1:
        dist.broadcast_object_list(obj, src=0, group=group)
    ok, payload = obj[0]
    if not ok:
        raise RuntimeError(payload)
    dev = torch.device(device)
    return C.RcclComm(rank, world, payload, dev.index if dev.index is not None else 0, float(init_timeout_s))
