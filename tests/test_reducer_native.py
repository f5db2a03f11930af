"""CPU tests of the C++ bucket reducer logic (csrc/bucket_schedule.h, csrc/rccl_reducer.cpp).

The GPU reducer (``BucketReducer``: RCCL on a comm stream) and the fake-cluster
reducer used here (``FakeRankReducer``: W host threads + a blocking in-process
SUM collective) share ONE scheduling class, ``BucketSchedule``.  So these
tests exercise, with 2-4 fake ranks and no GPU, exactly the decisions the
RCCL path takes at world 8: launch order, per-bucket counters, the split tail
bucket, and the producer-stream bookkeeping when marks arrive interleaved from
the compute stream (head gradients) and the weight-gradient side stream.
Reference behaviour being re-implemented: DDP's bucketed all-reduce
(train.py:121-122).
"""
import random
from concurrent.futures import ThreadPoolExecutor

import pytest
import torch

from can_distributed_pytorch_amd.models.cannet import CANNet
from can_distributed_pytorch_amd.ops import _ext
from can_distributed_pytorch_amd.ops.executor import CANNetExecutor
from can_distributed_pytorch_amd.parallel.reducer import plan_buckets, MIB
from can_distributed_pytorch_amd.utils.flat import FlatArena

MAIN, SIDE = 0x1000, 0x2000          # stream tags (any distinct 64-bit values)


@pytest.fixture(scope="module")
def C():
    m = _ext.load(build_if_missing=True)
    assert m is not None, "native extension failed to build"
    return m


def _cannet_plan():
    model = CANNet(backend="torch")
    ex = CANNetExecutor(model)
    order = ex.grad_ready_order()
    params = list(model.parameters())
    return ex, order, params


def test_schedule_order_counters_and_errors(C):
    # 6 params, 3 buckets: {0,1} {2,3,4} {5}
    pb = [0, 0, 1, 1, 1, 2]
    s = C.BucketSchedule(pb, 3)
    assert s.mark([2], MAIN) == []                 # bucket 1 not launchable before bucket 0
    assert s.pending(1) == 2
    assert s.mark([3, 4], SIDE) == []
    assert s.mark([1], SIDE) == []
    assert s.mark([0], MAIN) == [0, 1]             # completes 0, then 1 is already complete
    assert sorted(s.streams(0)) == [MAIN, SIDE] and sorted(s.streams(1)) == [MAIN, SIDE]
    with pytest.raises(RuntimeError, match="already launched"):
        s.mark([0], MAIN)
    assert s.finish() == [2]                       # param 5 never marked: reduced anyway
    s.begin()
    s.mark([5], MAIN)
    with pytest.raises(RuntimeError, match="twice"):
        s.mark([5], MAIN)
    with pytest.raises(RuntimeError, match="bad param"):
        s.mark([17], MAIN)


def _rank_marks(ex, order, rng):
    """Host-order marks of one backward: head grads on the compute stream first, every other layer's
    (weight, bias) from the weight-gradient side stream; the two streams' subsequences interleaved at random
    (each stream keeps its own order)."""
    head = [([ex.head_w_index, ex.head_b_index], MAIN)]
    rest = order[2:]
    side = []
    i = 0
    while i < len(rest):
        k = rng.choice([1, 2, 4])                  # the executor marks 1 (bias-less), 2 or 4 (context) params
        side.append((rest[i:i + k], SIDE))
        i += k
    out, a, b = [], list(head), list(side)
    while a or b:
        src = a if (a and (not b or rng.random() < 0.5)) else b
        out.append(src.pop(0))
    return out


@pytest.mark.parametrize("world", [2, 3, 4])
def test_fake_cluster_cannet_buckets(C, world):
    ex, order, params = _cannet_plan()
    arenas = [FlatArena([torch.nn.Parameter(p.detach().clone()) for p in params], "cpu", order=order)
              for _ in range(world)]
    buckets = plan_buckets(arenas[0], order, bucket_mb=25.0, first_bucket_mb=1.0, last_bucket_mb=1.0)
    nb = len(buckets)
    pb = [-1] * len(params)
    for b, bk in enumerate(buckets):
        for i in bk.params:
            pb[i] = b
    # DDP-like plan: small first bucket, 25 MiB caps, and the split tail (the last frontend layers, <= 1 MiB)
    assert buckets[0].numel * 4 <= 2 * MIB
    # (a bucket may overshoot its cap by its last tensor, as in DDP: backend.0.weight alone is 18 MiB)
    biggest = max(p.numel() for p in params) * 4
    assert all(bk.numel * 4 <= 25 * MIB + biggest for bk in buckets)
    tail = buckets[-1]
    assert tail.numel * 4 <= MIB and tail.params == order[-len(tail.params):]
    cl = C.FakeCluster(world, 20.0)
    reds = [C.FakeRankReducer(cl, r, arenas[r].grad.data_ptr(), [b.start for b in buckets],
                              [b.numel for b in buckets], pb) for r in range(world)]

    def run_rank(r, step):
        rng = random.Random(1000 * step + r)
        g = arenas[r].grad
        g.copy_(torch.arange(g.numel(), dtype=torch.float32) % 97 + 1000.0 * r + step)
        reds[r].begin()
        for idx, tag in _rank_marks(ex, order, rng):
            reds[r].mark_ready(idx, tag)
        reds[r].finish()
        return reds[r].log()

    for step in range(2):
        with ThreadPoolExecutor(world) as pool:
            logs = list(pool.map(lambda r: run_rank(r, step), range(world)))
        # identical collective sequence on every rank, strictly in bucket order
        for lg in logs:
            assert [b for b, _ in lg] == list(range(nb))
        # the collective waits on every producer stream of the bucket
        for b, streams in logs[0]:
            expect = {MAIN if i in (ex.head_w_index, ex.head_b_index) else SIDE for i in buckets[b].params}
            assert set(streams) == expect
        # in-place SUM over ranks
        base = torch.arange(arenas[0].grad.numel(), dtype=torch.float32) % 97
        expect = world * (base + step) + 1000.0 * sum(range(world))
        for r in range(world):
            assert torch.equal(arenas[r].grad, expect)
    assert cl.collectives == 2 * nb


def test_fake_cluster_detects_divergent_plans(C):
    """A rank whose bucket plan differs (e.g. another bucket cap) would issue a different collective
    sequence: the fake transport reports the mismatch instead of hanging (what RCCL would do)."""
    ex, order, params = _cannet_plan()
    arena = [FlatArena([torch.nn.Parameter(p.detach().clone()) for p in params], "cpu", order=order)
             for _ in range(2)]
    plans = [plan_buckets(arena[0], order, bucket_mb=25.0), plan_buckets(arena[1], order, bucket_mb=10.0)]
    cl = C.FakeCluster(2, 5.0)
    reds = []
    for r, bks in enumerate(plans):
        pb = [-1] * len(params)
        for b, bk in enumerate(bks):
            for i in bk.params:
                pb[i] = b
        reds.append(C.FakeRankReducer(cl, r, arena[r].grad.data_ptr(), [b.start for b in bks],
                                      [b.numel for b in bks], pb))

    def run(r):
        reds[r].begin()
        for i in order:
            reds[r].mark_ready([i], MAIN)
        reds[r].finish()

    with ThreadPoolExecutor(2) as pool:
        futs = [pool.submit(run, r) for r in range(2)]
        errs = [f.exception() for f in futs]
    assert any(e is not None and ("mismatch" in str(e) or "timed out" in str(e)) for e in errs), errs


def test_rccl_comm_failure_falls_back_to_torch_transport(monkeypatch):
    """If the owned RCCL communicator cannot be created, the reducer runs its buckets through torch.distributed
    (world 1 here: no all-reduce needed) instead of failing the run or mixing transports across ranks."""
    import warnings
    from can_distributed_pytorch_amd.parallel import reducer as R
    params = [torch.nn.Parameter(torch.randn(300)), torch.nn.Parameter(torch.randn(50))]
    arena = FlatArena(params, torch.device("cpu"), order=[1, 0])

    def boom(*a, **k):
        raise RuntimeError("rccl init refused")
    monkeypatch.setattr(R, "make_rccl_comm", boom)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        red = R.BucketedReducer(arena, [1, 0], bucket_mb=1.0, transport="rccl")
    assert red.transport == "torch" and red.comm is None and red._native is None
    assert any("torch.distributed" in str(x.message) for x in w)
    red.begin()
    red.mark_ready([1, 0])
    red.finish()
