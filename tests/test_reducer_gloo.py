"""Fake-cluster tests of the bucketed reducer and the distributed helpers (gloo, CPU, 2-3 ranks)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(fn, world, *args):
    port = _free_port()
    mp.spawn(_entry, args=(fn, world, port) + args, nprocs=world, join=True)


def _entry(rank, fn, world, port, *args):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fn(rank, world, *args)
    finally:
        dist.destroy_process_group()


def _bucket_case(rank, world, order_shuffle):
    from can_distributed_pytorch_amd.utils.flat import FlatArena
    from can_distributed_pytorch_amd.parallel.reducer import BucketedReducer
    torch.manual_seed(0)
    shapes = [(64, 3, 3, 3), (64,), (300, 200), (7,), (128, 64, 3, 3), (1000,), (5, 5)]
    params = [torch.nn.Parameter(torch.zeros(s)) for s in shapes]
    order = [6, 5, 4, 3, 2, 1, 0]
    arena = FlatArena(params, "cpu", order=order)
    red = BucketedReducer(arena, order, bucket_mb=0.1, first_bucket_mb=0.01, transport="torch")
    assert len(red.buckets) >= 3
    for step in range(2):
        grads = arena.grad_views()
        for i, g in enumerate(grads):
            g.copy_(torch.full_like(g, float(rank + 1 + 10 * i + 100 * step)))
        red.begin()
        marks = list(order)
        if order_shuffle:
            g = torch.Generator().manual_seed(rank + 7 * step)     # ranks mark in DIFFERENT orders
            marks = [marks[i] for i in torch.randperm(len(marks), generator=g).tolist()]
        for i in marks:
            red.mark_ready([i])
        red.finish()
        tot = sum(r + 1 for r in range(world))
        for i, g in enumerate(arena.grad_views()):
            expect = tot + world * (10 * i + 100 * step)
            assert torch.all(g == expect), (i, g.flatten()[:3], expect)


@pytest.mark.parametrize("shuffle", [False, True])
def test_bucketed_reducer_gloo(shuffle):
    _run(_bucket_case, 2, shuffle)


def _scalar_case(rank, world):
    from can_distributed_pytorch_amd.parallel import distributed as D
    v = torch.tensor([float(rank + 1)])
    D.reduce_value(v, average=True)
    assert abs(v.item() - (world + 1) / 2) < 1e-6
    vec = D.reduce_scalars(torch.tensor(1.0 * rank), torch.tensor(2.0), average=False)
    assert vec.tolist() == [sum(range(world)), 2.0 * world]
    assert D.get_world_size() == world and D.get_rank() == rank
    assert D.is_main_process() == (rank == 0)


def test_reduce_helpers_gloo():
    _run(_scalar_case, 3)


def _hook_case(rank, world):
    """Autograd path: post-accumulate hooks drive the reducer; result == mean-free SUM of per-rank grads."""
    from can_distributed_pytorch_amd.utils.flat import FlatArena
    from can_distributed_pytorch_amd.parallel.reducer import BucketedReducer
    torch.manual_seed(1)
    net = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 4))
    params = list(net.parameters())
    order = list(reversed(range(len(params))))
    arena = FlatArena(params, "cpu", order=order)
    red = BucketedReducer(arena, order, bucket_mb=0.001, first_bucket_mb=0.0005, transport="torch")
    red.attach_hooks()
    x = torch.randn(8, 16) + rank
    arena.grad.zero_()
    red.begin()
    net(x).pow(2).sum().backward()
    red.finish()
    got = [g.clone() for g in arena.grad_views()]
    # reference: full-batch grads from every rank's input, summed
    ref = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 4))
    ref.load_state_dict(net.state_dict())
    tot = [torch.zeros_like(p) for p in ref.parameters()]
    for r in range(world):
        ref.zero_grad()
        ref(torch.randn(8, 16, generator=None) * 0 + (x - rank + r)).pow(2).sum().backward()
        for t, p in zip(tot, ref.parameters()):
            t += p.grad
    for g, t in zip(got, tot):
        assert torch.allclose(g, t, rtol=1e-4, atol=1e-4)


def test_reducer_autograd_hooks_gloo():
    _run(_hook_case, 2)


def _consistency_case(rank, world):
    from can_distributed_pytorch_amd.parallel.consistency import check_replicas_consistent
    x = torch.arange(1000, dtype=torch.float32)
    assert check_replicas_consistent(x)
    y = x.clone()
    if rank == 1:
        y[17] += 1e-3
    try:
        check_replicas_consistent(y)
        raised = False
    except RuntimeError:
        raised = True
    assert raised


def test_replica_desync_detection_gloo():
    _run(_consistency_case, 2)


class _FakeExt:
    """Stands in for the native extension inside a spawned rank: scripted unique-id / communicator failures."""

    def __init__(self, rank, uid_fails=False, init_fails_on=None):
        self.rank, self.uid_fails, self.init_fails_on = rank, uid_fails, init_fails_on
        self.made = []

    def rccl_unique_id(self):
        if self.uid_fails:
            raise OSError("no network interface for the bootstrap")
        return b"\0" * 128

    def RcclComm(self, rank, world, uid, device, timeout):
        if rank == self.init_fails_on:
            raise ValueError("scripted init failure (not a RuntimeError)")
        ext = self

        class _Comm:
            aborted = False

            def abort(self):
                _Comm.aborted = True
        c = _Comm()
        ext.made.append(c)
        return c


def _comm_agreement_case(rank, world, uid_fails, init_fails_on):
    """Every rank returns from reducer construction (no rank stranded in a blocking call) and every rank falls back
    to the torch transport together; a communicator that did get made on a healthy rank is aborted."""
    import warnings
    from can_distributed_pytorch_amd.ops import _ext
    from can_distributed_pytorch_amd.parallel import reducer as R
    from can_distributed_pytorch_amd.utils.flat import FlatArena
    fake = _FakeExt(rank, uid_fails=uid_fails, init_fails_on=init_fails_on)
    _ext.require = lambda: fake
    params = [torch.nn.Parameter(torch.zeros(100)), torch.nn.Parameter(torch.zeros(10))]
    arena = FlatArena(params, "cpu", order=[1, 0])
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        red = R.BucketedReducer(arena, [1, 0], bucket_mb=1.0, transport="rccl")
    assert red.transport == "torch" and red._native is None
    assert all(c.aborted for c in fake.made)
    if not uid_fails and rank != init_fails_on:
        assert len(fake.made) == 1                 # this rank's own init succeeded, then it was aborted
    for g in arena.grad_views():
        g.fill_(rank + 1.0)
    red.begin()
    red.mark_ready([1, 0])
    red.finish()                                   # the fallback transport really reduces
    assert all(torch.all(g == sum(r + 1.0 for r in range(world))) for g in arena.grad_views())


@pytest.mark.parametrize("uid_fails,init_fails_on", [(True, None), (False, 1), (False, 0)])
def test_rccl_comm_failure_agreement_multirank(uid_fails, init_fails_on):
    _run(_comm_agreement_case, 3, uid_fails, init_fails_on)
