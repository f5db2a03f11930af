"""The flat-arena data-parallel step (engine/trainer.py ArenaStepper) against torch DDP + torch.optim.SGD
(the reference's train.py:121-126 stack), on CPU: one rank and a 2-rank gloo fake cluster."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batches(rank, n=3):
    from can_distributed_pytorch_amd.data.synthetic import make_synthetic_batch
    return [make_synthetic_batch(1, 32, 32, seed=100 * rank + i, device="cpu") for i in range(n)]


def _compare(rank, world):
    from can_distributed_pytorch_amd.engine.trainer import ArenaStepper, TorchStepper
    from can_distributed_pytorch_amd.models.cannet import CANNet
    torch.manual_seed(0)
    base = CANNet(backend="torch")
    m1, m2 = CANNet(backend="torch"), CANNet(backend="torch")
    m1.load_state_dict(base.state_dict())
    m2.load_state_dict(base.state_dict())
    ours = ArenaStepper("cpu", world=world, lr=1e-4, model=m1, bucket_mb=4.0)
    ref = TorchStepper("cpu", dtype="fp32", world=world, lr=1e-4, model=m2, bucket_mb=4.0)
    for img, gt in _batches(rank):
        lo = ours.step(img, gt)
        lr_ = ref.step(img, gt)
        # ours reports the rank-mean loss (reduce_value(loss, average=True)); torch's is this rank's
        if world == 1:
            assert torch.allclose(lo, lr_.reshape(1), rtol=1e-5)
    for (k, a), b in zip(m1.state_dict().items(), m2.state_dict().values()):
        assert torch.allclose(a, b, rtol=1e-4, atol=1e-7), (k, (a - b).abs().max())
    assert len(ours.reducer.buckets) >= 3


def test_arena_stepper_matches_torch_sgd_single_rank():
    _compare(0, 1)


def _entry(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _compare(rank, world)
    finally:
        dist.destroy_process_group()


def test_arena_stepper_matches_ddp_two_ranks():
    mp.spawn(_entry, args=(2, _free_port()), nprocs=2, join=True)


def test_grad_ready_order_matches_executor_schedule():
    from can_distributed_pytorch_amd.models.cannet import CANNet, grad_ready_order
    from can_distributed_pytorch_amd.ops import _ext
    m = CANNet(backend="torch")
    order = grad_ready_order(m)
    assert sorted(order) == list(range(len(list(m.parameters()))))
    if _ext.available():
        from can_distributed_pytorch_amd.ops.executor import CANNetExecutor
        assert CANNetExecutor(m).grad_ready_order() == order
