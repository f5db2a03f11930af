"""Spec-level CPU checks written from SURVEY §2.7 / §2.6 rather than from our own code paths:

* the context module (model/CANNet.py:39-91 of the reference) against an independent numpy oracle
  that spells out adaptive-avg-pool bins (floor / ceil, overlapping when H % S != 0), the 1x1
  convs, align_corners=True bilinear upsampling, the sigmoid weighting and the 1e-12 fusion;
* bucket planning (1 MiB first bucket, 25 MiB caps, contiguous slices in gradient-ready order) as a
  hypothesis property over random parameter shapes;
* distributed evaluation on a 2-rank gloo fake cluster: per-rank |sum(et) - sum(gt)|, SUM over
  ranks, divided by the DistributedSampler's PADDED total_size (utils/train_eval_utils.py:83,136,
  train.py:157 of the reference).
"""
import math
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
from hypothesis import given, settings, strategies as st


# --------------------------------------------------------------------------- context module oracle
def _adaptive_bins(n, s):
    return [(math.floor(i * n / s), math.ceil((i + 1) * n / s)) for i in range(s)]


def _pool(fv, s):                         # fv [C, H, W] -> [C, s, s]
    c, h, w = fv.shape
    out = np.zeros((c, s, s))
    for i, (h0, h1) in enumerate(_adaptive_bins(h, s)):
        for j, (w0, w1) in enumerate(_adaptive_bins(w, s)):
            out[:, i, j] = fv[:, h0:h1, w0:w1].mean(axis=(1, 2))
    return out


def _upsample_align_corners(a, h, w):     # a [C, s, s] -> [C, h, w]
    c, s, _ = a.shape
    out = np.zeros((c, h, w))
    for y in range(h):
        sy = y * (s - 1) / (h - 1) if h > 1 else 0.0
        y0 = min(int(math.floor(sy)), s - 1)
        y1 = min(y0 + 1, s - 1)
        fy = sy - y0
        for x in range(w):
            sx = x * (s - 1) / (w - 1) if w > 1 else 0.0
            x0 = min(int(math.floor(sx)), s - 1)
            x1 = min(x0 + 1, s - 1)
            fx = sx - x0
            out[:, y, x] = ((1 - fy) * (1 - fx) * a[:, y0, x0] + (1 - fy) * fx * a[:, y0, x1]
                            + fy * (1 - fx) * a[:, y1, x0] + fy * fx * a[:, y1, x1])
    return out


def _context_oracle(fv, convs):
    """fv [C, H, W] float64; convs {S: (W1 [C, C], W2 [C, C])} -> cat(fv, fi) [2C, H, W]."""
    c, h, w = fv.shape
    num = np.zeros_like(fv)
    den = np.zeros_like(fv)
    for s, (w1, w2) in convs.items():
        ave = np.einsum("oc,cij->oij", w1, _pool(fv, s))           # conv{S}_1, no ReLU (:44 commented out)
        up = _upsample_align_corners(ave, h, w)
        wgt = 1.0 / (1.0 + np.exp(-np.einsum("oc,chw->ohw", w2, up - fv)))
        num += wgt * up
        den += wgt
    return np.concatenate([fv, num / (den + 1e-12)], 0)


@pytest.mark.parametrize("h,w", [(17, 30), (12, 16), (7, 9)])
def test_context_module_matches_spec_oracle(h, w):
    """Overlapping bins: 17 % 6, 30 % 4, 7 % 3 ... != 0."""
    from can_distributed_pytorch_amd.models.cannet import CANNet, cannet_forward_reference, CONTEXT_SCALES
    torch.manual_seed(3)
    m = CANNet(backend="torch").double()
    m.frontend = torch.nn.Identity()
    m._modules["backend"] = torch.nn.Identity()
    m.output_layer = torch.nn.Identity()
    for s in CONTEXT_SCALES:      # larger weights than the 0.01 init so the sigmoids are not all ~0.5
        for k in (1, 2):
            torch.nn.init.normal_(getattr(m, f"conv{s}_{k}").weight, std=0.05)
    fv = torch.randn(1, 512, h, w, dtype=torch.float64).relu()
    with torch.no_grad():
        got = cannet_forward_reference(m, fv)[0].numpy()
    convs = {s: (getattr(m, f"conv{s}_1").weight.detach().view(512, 512).numpy(),
                 getattr(m, f"conv{s}_2").weight.detach().view(512, 512).numpy()) for s in CONTEXT_SCALES}
    ref = _context_oracle(fv[0].numpy(), convs)
    assert got.shape == (1024, h, w)
    np.testing.assert_allclose(got, ref, rtol=1e-9, atol=1e-10)


def test_adaptive_bins_overlap_like_survey():
    """H = 135, S = 6 -> bins (0, 23), (22, 45), ..."""
    b = _adaptive_bins(135, 6)
    assert b[0] == (0, 23) and b[1] == (22, 45)
    x = torch.arange(135, dtype=torch.float64).view(1, 1, 135, 1)
    got = torch.nn.functional.adaptive_avg_pool2d(x, (6, 1)).flatten().tolist()
    assert got == pytest.approx([float(np.arange(a, e).mean()) for a, e in b])


# --------------------------------------------------------------------------- bucket planning property
@settings(max_examples=60, deadline=None)
@given(sizes=st.lists(st.integers(1, 400_000), min_size=1, max_size=40),
       cap=st.sampled_from([0.25, 1.0, 4.0]), first=st.sampled_from([0.05, 0.5, 1.0]),
       seed=st.integers(0, 1000), last=st.sampled_from([None, 0.1, 1.0]))
def test_plan_buckets_properties(sizes, cap, first, seed, last):
    from can_distributed_pytorch_amd.utils.flat import FlatArena
    from can_distributed_pytorch_amd.parallel.reducer import plan_buckets, MIB
    params = [torch.nn.Parameter(torch.zeros(n)) for n in sizes]
    order = torch.randperm(len(sizes), generator=torch.Generator().manual_seed(seed)).tolist()
    arena = FlatArena(params, "cpu", order=order)
    bks = plan_buckets(arena, order, bucket_mb=cap, first_bucket_mb=first, last_bucket_mb=last)
    # every parameter exactly once, in ready order, buckets contiguous and covering the arena
    assert [i for b in bks for i in b.params] == order
    assert bks[0].start == 0 and bks[-1].end == arena.numel
    for a, b in zip(bks, bks[1:]):
        assert a.end == b.start
    padded = {i: arena.slot(i)[1] - arena.slot(i)[0] for i in order}     # slots padded to 64 elements
    for b in bks:
        assert b.numel == sum(padded[i] for i in b.params)
        assert all(padded[i] >= sizes[i] and padded[i] % 64 == 0 for i in b.params)
    # greedy part: every bucket but the tail reached its cap, and dropping its last parameter would not have
    greedy = plan_buckets(arena, order, bucket_mb=cap, first_bucket_mb=first, last_bucket_mb=None)
    caps = [first] + [cap] * (len(greedy) - 1)
    for b, c in zip(greedy[:-1], caps):
        assert b.numel * 4 >= c * MIB
        assert (b.numel - padded[b.params[-1]]) * 4 < c * MIB
    assert [b.params for b in bks[:len(greedy) - 1]] == [b.params for b in greedy[:-1]]
    # tail split: the greedy tail becomes (head, tail) with the tail <= last cap (or one parameter)
    if last is not None and len(bks) == len(greedy) + 1:
        assert bks[-2].params + bks[-1].params == greedy[-1].params
        assert bks[-1].numel * 4 <= last * MIB or len(bks[-1].params) == 1
        assert len(bks[-2].params) >= 1
    else:
        assert len(bks) == len(greedy)


# --------------------------------------------------------------------------- distributed MAE normalisation
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _CountDS(torch.utils.data.Dataset):
    """Item i: image whose pixel sum encodes i, GT density with sum 10 * i."""
    def __len__(self):
        return 5

    def __getitem__(self, i):
        img = torch.full((3, 8, 8), float(i) / 192.0)          # sum over 3x8x8 = i
        gt = torch.zeros(1, 1, 1)
        gt[0, 0, 0] = 10.0 * i
        return img, gt


class _SumModel(torch.nn.Module):
    def forward(self, x):                                        # et sum = 3 * sum(img)
        return 3.0 * x.sum(dim=(1, 2, 3)).view(-1, 1, 1, 1)


def _eval_rank(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from can_distributed_pytorch_amd.engine.train_eval import evaluate
        ds = _CountDS()
        smp = torch.utils.data.DistributedSampler(ds, num_replicas=world, rank=rank, shuffle=True, seed=7)
        dl = torch.utils.data.DataLoader(ds, batch_size=1, sampler=smp)
        mae_sum = evaluate(_SumModel(), dl, "cpu", epoch=0)
        if rank == 0:
            q.put((mae_sum, smp.total_size, list(smp)))
        else:
            q.put((None, None, list(smp)))
    finally:
        dist.destroy_process_group()


def test_distributed_mae_sums_ranks_and_divides_by_padded_size():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world = 2
    port = _free_port()
    procs = [ctx.Process(target=_eval_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    mae_sum, total, _ = next(r for r in res if r[0] is not None)
    indices = [i for r in res for i in r[2]]
    assert total == 6 and len(indices) == 6 and sorted(set(indices)) == list(range(5))   # one index repeated
    expect = sum(abs(3.0 * i - 10.0 * i) for i in indices)
    assert mae_sum == pytest.approx(expect)
    assert mae_sum / total == pytest.approx(expect / 6)     # train.py: padded size, not len(dataset)
