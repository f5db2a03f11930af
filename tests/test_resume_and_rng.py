"""Exact resume and data-augmentation randomness (CPU).

* resume: save_train_state -> load_train_state -> k steps is BITWISE equal to k more steps of the
  uninterrupted run (weights, optimizer momentum, and every RNG stream);
* flips: a pure function of (seed, epoch, index): DataLoader workers do not replay one stream (ADVICE r1:
  a ``random.Random`` pickled into each worker did), and resumed epochs draw the same flips.
"""
import os
import random

import numpy as np
import pytest
import torch

from can_distributed_pytorch_amd.data.dataset import CrowdDataset, EpochTaggedSampler, flip_draw
from can_distributed_pytorch_amd.utils.checkpoint import load_train_state, save_train_state


def _stepper(seed):
    from can_distributed_pytorch_amd.engine.trainer import TorchStepper
    from can_distributed_pytorch_amd.models import CANNet
    torch.manual_seed(seed)
    m = CANNet(backend="torch")
    for mod in m.modules():                       # He init: visible gradients in a few steps
        if isinstance(mod, torch.nn.Conv2d):
            torch.nn.init.normal_(mod.weight, std=(2.0 / (mod.in_channels * 9)) ** 0.5)
    return TorchStepper("cpu", dtype="fp32", lr=1e-6, model=m)


def _batch(step):
    g = torch.Generator().manual_seed(100 + step)
    return torch.randn(1, 3, 32, 32, generator=g), torch.rand(1, 1, 4, 4, generator=g)


def test_resume_is_bitwise_exact(tmp_path):
    # oneDNN may pick a different conv algorithm on a model's first call than on later ones, and multithreaded
    # CPU reductions change the summation order run to run (measured: the last bits of some gradients
    # differed), so the comparison runs on ATen's native CPU convolution with one thread: deterministic
    nt = torch.get_num_threads()
    torch.set_num_threads(1)
    try:
        with torch.backends.mkldnn.flags(enabled=False):
            _resume_case(tmp_path)
    finally:
        torch.set_num_threads(nt)


def _resume_case(tmp_path):
    a = _stepper(0)
    for s in range(3):
        a.step(*_batch(s))
    path = os.path.join(tmp_path, "last_state.pth")
    torch.manual_seed(77)
    np.random.seed(78)
    random.seed(79)
    save_train_state(path, a.model, None, epoch=4, min_mae=12.5, optimizer=a.opt, min_epoch=2)
    for s in range(3, 5):
        a.step(*_batch(s))
    draws_a = (torch.rand(3), np.random.rand(3), [random.random() for _ in range(3)])

    b = _stepper(1)                                # different init: everything must come from the file
    torch.manual_seed(0)
    np.random.seed(0)
    random.seed(0)
    rs = load_train_state(path, b.model, optimizer=b.opt)
    assert (rs["epoch"], rs["min_mae"], rs["min_epoch"]) == (4, 12.5, 2)
    for s in range(3, 5):
        b.step(*_batch(s))
    draws_b = (torch.rand(3), np.random.rand(3), [random.random() for _ in range(3)])
    for (n, pa), pb in zip(a.model.named_parameters(), b.model.parameters()):
        assert torch.equal(pa, pb), n
    assert torch.equal(draws_a[0], draws_b[0])
    assert np.array_equal(draws_a[1], draws_b[1])
    assert draws_a[2] == draws_b[2]


def test_flip_draw_is_balanced_and_epoch_dependent():
    f = [flip_draw(0, 0, i) for i in range(4000)]
    assert 0.45 < sum(f) / len(f) < 0.55
    g = [flip_draw(0, 1, i) for i in range(4000)]
    assert f != g
    assert [flip_draw(3, 5, i) for i in range(50)] == [flip_draw(3, 5, i) for i in range(50)]


def _write_set(root, n=12, h=32, w=48):
    from PIL import Image
    img_dir, gt_dir = os.path.join(root, "images"), os.path.join(root, "gt")
    os.makedirs(img_dir)
    os.makedirs(gt_dir)
    rng = np.random.default_rng(0)
    for i in range(n):
        # left half dark, right half bright: a flip is visible in the mean of the left half
        a = np.zeros((h, w, 3), np.uint8)
        a[:, w // 2:] = 255
        Image.fromarray(a).save(os.path.join(img_dir, f"IMG_{i}.png"))
        np.save(os.path.join(gt_dir, f"IMG_{i}.npy"), rng.random((h, w)).astype(np.float32))
    return img_dir, gt_dir


def _flips_via_loader(ds, epoch, workers):
    from torch.utils.data import DataLoader, DistributedSampler, BatchSampler
    smp = DistributedSampler(ds, num_replicas=1, rank=0, shuffle=True, seed=0)
    smp.set_epoch(epoch)
    bs = BatchSampler(EpochTaggedSampler(smp), 1, drop_last=False)
    dl = DataLoader(ds, batch_sampler=bs, num_workers=workers)
    order = list(smp)
    flips = {}
    for i, (img, _) in zip(order, dl):
        flips[i] = bool(img[0, 0, :, : img.shape[-1] // 2].mean() > 0)   # bright left half => flipped
    return flips


def test_worker_flips_match_in_process_and_differ_per_epoch(tmp_path):
    img_dir, gt_dir = _write_set(str(tmp_path))
    ds = CrowdDataset(img_dir, gt_dir, gt_downsample=8, phase="train", seed=5)
    f0 = _flips_via_loader(ds, 0, workers=0)
    f0w = _flips_via_loader(ds, 0, workers=2)
    assert f0 == f0w                                   # two workers: no shared/replayed stream
    assert f0 == {i: flip_draw(5, 0, i) for i in range(len(ds))}
    f1 = _flips_via_loader(ds, 1, workers=2)
    assert f1 == {i: flip_draw(5, 1, i) for i in range(len(ds))} and f1 != f0
