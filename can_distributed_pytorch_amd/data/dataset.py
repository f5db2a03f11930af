"""CrowdDataset — reference data contract (model/CrowdDataset.py:11-69).

``CrowdDataset(img_root, gt_dmap_root, gt_downsample=1, phase='train')``
lists the files of ``img_root``; item i = (image [3,H',W'] float32 ImageNet-
normalised, density [1,H'/d,W'/d] float32) with H', W' the largest multiples
of d, a random horizontal flip of BOTH in phase 'train', and the ground
truth loaded from ``gt_dmap_root/<name>.npy`` (``.jpg`` -> ``.npy``).

Differences: gt_downsample <= 1 works (Q8), integer
images only are /255 (Q14), decoding uses PIL (cv2 is not a dependency).
The random flip (model/CrowdDataset.py:48-50, Python ``random`` there) is a
pure function of (seed, epoch, index) — a counter-based hash, no RNG state:
DataLoader workers cannot replay one another's stream (a ``random.Random``
pickled into every worker would), and a resumed run draws exactly the flips
of an uninterrupted one.  The epoch comes from ``set_epoch`` or, with
worker processes, travels with the index (``EpochTaggedSampler``).
``SyntheticCrowdDataset`` provides the same item contract without files
(benchmarks, tests, smoke runs).
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np
import torch
from torch.utils.data import Dataset

from .transforms import _axis_weights, prepare_pair

IMG_EXT = (".jpg", ".jpeg", ".png", ".bmp", ".tif", ".tiff")
_M64 = (1 << 64) - 1


def _splitmix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & _M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & _M64
    return x ^ (x >> 31)


def flip_draw(seed: int, epoch: int, index: int) -> bool:
    """The p=0.5 horizontal flip of sample ``index`` in ``epoch`` (stateless, worker-independent)."""
    return bool(_splitmix64(_splitmix64(_splitmix64(seed & _M64) ^ (epoch & _M64)) ^ (index & _M64)) >> 63)


def density_to_gt(dmap: np.ndarray, h: int, w: int, downsample: int, flip: bool) -> np.ndarray:
    """The density half of prepare_pair (model/CrowdDataset.py:48-62): optional flip, cv2 INTER_LINEAR resize to
    (W//d, H//d) of the IMAGE's size, x d^2.  Returns fp32 [1, H//d, W//d]."""
    if tuple(dmap.shape) != (h, w):
        raise ValueError("density must match the image size")
    rows, cols = h // downsample, w // downsample
    if (rows, cols) == (h, w):
        dm = np.asarray(dmap, dtype=np.float64)[:, ::-1] if flip else np.asarray(dmap, dtype=np.float64)
    else:
        # gather the rows the vertical taps use first (a memory-mapped map is read only there), then resize
        y0, y1, fy = _axis_weights(h, rows)
        x0, x1, fx = _axis_weights(w, cols)
        if flip:                                 # flip before resize == mirrored column taps
            x0, x1 = w - 1 - x0, w - 1 - x1
        need = np.unique(np.concatenate([y0, y1]))
        sub = np.asarray(dmap[need], dtype=np.float64)
        pos = np.searchsorted(need, np.arange(h))
        r = sub[pos[y0]] * (1.0 - fy)[:, None] + sub[pos[y1]] * fy[:, None]
        dm = r[:, x0] * (1.0 - fx)[None] + r[:, x1] * fx[None]
    return (dm * (downsample * downsample))[None].astype(np.float32)


class EpochTaggedSampler:
    """Wraps a sampler (e.g. DistributedSampler) so that every index carries the sampler's epoch:
    yields (index, epoch) pairs, which ``CrowdDataset.__getitem__`` accepts.  Needed because persistent
    DataLoader workers hold their own copy of the dataset (``dataset.set_epoch`` in the main process would
    not reach them)."""

    def __init__(self, sampler):
        self.sampler = sampler

    def set_epoch(self, epoch: int):
        self.sampler.set_epoch(epoch)

    def __iter__(self):
        ep = int(getattr(self.sampler, "epoch", 0))
        for i in self.sampler:
            yield (int(i), ep)

    def __len__(self):
        return len(self.sampler)

    def __getattr__(self, name):          # total_size, num_replicas, ... of the wrapped sampler
        return getattr(self.sampler, name)


def imread(path: str) -> np.ndarray:
    from PIL import Image
    with Image.open(path) as im:
        if im.mode not in ("L", "RGB", "RGBA"):
            im = im.convert("RGB")
        return np.asarray(im)


class CrowdDataset(Dataset):
    def __init__(self, img_root: str, gt_dmap_root: str, gt_downsample: int = 1, phase: str = "train",
                 seed: Optional[int] = None, raw: bool = False):
        self.img_root = img_root
        self.gt_dmap_root = gt_dmap_root
        self.gt_downsample = max(1, int(gt_downsample))
        self.phase = phase
        self.img_names = sorted(f for f in os.listdir(img_root)
                                if os.path.isfile(os.path.join(img_root, f)) and f.lower().endswith(IMG_EXT))
        self.n_samples = len(self.img_names)
        self.seed = 0 if seed is None else int(seed)
        self.epoch = 0
        # raw=True: return (uint8 image, full-res density, flip) and let the GPU
        # preprocess it (ops/preprocess.py) instead of resizing on the CPU
        self.raw = raw

    def __len__(self):
        return self.n_samples

    def set_epoch(self, epoch: int):
        self.epoch = int(epoch)

    def gt_path(self, name: str) -> str:
        stem = os.path.splitext(name)[0]
        return os.path.join(self.gt_dmap_root, stem + ".npy")

    def __getitem__(self, index):
        epoch = self.epoch
        if isinstance(index, (tuple, list)):
            index, epoch = int(index[0]), int(index[1])
        if not 0 <= index < len(self):
            raise IndexError("index range error")
        name = self.img_names[index]
        img = imread(os.path.join(self.img_root, name))
        flip = self.phase == "train" and flip_draw(self.seed, epoch, index)
        if self.raw:
            # the GPU resizes / normalises the image; the ground truth is brought to its 1/d resolution here,
            # reading only the source rows the bilinear taps touch (memory-mapped: ~1/4 of a full-resolution
            # fp32 map), so a batch moves ~8x fewer host bytes than shipping full-resolution densities
            if img.dtype != np.uint8:
                img = np.clip(np.asarray(img, dtype=np.float64) * (255.0 if img.dtype.kind == "f" else 1.0),
                              0, 255).astype(np.uint8)
            dmap = np.load(self.gt_path(name), mmap_mode="r")        # allow_pickle=False (default)
            gt = density_to_gt(dmap, img.shape[0], img.shape[1], self.gt_downsample, flip)
            return torch.from_numpy(np.require(img, requirements=("C", "W"))), torch.from_numpy(gt), flip
        dmap = np.load(self.gt_path(name))                       # allow_pickle=False (default)
        im, dm = prepare_pair(img, dmap, self.gt_downsample, flip)
        return torch.from_numpy(np.ascontiguousarray(im)), torch.from_numpy(np.ascontiguousarray(dm))


class SyntheticCrowdDataset(Dataset):
    """Deterministic synthetic crowd images of a fixed size (same item contract)."""

    def __init__(self, n: int, height: int = 768, width: int = 1024, gt_downsample: int = 8, seed: int = 0,
                 heads=(100, 1500)):
        from .synthetic import make_synthetic_batch
        self._make = make_synthetic_batch
        self.n, self.h, self.w = n, height, width
        self.seed = seed
        self.heads = heads
        self.gt_downsample = gt_downsample
        if gt_downsample != 8:
            raise ValueError("synthetic density maps are produced at 1/8 resolution")

    def __len__(self):
        return self.n

    def __getitem__(self, index):
        if isinstance(index, (tuple, list)):
            index = int(index[0])
        img, gt = self._make(1, self.h, self.w, seed=self.seed * 100003 + index, heads=self.heads)
        return img[0], gt[0]
