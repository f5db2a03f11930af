"""GPU input pipeline: decoded uint8 image + full-res density -> network inputs.

Same result as CrowdDataset's CPU transform (data/transforms.py:prepare_pair,
reference model/CrowdDataset.py:38-67) but computed by csrc/preprocess.hip
on the GPU, writing the first conv layer's NHWC4 bf16 layout directly.

Per batch: the DataLoader worker packs the decoded samples back to back
(``PackedCollate``: one uint8 image buffer, one fp32 density buffer, a
descriptor table), the main process makes one pinned H2D copy of each and
ONE kernel launch turns the batch into network inputs (``preprocess_packed``).
``preprocess_batch`` is the per-sample form (tests / variable-size use).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import torch

from . import _ext


def preprocess_batch(images: Sequence[torch.Tensor], densities: Sequence[torch.Tensor], flips: Sequence[bool],
                     device, downsample: int = 8, dtype: torch.dtype = torch.bfloat16) -> Tuple[torch.Tensor, torch.Tensor]:
    """images: uint8 [H,W] / [H,W,C] (CPU or GPU), densities: fp32 [H,W].  All samples must
    resize to the same (H//d*d, W//d*d).  Returns (x4 [N,Ho,Wo,4] bf16/fp16, gt [N,1,Ho/d,Wo/d] fp32)."""
    C = _ext.require()
    dev = torch.device(device)
    n = len(images)
    if not (n == len(densities) == len(flips)) or n == 0:
        raise ValueError("images, densities and flips must have the same non-zero length")
    h0, w0 = images[0].shape[:2]
    ho, wo = (h0 // downsample) * downsample, (w0 // downsample) * downsample
    from .conv import dt_code
    dt = dt_code(dtype)
    x4 = torch.empty(n, ho, wo, 4, dtype=dtype, device=dev)
    gt = torch.empty(n, 1, ho // downsample, wo // downsample, dtype=torch.float32, device=dev)
    st = _ext.stream_ptr(dev)
    for i, (im, dm, fl) in enumerate(zip(images, densities, flips)):
        if im.dtype != torch.uint8:
            raise ValueError("images must be uint8 (decoded JPEG/PNG)")
        hh, ww = im.shape[:2]
        if (hh // downsample * downsample, ww // downsample * downsample) != (ho, wo):
            raise ValueError("all samples of a batch must resize to the same shape")
        im = im.to(dev, non_blocking=True).contiguous()
        ch = 1 if im.dim() == 2 else im.shape[2]
        dm = dm.to(dev, dtype=torch.float32, non_blocking=True).contiguous()
        if tuple(dm.shape) != (hh, ww):
            raise ValueError("density must match the image size")
        C.preprocess_image(im.data_ptr(), hh, ww, ch, int(bool(fl)), x4[i].data_ptr(), ho, wo, dt, st)
        C.preprocess_density(dm.data_ptr(), hh, ww, int(bool(fl)), gt[i].data_ptr(), ho // downsample,
                             wo // downsample, float(downsample * downsample), st)
    return x4, gt


class RawCollate:
    """collate_fn for CrowdDataset(raw=True): keeps samples as lists (variable sizes allowed until preprocessing)."""

    def __call__(self, batch: List):
        imgs, dens, flips = zip(*batch)
        return list(imgs), list(dens), list(flips)


class PackedCollate:
    """collate_fn for CrowdDataset(raw=True) that packs a batch for ONE H2D copy of the images and ONE launch:
    returns (images uint8 [sum of H*W*C], gt fp32 [n,1,H/d,W/d], desc int64 [n, 8], (Ho, Wo)) with
    desc[i] = (image byte offset, H0, W0, C, flip, 0, 0, 0).  The raw dataset already brought each ground truth
    to 1/d resolution (flip and x d^2 included), so only the images are resized on the GPU.  Runs in the
    loader workers; pin_memory=True pins both buffers."""

    def __init__(self, downsample: int = 8):
        self.ds = downsample

    def __call__(self, batch: List):
        imgs, gts, flips = zip(*batch)
        h0, w0 = imgs[0].shape[:2]
        ho, wo = (h0 // self.ds) * self.ds, (w0 // self.ds) * self.ds
        desc = torch.zeros(len(imgs), 8, dtype=torch.int64)
        ioff = 0
        for i, (im, g, fl) in enumerate(zip(imgs, gts, flips)):
            hh, ww = im.shape[:2]
            if (hh // self.ds * self.ds, ww // self.ds * self.ds) != (ho, wo):
                raise ValueError("all samples of a batch must resize to the same shape")
            if tuple(g.shape) != (1, ho // self.ds, wo // self.ds):
                raise ValueError("raw samples must carry the 1/d ground truth [1, H/d, W/d]")
            ch = 1 if im.dim() == 2 else im.shape[2]
            desc[i] = torch.tensor([ioff, hh, ww, ch, int(bool(fl)), 0, 0, 0])
            ioff += hh * ww * ch
        ibuf = torch.cat([im.reshape(-1) for im in imgs])
        return ibuf, torch.stack(gts), desc, (ho, wo)


def preprocess_packed(packed, device, downsample: int = 8, dtype: torch.dtype = torch.bfloat16):
    """PackedCollate output -> (x4 [N,Ho,Wo,4] 16-bit NHWC4, gt [N,1,Ho/d,Wo/d] fp32): one copy per buffer and one
    launch for the whole batch of images."""
    C = _ext.require()
    ibuf, gt, desc, (ho, wo) = packed
    if ibuf.dtype != torch.uint8 or gt.dtype != torch.float32 or desc.dtype != torch.int64:
        raise ValueError("packed batch: uint8 images, fp32 ground truth, int64 descriptors")
    dev = torch.device(device)
    n = desc.shape[0]
    from .conv import dt_code
    ib = ibuf.to(dev, non_blocking=True)
    ds = desc.to(dev, non_blocking=True)
    gtd = gt.to(dev, non_blocking=True)
    x4 = torch.empty(n, ho, wo, 4, dtype=dtype, device=dev)
    C.preprocess_batch(ib.data_ptr(), 0, ds.data_ptr(), n, x4.data_ptr(), 0, ho, wo, downsample, dt_code(dtype),
                       _ext.stream_ptr(dev))
    return x4, gtd
