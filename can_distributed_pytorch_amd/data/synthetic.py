"""Synthetic crowd images + density maps (no dataset download is possible here).

Shapes follow the reference's data contract (model/CrowdDataset.py:53-67):
image  [3, H, W] ImageNet-normalised float, H, W multiples of 8;
density [1, H/8, W/8], resized from the full-res map and multiplied by 64 so
that its sum stays the head count.

Generation is cheap and deterministic per seed.  Heads are drawn as clustered
2-D points; the full-resolution density is the sum of per-head Gaussians
(fixed sigma here — the geometry-adaptive generator lives in
data/density.py), and the 1/8 map is produced by 8x8 sum pooling, which
preserves the count exactly.
"""
from __future__ import annotations

import math
from typing import Tuple

import torch

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def synthetic_points(n_heads: int, h: int, w: int, gen: torch.Generator) -> torch.Tensor:
    """[n,2] float (x=col, y=row) points in clusters (crowds are clumpy)."""
    n_clusters = max(1, n_heads // 64)
    centers = torch.rand(n_clusters, 2, generator=gen) * torch.tensor([w, h])
    spread = torch.rand(n_clusters, 1, generator=gen) * 0.15 * min(h, w) + 4.0
    idx = torch.randint(0, n_clusters, (n_heads,), generator=gen)
    pts = centers[idx] + torch.randn(n_heads, 2, generator=gen) * spread[idx]
    pts[:, 0].clamp_(0, w - 1)
    pts[:, 1].clamp_(0, h - 1)
    return pts


def density_from_points_fixed(points: torch.Tensor, h: int, w: int, sigma: float = 4.0) -> torch.Tensor:
    """Full-res density [h,w] with a fixed-sigma Gaussian per head (separable, exact mass inside the image)."""
    dens = torch.zeros(h, w, dtype=torch.float32, device=points.device)
    if points.numel() == 0:
        return dens
    r = int(4 * sigma + 0.5)
    ks = torch.arange(-r, r + 1, device=points.device, dtype=torch.float32)
    g = torch.exp(-0.5 * (ks / sigma) ** 2)
    g = g / g.sum()
    ys = points[:, 1].long().clamp(0, h - 1)
    xs = points[:, 0].long().clamp(0, w - 1)
    delta = torch.zeros(h, w, device=points.device)
    delta.index_put_((ys, xs), torch.ones_like(ys, dtype=torch.float32), accumulate=True)
    k = g.view(1, 1, -1)
    tmp = torch.nn.functional.conv1d(delta.view(h, 1, w), k, padding=r).view(h, w)
    dens = torch.nn.functional.conv1d(tmp.t().contiguous().view(w, 1, h), k, padding=r).view(w, h).t()
    return dens.contiguous()


def make_synthetic_batch(batch: int, h: int, w: int, seed: int = 0, device="cpu",
                         heads: Tuple[int, int] = (100, 1500)) -> Tuple[torch.Tensor, torch.Tensor]:
    """Returns (img [B,3,H,W] normalised fp32, gt [B,1,H/8,W/8] fp32) on ``device``."""
    assert h % 8 == 0 and w % 8 == 0, "H and W must be multiples of 8"
    gen = torch.Generator().manual_seed(seed)
    imgs = torch.empty(batch, 3, h, w)
    gts = torch.empty(batch, 1, h // 8, w // 8)
    mean = torch.tensor(IMAGENET_MEAN).view(3, 1, 1)
    std = torch.tensor(IMAGENET_STD).view(3, 1, 1)
    for b in range(batch):
        n = int(torch.randint(heads[0], heads[1] + 1, (1,), generator=gen))
        pts = synthetic_points(n, h, w, gen)
        dens = density_from_points_fixed(pts, h, w)
        # texture: smooth noise + bright blobs where heads are
        base = torch.rand(3, h // 16, w // 16, generator=gen)
        img = torch.nn.functional.interpolate(base[None], size=(h, w), mode="bilinear", align_corners=False)[0]
        img = (0.7 * img + 0.3 * (dens / (dens.max() + 1e-6))[None]).clamp(0, 1)
        imgs[b] = (img - mean) / std
        gts[b, 0] = dens.view(h // 8, 8, w // 8, 8).sum(dim=(1, 3))
    return imgs.to(device), gts.to(device)


def make_synthetic_batch_gpu(batch: int, h: int, w: int, seed: int = 0, device="cuda",
                             heads: Tuple[int, int] = (100, 1500), dtype: torch.dtype = torch.bfloat16,
                             nhwc4: bool = True, seeds=None):
    """The same recipe rendered on the GPU (csrc/preprocess.hip synth_render + the density splat of
    csrc/density.hip): only the head points and a coarse noise grid are drawn on the host.  Returns
    (x4 [B,H,W,4] 16-bit NHWC4 — the first layer's input layout — or, nhwc4=False, img [B,3,H,W] fp32,
    gt [B,1,H/8,W/8] fp32).  Statistically the CPU generator's images; not bitwise (different resampling
    order), and reproducible per seed to fp32 rounding only (the density splat adds with fp32 atomics).  seeds: optional per-image seeds (image i a function of seeds[i] alone: sharded datasets)."""
    from ..ops import _ext
    from ..ops.conv import dt_code
    C = _ext.require()
    assert h % 16 == 0 and w % 16 == 0, "H and W must be multiples of 16"
    dev = torch.device(device)
    gens = [torch.Generator().manual_seed(int(sd)) for sd in seeds] if seeds is not None else \
        [torch.Generator().manual_seed(seed)] * batch
    if len(gens) != batch:
        raise ValueError("len(seeds) != batch")
    pts, noise = [], torch.empty(batch, 3, h // 16, w // 16)
    for b, gen in enumerate(gens):
        n = int(torch.randint(heads[0], heads[1] + 1, (1,), generator=gen))
        pts.append(synthetic_points(n, h, w, gen))
        noise[b] = torch.rand(3, h // 16, w // 16, generator=gen)
    dens = torch.zeros(batch, h, w, dtype=torch.float32, device=dev)
    st = _ext.stream_ptr(dev)
    for b, p in enumerate(pts):
        pd = p.to(dev).contiguous()
        sig = torch.empty(pd.shape[0], dtype=torch.float32, device=dev)
        C.density_map(pd.data_ptr(), pd.shape[0], h, w, sig.data_ptr(), dens[b].data_ptr(), 0, st, 4.0)
    x4 = torch.empty(batch, h, w, 4, dtype=dtype, device=dev)
    gt = torch.empty(batch, 1, h // 8, w // 8, dtype=torch.float32, device=dev)
    dmax = torch.empty(batch, dtype=torch.float32, device=dev)
    nz = noise.to(dev)
    C.synth_render(dens.data_ptr(), nz.data_ptr(), dmax.data_ptr(), x4.data_ptr(), gt.data_ptr(), batch, h, w,
                   dt_code(dtype), st)
    if nhwc4:
        return x4, gt
    return x4[..., :3].float().permute(0, 3, 1, 2).contiguous(), gt


class SyntheticGPULoader:
    """Batches of a synthetic crowd set rendered on the GPU, driven by a (distributed) batch sampler: image
    ``index`` is a function of (seed, index) only, so ranks shard it exactly like a file dataset.  Yields
    (x4 [B,H,W,4] NHWC4 16-bit, gt [B,1,H/8,W/8] fp32) already on ``device``."""

    def __init__(self, batch_sampler, h: int, w: int, seed: int, device, dtype=torch.bfloat16,
                 heads: Tuple[int, int] = (100, 1500)):
        self.bs, self.h, self.w, self.seed = batch_sampler, h, w, seed
        self.device, self.dtype, self.heads = device, dtype, heads

    def __len__(self):
        return len(self.bs)

    def __iter__(self):
        for idx in self.bs:
            idx = [int(i[0]) if isinstance(i, (tuple, list)) else int(i) for i in idx]
            yield make_synthetic_batch_gpu(len(idx), self.h, self.w, device=self.device, heads=self.heads,
                                           dtype=self.dtype, seeds=[self.seed * 100003 + i for i in idx])


def expected_flops_per_image(h: int, w: int) -> float:
    """Forward conv FLOPs (2*MAC) of CANNet at HxW input (733.4 GF at 768x1024)."""
    from ..models.cannet import FRONTEND_CFG, BACKEND_CFG
    fl = 0.0
    c, hh, ww = 3, h, w
    for v in FRONTEND_CFG:
        if v == "M":
            hh //= 2
            ww //= 2
            continue
        fl += 2.0 * hh * ww * c * v * 9
        c = v
    p = hh * ww
    fl += sum(2.0 * s * s * 512 * 512 for s in (1, 2, 3, 6)) + 4 * 2.0 * p * 512 * 512
    c = 1024
    for v in BACKEND_CFG:
        fl += 2.0 * p * c * v * 9
        c = v
    fl += 2.0 * p * 64
    return fl


__all__ = ["make_synthetic_batch", "make_synthetic_batch_gpu", "SyntheticGPULoader", "synthetic_points", "density_from_points_fixed",
           "expected_flops_per_image", "IMAGENET_MEAN", "IMAGENET_STD"]
