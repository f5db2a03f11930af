"""Density-map overlays (reference utils/train_eval_utils.py:88-118, Q7 std typo fixed)."""
from __future__ import annotations

import os

import numpy as np
import torch

MEAN = np.array([0.485, 0.456, 0.406], dtype=np.float32)
STD = np.array([0.229, 0.224, 0.225], dtype=np.float32)


def denormalize(img: torch.Tensor) -> np.ndarray:
    x = img.detach().float().cpu().permute(1, 2, 0).numpy()
    return np.clip(x * STD + MEAN, 0, 1)


def _upsample(d: np.ndarray, h: int, w: int) -> np.ndarray:
    from ..data.transforms import resize_linear
    return resize_linear(d.astype(np.float32), w, h)


def save_overlays(img, gt, et, epoch, out_dir="checkpoints/temp"):
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    os.makedirs(out_dir, exist_ok=True)
    im = denormalize(img)
    h, w = im.shape[:2]
    paths = []
    for tag, d in (("gt", gt), ("et", et)):
        dm = _upsample(d.detach().float().cpu().numpy().reshape(d.shape[-2], d.shape[-1]), h, w)
        fig = plt.figure()
        plt.axis("off")
        plt.imshow(im)
        plt.imshow(dm, alpha=0.5, cmap="turbo")
        p = os.path.join(out_dir, f"temp_{tag}_{epoch}.png")
        fig.savefig(p, bbox_inches="tight", pad_inches=0)
        plt.close(fig)
        paths.append(p)
    return paths
