"""Geometry-adaptive Gaussian ground-truth density maps.

Reference: data_preparation/k_nearest_gaussian_kernel.py:14-92.

* ``gaussian_filter_density(img_or_shape, points)`` — CPU version with the
  reference semantics (KD-tree 4-NN, sigma = 0.1*(d1+d2+d3), single head:
  avg(shape)/4, heads at (row=int(y), col=int(x)), out-of-image heads
  skipped).  Instead of filtering a full H*W delta image per head
  (O(N*H*W)), each head adds the clipped outer product of two normalised 1-D
  Gaussians of radius int(4*sigma+0.5) — identical to
  scipy.ndimage.gaussian_filter(delta, sigma, mode='constant') (truncate 4).
* ``density_map_gpu(points, H, W)`` — the same on the GPU (csrc/density.hip:
  brute-force kNN + per-head splat).
* ``generate_dataset_density(root)`` — the offline driver (ShanghaiTech layout:
  images/*.jpg + ground_truth/GT_IMG_*.mat -> ground_truth/IMG_*.npy).
"""
from __future__ import annotations

import glob
import os
from typing import Sequence, Tuple, Union

import numpy as np
import torch


def _shape_of(img_or_shape) -> Tuple[int, int]:
    if isinstance(img_or_shape, (tuple, list)):
        return int(img_or_shape[0]), int(img_or_shape[1])
    return int(img_or_shape.shape[0]), int(img_or_shape.shape[1])


def _kernel1d(sigma: float) -> np.ndarray:
    r = int(4.0 * sigma + 0.5)
    x = np.arange(-r, r + 1, dtype=np.float64)
    k = np.exp(-0.5 * (x / sigma) ** 2)
    return k / k.sum()


def knn_sigmas(points: np.ndarray, shape: Tuple[int, int]) -> np.ndarray:
    n = len(points)
    if n == 0:
        return np.zeros(0)
    if n == 1:
        return np.array([np.average(np.array(shape, dtype=np.float64)) / 2.0 / 2.0])
    from scipy.spatial import KDTree
    tree = KDTree(points.copy(), leafsize=2048)
    k = min(4, n)
    dist, _ = tree.query(points, k=k)
    return 0.1 * dist[:, 1:].sum(axis=1)


def gaussian_filter_density(img_or_shape, points: Union[np.ndarray, Sequence]) -> np.ndarray:
    """points: [[col, row], ...] (x, y).  Returns float32 [H, W]."""
    h, w = _shape_of(img_or_shape)
    pts = np.asarray(points, dtype=np.float64).reshape(-1, 2)
    density = np.zeros((h, w), dtype=np.float64)
    if len(pts) == 0:
        return density.astype(np.float32)
    sig = knn_sigmas(pts, (h, w))
    for (x, y), s in zip(pts, sig):
        if x < 0 or y < 0:
            continue
        c, r = int(x), int(y)
        if r >= h or c >= w:
            continue
        if s <= 0:
            density[r, c] += 1.0
            continue
        k = _kernel1d(float(s))
        R = (len(k) - 1) // 2
        r0, r1 = max(0, r - R), min(h - 1, r + R)
        c0, c1 = max(0, c - R), min(w - 1, c + R)
        density[r0:r1 + 1, c0:c1 + 1] += np.outer(k[r0 - r + R:r1 - r + R + 1], k[c0 - c + R:c1 - c + R + 1])
    return density.astype(np.float32)


def density_map_gpu(points, h: int, w: int, device="cuda", max_radius: int = 0) -> torch.Tensor:
    """GPU density map [h, w] fp32 for points [[x, y], ...]."""
    from ..ops import _ext
    C = _ext.require()
    pts = torch.as_tensor(np.asarray(points, dtype=np.float32).reshape(-1, 2), device=device).contiguous()
    out = torch.zeros(h, w, dtype=torch.float32, device=device)
    n = pts.shape[0]
    if n == 0:
        return out
    sig = torch.empty(n, dtype=torch.float32, device=device)
    C.density_map(pts.data_ptr(), n, h, w, sig.data_ptr(), out.data_ptr(), max_radius, _ext.stream_ptr(device))
    return out


def load_sha_points(mat_path: str) -> np.ndarray:
    """ShanghaiTech GT_IMG_*.mat -> N x 2 (x=col, y=row) (reference :79-81)."""
    from scipy.io import loadmat
    mat = loadmat(mat_path)
    return np.asarray(mat["image_info"][0, 0][0, 0][0], dtype=np.float64)


def generate_dataset_density(root: str, parts=("train_data", "test_data"), use_gpu: bool = False) -> int:
    """Offline driver (reference :58-92): writes ground_truth/IMG_k.npy next to images/IMG_k.jpg."""
    from .dataset import imread
    count = 0
    for part in parts:
        for img_path in sorted(glob.glob(os.path.join(root, part, "images", "*.jpg"))):
            mat = img_path.replace(".jpg", ".mat").replace("images", "ground_truth").replace("IMG_", "GT_IMG_")
            img = imread(img_path)
            pts = load_sha_points(mat)
            if use_gpu and torch.cuda.is_available():
                d = density_map_gpu(pts, img.shape[0], img.shape[1]).cpu().numpy()
            else:
                d = gaussian_filter_density(img, pts)
            out = img_path.replace(".jpg", ".npy").replace("images", "ground_truth")
            os.makedirs(os.path.dirname(out), exist_ok=True)
            np.save(out, d)
            count += 1
    return count


if __name__ == "__main__":  # pragma: no cover
    import argparse
    ap = argparse.ArgumentParser(description="generate geometry-adaptive density maps (ShanghaiTech layout)")
    ap.add_argument("root")
    ap.add_argument("--gpu", action="store_true")
    a = ap.parse_args()
    print(generate_dataset_density(a.root, use_gpu=a.gpu), "maps written")
