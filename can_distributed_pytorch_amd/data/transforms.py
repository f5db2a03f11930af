"""Image/density-map transforms with the reference's exact semantics, without OpenCV.

The reference resizes with cv2.resize(..., INTER_LINEAR) (model/CrowdDataset.py:57-61):
half-pixel-centre bilinear interpolation, source coordinates clamped to the
border, NO anti-aliasing when shrinking (the 1/8 density map is point-sampled
between pixels 8x+3 and 8x+4, then multiplied by 64).  ``resize_linear`` is a
separable float64 implementation of that rule (cv2 computes float images in
float arithmetic, so this matches it to rounding).
"""
from __future__ import annotations

import numpy as np

IMAGENET_MEAN = np.array([0.485, 0.456, 0.406], dtype=np.float32)
IMAGENET_STD = np.array([0.229, 0.224, 0.225], dtype=np.float32)


def _axis_weights(in_size: int, out_size: int):
    scale = in_size / out_size
    src = (np.arange(out_size, dtype=np.float64) + 0.5) * scale - 0.5
    x0 = np.floor(src)
    frac = src - x0
    x0 = x0.astype(np.int64)
    # cv2 border handling: clamp both taps into [0, in-1]; a coordinate left
    # of 0 collapses onto pixel 0 (weight moves entirely to the clamped tap)
    neg = x0 < 0
    frac[neg] = 0.0
    x0[neg] = 0
    x1 = np.minimum(x0 + 1, in_size - 1)
    x0 = np.minimum(x0, in_size - 1)
    return x0, x1, frac


def resize_linear(arr: np.ndarray, out_w: int, out_h: int) -> np.ndarray:
    """cv2.resize(arr, (out_w, out_h), interpolation=INTER_LINEAR) for HxW or HxWxC float arrays."""
    h, w = arr.shape[:2]
    if (h, w) == (out_h, out_w):
        return arr.copy()
    a = arr.astype(np.float64, copy=False)
    y0, y1, fy = _axis_weights(h, out_h)
    x0, x1, fx = _axis_weights(w, out_w)
    shape_y = (-1,) + (1,) * (a.ndim - 1)
    rows = a[y0] * (1.0 - fy).reshape(shape_y) + a[y1] * fy.reshape(shape_y)
    shape_x = (1, -1) + (1,) * (a.ndim - 2)
    out = rows[:, x0] * (1.0 - fx).reshape(shape_x) + rows[:, x1] * fx.reshape(shape_x)
    return out.astype(arr.dtype if arr.dtype.kind == "f" else np.float64)


def to_unit_float(img: np.ndarray) -> np.ndarray:
    """Integer images /255 -> [0,1]; float images are kept (reference Q14: PNGs are already float)."""
    if img.dtype.kind in "ui":
        return img.astype(np.float64) / 255.0
    return img.astype(np.float64)


def gray_to_rgb(img: np.ndarray) -> np.ndarray:
    if img.ndim == 2:
        img = img[:, :, None]
    if img.shape[2] == 1:
        img = np.concatenate([img, img, img], axis=2)
    if img.shape[2] == 4:  # RGBA -> RGB
        img = img[:, :, :3]
    return img


def normalize_chw(img_hwc: np.ndarray) -> np.ndarray:
    chw = img_hwc.transpose(2, 0, 1).astype(np.float32)
    return (chw - IMAGENET_MEAN[:, None, None]) / IMAGENET_STD[:, None, None]


def prepare_pair(img: np.ndarray, dmap: np.ndarray, downsample: int = 8, flip: bool = False):
    """Full reference transform (model/CrowdDataset.py:38-67): returns (img CHW f32, dmap 1xhxw f32)."""
    img = gray_to_rgb(to_unit_float(img))
    if flip:
        img = img[:, ::-1]
        dmap = dmap[:, ::-1]
    if downsample < 1:
        raise ValueError("downsample must be >= 1")
    rows, cols = img.shape[0] // downsample, img.shape[1] // downsample
    img = resize_linear(np.ascontiguousarray(img), cols * downsample, rows * downsample)
    dm = resize_linear(np.ascontiguousarray(dmap, dtype=np.float32), cols, rows) * (downsample * downsample)
    return normalize_chw(img), dm[None].astype(np.float32)
