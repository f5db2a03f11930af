"""Data layer: cv2-equivalent resize, CrowdDataset contract, density generator vs SciPy (CPU)."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from can_distributed_pytorch_amd.data import transforms as T
from can_distributed_pytorch_amd.data.density import gaussian_filter_density, knn_sigmas


@pytest.mark.parametrize("hw,out", [((37, 53), (29, 41)), ((64, 96), (8, 12)), ((20, 30), (40, 60)), ((5, 7), (5, 7))])
def test_resize_linear_matches_half_pixel_bilinear(hw, out):
    rng = np.random.default_rng(0)
    a = rng.random(hw + (3,))
    got = T.resize_linear(a, out[1], out[0])
    ref = F.interpolate(torch.from_numpy(a).permute(2, 0, 1)[None], size=out, mode="bilinear",
                        align_corners=False, antialias=False)[0].permute(1, 2, 0).numpy()
    assert got.shape == ref.shape
    assert np.abs(got - ref).max() < 1e-9


def test_density_downsample_times_64_semantics():
    """1/8 map = point-sampled bilinear (pixels 8x+3, 8x+4 averaged) x 64 (model/CrowdDataset.py:58-60)."""
    rng = np.random.default_rng(1)
    d = rng.random((32, 48)).astype(np.float32)
    dm = T.resize_linear(d, 6, 4) * 64
    expect = 64 * 0.25 * (d[3::8][:, 3::8] + d[3::8][:, 4::8] + d[4::8][:, 3::8] + d[4::8][:, 4::8])
    assert np.allclose(dm, expect, atol=1e-5)


def test_prepare_pair_flip_and_normalise():
    rng = np.random.default_rng(2)
    img = (rng.random((40, 56, 3)) * 255).astype(np.uint8)
    dm = rng.random((40, 56)).astype(np.float32)
    a, ga = T.prepare_pair(img, dm, 8, flip=False)
    b, gb = T.prepare_pair(img, dm, 8, flip=True)
    assert a.shape == (3, 40, 56) and ga.shape == (1, 5, 7)
    assert np.allclose(a[:, :, ::-1], b, atol=1e-6)
    assert np.allclose(ga[:, :, ::-1], gb, atol=1e-6)
    raw = img.astype(np.float64) / 255
    expect = (raw[..., 0] - 0.485) / 0.229
    assert np.allclose(a[0], expect, atol=1e-5)


def test_gray_and_float_inputs():
    g = np.full((16, 16), 128, np.uint8)
    a, _ = T.prepare_pair(g, np.zeros((16, 16), np.float32), 8)
    assert a.shape == (3, 16, 16)
    f = np.full((16, 16, 3), 0.5, np.float32)   # float image: NOT divided by 255 (Q14)
    b, _ = T.prepare_pair(f, np.zeros((16, 16), np.float32), 8)
    assert np.allclose(b[1], (0.5 - 0.456) / 0.224, atol=1e-5)


def test_crowd_dataset_files(tmp_path):
    from PIL import Image
    from can_distributed_pytorch_amd.data.dataset import CrowdDataset
    (tmp_path / "img").mkdir()
    (tmp_path / "gt").mkdir()
    rng = np.random.default_rng(3)
    for i in range(3):
        Image.fromarray((rng.random((35 + i, 50, 3)) * 255).astype(np.uint8)).save(tmp_path / "img" / f"IMG_{i}.jpg")
        np.save(tmp_path / "gt" / f"IMG_{i}.npy", rng.random((35 + i, 50)).astype(np.float32))
    ds = CrowdDataset(str(tmp_path / "img"), str(tmp_path / "gt"), gt_downsample=8, phase="test")
    assert len(ds) == 3
    x, y = ds[0]
    assert x.dtype == torch.float32 and x.shape == (3, 32, 48) and y.shape == (1, 4, 6)
    with pytest.raises(IndexError):
        ds[3]
    ds1 = CrowdDataset(str(tmp_path / "img"), str(tmp_path / "gt"), gt_downsample=1, phase="train", seed=0)
    x1, y1 = ds1[2]
    assert x1.shape == (3, 37, 50) and y1.shape == (1, 37, 50)


def _reference_density(shape, pts):
    """The reference's O(N*H*W) procedure, verbatim semantics, with scipy."""
    from scipy.ndimage import gaussian_filter
    from scipy.spatial import KDTree
    h, w = shape
    dens = np.zeros(shape, np.float32)
    tree = KDTree(pts.copy(), leafsize=2048)
    dist, _ = tree.query(pts, k=4)
    for i, pt in enumerate(pts):
        d = np.zeros(shape, np.float32)
        if int(pt[1]) < h and int(pt[0]) < w:
            d[int(pt[1]), int(pt[0])] = 1.0
        else:
            continue
        sigma = (dist[i][1] + dist[i][2] + dist[i][3]) * 0.1
        dens += gaussian_filter(d, sigma, mode="constant")
    return dens


def test_density_matches_scipy_reference():
    rng = np.random.default_rng(4)
    h, w = 60, 80
    pts = np.stack([rng.random(40) * w * 1.05, rng.random(40) * h * 1.05], 1)   # a few out of bounds
    got = gaussian_filter_density((h, w), pts)
    ref = _reference_density((h, w), pts)
    assert np.abs(got - ref).max() < 1e-6
    inside = ((pts[:, 0] < w) & (pts[:, 1] < h)).sum()
    assert got.sum() <= inside + 1e-3


def test_density_single_point_and_empty():
    d0 = gaussian_filter_density((20, 30), np.zeros((0, 2)))
    assert d0.shape == (20, 30) and d0.sum() == 0
    d1 = gaussian_filter_density((40, 40), np.array([[20.0, 20.0]]))
    assert 0.85 < d1.sum() < 1.0                 # sigma = avg(shape)/4 = 10: +-2 sigma inside the image
    assert knn_sigmas(np.array([[1.0, 1.0]]), (40, 40))[0] == 10.0


def test_density_to_gt_matches_prepare_pair_memmap(tmp_path):
    """The raw (GPU-preprocessed) dataset's CPU ground-truth path == prepare_pair's density output, bitwise,
    with and without the flip, reading the .npy memory-mapped."""
    import numpy as np
    from can_distributed_pytorch_amd.data.dataset import density_to_gt
    from can_distributed_pytorch_amd.data.transforms import prepare_pair
    rng = np.random.default_rng(12)
    for (h, w) in [(77, 101), (64, 96), (35, 17)]:
        d = rng.random((h, w)).astype(np.float32)
        img = (rng.random((h, w, 3)) * 255).astype(np.uint8)
        path = tmp_path / f"d{h}.npy"
        np.save(path, d)
        mm = np.load(path, mmap_mode="r")
        for flip in (False, True):
            ref = prepare_pair(img, d, 8, flip)[1]
            assert np.array_equal(density_to_gt(mm, h, w, 8, flip), ref)
