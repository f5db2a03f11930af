#!/usr/bin/env python
"""Write a local ShanghaiTech-layout crowd set of JPEGs + .npy density maps (no dataset can be downloaded):
<root>/{train_data,test_data}/{images/IMG_k.jpg, ground_truth/IMG_k.npy}, the layout train.py --data_root reads
(reference model/CrowdDataset.py:16-46).  Images are the synthetic crowd recipe (data/synthetic.py) at full
resolution, JPEG quality 90; densities are full-resolution fp32 maps (count = heads inside the image).

usage: python scripts/make_jpeg_set.py --root /tmp/sha_synth --train 192 --test 32 --height 768 --width 1024
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from can_distributed_pytorch_amd.data.synthetic import (IMAGENET_MEAN, IMAGENET_STD,  # noqa: E402
                                                        density_from_points_fixed, synthetic_points)


# ShanghaiTech Part A mixes image sizes (mostly <= 1024 on the long side, landscape and portrait); these (H, W) pairs
# follow that spread.  After CrowdDataset's resize to multiples of 8 most widths are not multiples of 128, so the
# native kernels run their ragged (masked) tiles.
MIXED_SIZES = [(768, 1024), (683, 1024), (1024, 768), (576, 768), (480, 640), (400, 600), (600, 800), (765, 1020),
               (532, 800), (704, 1000), (450, 680), (1000, 667), (620, 900), (384, 512), (720, 960), (510, 760)]


def render(seed, h, w, heads=(100, 1500)):
    gen = torch.Generator().manual_seed(seed)
    n = int(torch.randint(heads[0], heads[1] + 1, (1,), generator=gen))
    pts = synthetic_points(n, h, w, gen)
    dens = density_from_points_fixed(pts, h, w)
    base = torch.rand(3, h // 16, w // 16, generator=gen)
    img = torch.nn.functional.interpolate(base[None], size=(h, w), mode="bilinear", align_corners=False)[0]
    img = (0.7 * img + 0.3 * (dens / (dens.max() + 1e-6))[None]).clamp(0, 1)
    return (img.permute(1, 2, 0).numpy() * 255 + 0.5).astype(np.uint8), dens.numpy().astype(np.float32)


def _write(job):
    idir, gdir, k, seed, h, w = job
    from PIL import Image
    torch.set_num_threads(1)
    img, dens = render(seed, h, w)
    Image.fromarray(img).save(os.path.join(idir, f"IMG_{k + 1}.jpg"), quality=90)
    np.save(os.path.join(gdir, f"IMG_{k + 1}.npy"), dens)
    return k


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--root", required=True)
    ap.add_argument("--train", type=int, default=192)
    ap.add_argument("--test", type=int, default=32)
    ap.add_argument("--height", type=int, default=768)
    ap.add_argument("--width", type=int, default=1024)
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--mixed", action="store_true",
                    help="ShanghaiTech-A-like mixed sizes (landscape / portrait, W %% 128 != 0 for most) instead of "
                         "--height x --width")
    a = ap.parse_args()
    _ = (IMAGENET_MEAN, IMAGENET_STD)
    from multiprocessing import Pool
    for part, n, off in (("train_data", a.train, 0), ("test_data", a.test, 100000)):
        idir, gdir = os.path.join(a.root, part, "images"), os.path.join(a.root, part, "ground_truth")
        os.makedirs(idir, exist_ok=True)
        os.makedirs(gdir, exist_ok=True)
        if a.mixed:
            jobs = [(idir, gdir, k, off + k) + MIXED_SIZES[(off + k) % len(MIXED_SIZES)] for k in range(n)]
        else:
            jobs = [(idir, gdir, k, off + k, a.height, a.width) for k in range(n)]
        with Pool(a.workers) as pool:
            for i, _k in enumerate(pool.imap_unordered(_write, jobs)):
                if (i + 1) % 64 == 0:
                    print(part, i + 1, "/", n, flush=True)
    print("wrote", a.train, "+", a.test, "images to", a.root)


if __name__ == "__main__":
    main()
