#!/usr/bin/env python
"""Test-set MAE and density-map viewer (reference: test.py — cal_mae, estimate_density_map).

    python test.py --data_root data/Shanghai_part_A/ --checkpoint checkpoints/epoch_354.pth
    python test.py --synthetic 768x1024 --checkpoint checkpoints/epoch_0.pth --show 3

Checkpoints in either layout load (plain CANNet state_dict, or the reference's
own DDP ``module.``-prefixed file — the reference's strict load fails on those).
MAE = mean |sum(pred) - sum(gt)| over the test images, one image per batch
(test.py:24-35); RMSE is reported too.  Runs on the native HIP executor on a GPU.
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from can_distributed_pytorch_amd.models import CANNet  # noqa: E402
from can_distributed_pytorch_amd.utils.checkpoint import load_checkpoint  # noqa: E402


def _dataset(img_root, gt_root, synthetic=""):
    from can_distributed_pytorch_amd.data import CrowdDataset, SyntheticCrowdDataset
    if synthetic:
        h, w = (int(v) for v in synthetic.lower().split("x"))
        return SyntheticCrowdDataset(16, h, w, seed=1)
    return CrowdDataset(img_root, gt_root, 8, phase="test")


def cal_mae(img_root, gt_dmap_root, model_param_path, device=None, synthetic=""):
    """Mean absolute count error over the test set (test.py:10-35)."""
    from can_distributed_pytorch_amd.engine.train_eval import evaluate_per_image
    device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
    model = CANNet(load_weights=True)
    load_checkpoint(model, model_param_path, strict=True)
    model.to(device)
    loader = torch.utils.data.DataLoader(_dataset(img_root, gt_dmap_root, synthetic), batch_size=1, shuffle=False)
    mae, rmse = evaluate_per_image(model, loader, device)
    print(f"model_param_path: {model_param_path}, mae: {mae}, rmse: {rmse}")
    return mae, rmse


@torch.no_grad()
def estimate_density_map(img_root, gt_dmap_root, model_param_path, index, out_png="density_map.png", device=None,
                         synthetic=""):
    """Predicted density map of the index-th test image (test.py:38-62), saved as a PNG (jet colormap)."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
    model = CANNet(load_weights=True)
    load_checkpoint(model, model_param_path, strict=True)
    model.to(device).eval()
    img, gt = _dataset(img_root, gt_dmap_root, synthetic)[index]
    et = model(img[None].to(device)).squeeze(0).squeeze(0).float().cpu().numpy()
    print(et.shape, "pred count", float(et.sum()), "gt count", float(gt.sum()))
    plt.imsave(out_png, et, cmap="jet")
    return et


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--data_root", default="./data/Shanghai_part_A/")
    ap.add_argument("--checkpoint", default="./checkpoints/epoch_354.pth")
    ap.add_argument("--synthetic", default="")
    ap.add_argument("--show", type=int, default=-1, help="save the density map of this test index")
    ap.add_argument("--device", default=None)
    a = ap.parse_args()
    img_root = os.path.join(a.data_root, "test_data", "images")
    gt_root = os.path.join(a.data_root, "test_data", "ground_truth")
    cal_mae(img_root, gt_root, a.checkpoint, a.device, a.synthetic)
    if a.show >= 0:
        estimate_density_map(img_root, gt_root, a.checkpoint, a.show, device=a.device, synthetic=a.synthetic)
