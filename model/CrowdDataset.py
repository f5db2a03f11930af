"""Compatibility module for ``from model.CrowdDataset import CrowdDataset`` (reference layout)."""
from can_distributed_pytorch_amd.data.dataset import CrowdDataset  # noqa: F401


if __name__ == "__main__":
    # dataset smoke test (reference model/CrowdDataset.py:73-86): one sample's shapes and ranges
    import sys
    if len(sys.argv) < 3:
        from can_distributed_pytorch_amd.data import SyntheticCrowdDataset
        ds = SyntheticCrowdDataset(1, 256, 256)
    else:
        ds = CrowdDataset(sys.argv[1], sys.argv[2], gt_downsample=8, phase="train")
    img, gt = ds[0]
    print(tuple(img.shape), float(img.min()), float(img.max()), tuple(gt.shape), float(gt.sum()))
