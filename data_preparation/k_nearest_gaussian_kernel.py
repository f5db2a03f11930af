"""Compatibility entry point for the reference's GT generator script
(data_preparation/k_nearest_gaussian_kernel.py).  Usage:
    python data_preparation/k_nearest_gaussian_kernel.py <ShanghaiTech part root> [--gpu]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from can_distributed_pytorch_amd.data.density import gaussian_filter_density, generate_dataset_density  # noqa: E402,F401

if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--gpu", action="store_true")
    a = ap.parse_args()
    print(generate_dataset_density(a.root, use_gpu=a.gpu), "density maps written")
