"""Compatibility module for ``from model.CrowdDataset import CrowdDataset`` (reference layout)."""
from can_distributed_pytorch_amd.data.dataset import CrowdDataset  # noqa: F401
