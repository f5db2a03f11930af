"""Compatibility package: ``from model import CANNet, CrowdDataset`` as in the
reference (model/__init__.py).  The implementation lives in can_distributed_pytorch_amd."""
from can_distributed_pytorch_amd.models.cannet import CANNet, make_layers  # noqa: F401
from can_distributed_pytorch_amd.data.dataset import CrowdDataset  # noqa: F401
