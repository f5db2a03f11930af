"""Compatibility module for ``from model.CANNet import CANNet`` (reference layout)."""
from can_distributed_pytorch_amd.models.cannet import CANNet, make_layers  # noqa: F401
