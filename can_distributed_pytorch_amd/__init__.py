"""can_distributed_pytorch_amd — MI355X-native CANNet training/eval framework.

Capabilities of zgzhengSEU/CAN-distributed-pytorch, re-designed for gfx950:
hand-written MFMA HIP kernels for the hot ops, a native RCCL bucketed
gradient reducer, hipGraph-captured training steps.  See SURVEY.md.
"""
from .models.cannet import CANNet, make_layers  # noqa: F401

__version__ = "0.1.0"
