"""CANNet — Context-Aware Crowd Counting network (Liu, Salzmann, Fua, CVPR 2019).

Parity targets in the reference (`/root/reference`):
  * module layout / state_dict names   — model/CANNet.py:8-25
  * forward math (context module)       — model/CANNet.py:39-91
  * weight init (normal std 0.01)       — model/CANNet.py:93-101
  * make_layers cfg builder             — model/CANNet.py:104-121
  * VGG-16 positional frontend transfer — model/CANNet.py:26-35

Design (MI355X-first, not a port):
  * The nn.Module keeps the reference's parameter names/shapes so `.pth`
    checkpoints are interchangeable (both the plain and the DDP
    ``module.``-prefixed layout load).
  * On a GPU tensor the forward runs through the native executor
    (:mod:`can_distributed_pytorch_amd.ops.executor`): NHWC bf16 activations,
    hand-written gfx950 MFMA implicit-GEMM convolutions with fused epilogues,
    fused context module, and a hand-scheduled backward that hands finished
    gradient buckets to the RCCL reducer while later layers are still running.
    If the HIP extension is missing on a GPU this raises — there is no silent
    eager fallback.
  * On CPU (and with ``backend="torch"``) the forward is the plain ATen graph
    of the reference; it is the numerical oracle for every kernel test and the
    "reference stack" used to measure stock PyTorch-ROCm throughput.
"""
from __future__ import annotations

import collections
import os
from typing import Dict, Iterable, List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

FRONTEND_CFG = [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512]
BACKEND_CFG = [512, 512, 512, 256, 128, 64]
CONTEXT_SCALES = (1, 2, 3, 6)
FUSE_EPS = 1e-12  # model/CANNet.py:84


def make_layers(cfg, in_channels: int = 3, batch_norm: bool = False, dilation: bool = False) -> nn.Sequential:
    """cfg list -> Sequential(Conv3x3[,BN],ReLU | MaxPool2x2).  (model/CANNet.py:104-121)

    ``dilation=True`` selects the backend form: dilation 2, padding 2.
    """
    d = 2 if dilation else 1
    layers: List[nn.Module] = []
    c = in_channels
    for v in cfg:
        if v == "M":
            layers.append(nn.MaxPool2d(kernel_size=2, stride=2))
            continue
        layers.append(nn.Conv2d(c, v, kernel_size=3, padding=d, dilation=d))
        if batch_norm:
            layers.append(nn.BatchNorm2d(v))
        layers.append(nn.ReLU(inplace=True))
        c = v
    return nn.Sequential(*layers)


def _conv_layers(seq: nn.Sequential) -> List[nn.Conv2d]:
    return [m for m in seq if isinstance(m, nn.Conv2d)]


class CANNet(nn.Module):
    """Reference-compatible CANNet.

    Args:
        load_weights: reference semantics — ``False`` means "initialise"
            (normal(0, 0.01) + optional VGG-16 frontend transfer), ``True``
            means "weights will be loaded from a checkpoint, skip init".
        vgg16_path: optional local torchvision-layout VGG-16 state_dict
            (``features.{0..28}.*``); the first 20 tensors are copied into the
            frontend positionally, exactly as the reference does. The
            reference downloads it from the network; there is no network
            here, so by default the frontend stays random-initialised.
            Also read from ``$CANNET_VGG16`` when not given.
        backend: ``"auto"`` (native HIP executor on GPU tensors, ATen on CPU),
            ``"hip"`` (force native; raises on CPU), ``"torch"`` (plain ATen
            graph everywhere — the stock-PyTorch reference stack), ``"hip_fp32"``
            (fp32 training numerics: every convolution as split-bf16 on the
            MFMA kernels, ops/fp32.py; GPU only).
    """

    def __init__(self, load_weights: bool = False, vgg16_path: Optional[str] = None,
                 backend: str = "auto", batch_norm: bool = False):
        super().__init__()
        if backend not in ("auto", "hip", "torch", "hip_fp32"):
            raise ValueError(f"unknown backend {backend!r}")
        self.frontend_feat = list(FRONTEND_CFG)
        self.backend_feat = list(BACKEND_CFG)
        self.frontend = make_layers(self.frontend_feat, batch_norm=batch_norm)
        self.backend = make_layers(self.backend_feat, in_channels=1024, batch_norm=batch_norm, dilation=True)
        self.output_layer = nn.Conv2d(64, 1, kernel_size=1)
        for s in CONTEXT_SCALES:
            setattr(self, f"conv{s}_1", nn.Conv2d(512, 512, kernel_size=1, bias=False))
            setattr(self, f"conv{s}_2", nn.Conv2d(512, 512, kernel_size=1, bias=False))
        # `backend` is the reference's nn.Sequential name (state_dict
        # compatibility), so the execution backend lives in `exec_backend`.
        self.exec_backend = backend
        self._executor = None
        if not load_weights:
            self._initialize_weights()
            path = vgg16_path or os.environ.get("CANNET_VGG16")
            if path:
                self.load_vgg16_frontend(path)

    # ------------------------------------------------------------------ init
    def _initialize_weights(self) -> None:
        """normal(0, 0.01) conv weights, zero bias; BN (1, 0).  (model/CANNet.py:93-101)"""
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.normal_(m.weight, std=0.01)
                if m.bias is not None:
                    nn.init.constant_(m.bias, 0)
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def load_vgg16_frontend(self, path: str) -> None:
        """Positional copy of the first len(frontend.state_dict()) VGG-16 tensors.

        Same mapping as model/CANNet.py:30-35 (features.{0,2,5,...,21}.{weight,bias}).
        Loaded with ``weights_only=True`` — nothing in the file is executed.
        """
        sd = torch.load(path, map_location="cpu", weights_only=True)
        if "state_dict" in sd and isinstance(sd["state_dict"], dict):
            sd = sd["state_dict"]
        src = list(sd.values())
        dst_keys = list(self.frontend.state_dict().keys())
        fsd = collections.OrderedDict((k, src[i]) for i, k in enumerate(dst_keys))
        self.frontend.load_state_dict(fsd)

    # ------------------------------------------------------------ checkpoint
    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        """Accepts both the plain and the DDP (``module.``-prefixed) key layout.

        The reference saves `DDP.state_dict()` (train.py:161) and then loads it
        into a bare CANNet with strict=False, which silently loads nothing
        (SURVEY Appendix A, Q1).  Here the prefix is stripped first.
        """
        state_dict = strip_module_prefix(state_dict)
        return super().load_state_dict(state_dict, strict=strict, assign=assign)

    # --------------------------------------------------------------- helpers
    def frontend_convs(self) -> List[nn.Conv2d]:
        return _conv_layers(self.frontend)

    def backend_convs(self) -> List[nn.Conv2d]:
        return _conv_layers(self._modules["backend"])

    def context_convs(self) -> Dict[int, tuple]:
        return {s: (getattr(self, f"conv{s}_1"), getattr(self, f"conv{s}_2")) for s in CONTEXT_SCALES}

    def _use_native(self, x: torch.Tensor) -> bool:
        if self.exec_backend == "torch":
            return False
        if self.exec_backend == "hip":
            if not x.is_cuda:
                raise RuntimeError("backend='hip' needs a GPU tensor")
            return True
        return x.is_cuda

    # --------------------------------------------------------------- forward
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.exec_backend == "hip_fp32":
            if not x.is_cuda:
                raise RuntimeError("backend='hip_fp32' needs a GPU tensor")
            from ..ops.fp32 import cannet_forward_fp32
            return cannet_forward_fp32(self, x)
        if self._use_native(x):
            if self._executor is None:
                from ..ops.executor import CANNetExecutor  # raises loudly if the HIP extension is missing
                self._executor = CANNetExecutor(self)
            return self._executor(x)
        return cannet_forward_reference(self, x)


def cannet_forward_reference(model: CANNet, x: torch.Tensor) -> torch.Tensor:
    """Plain-ATen forward with the reference's math (model/CANNet.py:39-91)."""
    fv = model.frontend(x)
    h, w = fv.shape[2], fv.shape[3]
    num = None
    den = None
    for s in CONTEXT_SCALES:
        c1, c2 = getattr(model, f"conv{s}_1"), getattr(model, f"conv{s}_2")
        ave = c1(F.adaptive_avg_pool2d(fv, (s, s)))
        up = F.interpolate(ave, size=(h, w), mode="bilinear", align_corners=True)
        wgt = torch.sigmoid(c2(up - fv))
        num = wgt * up if num is None else num + wgt * up
        den = wgt if den is None else den + wgt
    fi = num / (den + FUSE_EPS)
    y = torch.cat((fv, fi), 1)
    y = model._modules["backend"](y)
    return model.output_layer(y)


def grad_ready_order(model: CANNet) -> List[int]:
    """model.parameters() indices in the order a backward produces their gradients: output head, backend (last
    layer first), conv{S}_2, conv{S}_1, frontend (last layer first).  The native executor's schedule
    (ops/executor.py CANNetExecutor.grad_ready_order) and the flat gradient arena follow it, so DDP-style buckets
     are contiguous slices."""
    pid = {id(p): i for i, p in enumerate(model.parameters())}
    order = [pid[id(model.output_layer.weight)], pid[id(model.output_layer.bias)]]
    for m in reversed(model.backend_convs()):
        order += [pid[id(m.weight)], pid[id(m.bias)]]
    order += [pid[id(getattr(model, f"conv{s}_2").weight)] for s in CONTEXT_SCALES]
    order += [pid[id(getattr(model, f"conv{s}_1").weight)] for s in CONTEXT_SCALES]
    for m in reversed(model.frontend_convs()):
        order += [pid[id(m.weight)], pid[id(m.bias)]]
    rest = [i for i in range(len(pid)) if i not in set(order)]       # BN variant: its affine params last
    return order + rest


def strip_module_prefix(state_dict) -> "collections.OrderedDict[str, torch.Tensor]":
    out = collections.OrderedDict()
    for k, v in state_dict.items():
        out[k[7:] if k.startswith("module.") else k] = v
    return out


def reference_state_dict_keys() -> List[str]:
    """Key order of the reference's CANNet.state_dict()."""
    keys = []
    for i in (0, 2, 5, 7, 10, 12, 14, 17, 19, 21):
        keys += [f"frontend.{i}.weight", f"frontend.{i}.bias"]
    for i in (0, 2, 4, 6, 8, 10):
        keys += [f"backend.{i}.weight", f"backend.{i}.bias"]
    keys += ["output_layer.weight", "output_layer.bias"]
    for s in CONTEXT_SCALES:
        keys += [f"conv{s}_1.weight", f"conv{s}_2.weight"]
    return keys
