"""`torch.ops.cannet.*`: the native gfx950 kernels as PyTorch custom operators (SURVEY §7.1 "host framework").

The CANNet executor (ops/executor.py) schedules the whole network itself.  These registrations expose the same
kernels to ANY model: each op has a real GPU implementation (the MFMA kernels), a fake (meta) implementation for
shape propagation — so ``torch.compile`` traces them without graph breaks and ``FakeTensorMode`` works without a
GPU — and an autograd formula built from the native backward kernels.

  cannet::conv2d_nhwc(x, weight, bias, dilation, relu) -> y
      x [N,H,W,Ci] bf16/fp16 (NHWC, contiguous), weight [Co,Ci,k,k] fp32 master (k = 1 or 3), bias [Co] fp32 or
      None; stride 1, 'same' padding dilation*(k//2); y = [relu](conv(x, weight) + bias) in x.dtype.
      Ci, Co multiples of 64 (the first 3-channel layer has its own kernel inside the executor).
      Forward: conv_igemm (bias + ReLU epilogue).  Backward: dY masked by y > 0, the data gradient on the same
      kernel with the flipped / transposed weight pack, the weight + bias gradients on the split-pixel weight-
      gradient kernels (fp32, deterministic slab reduction) — the reference's nn.Conv2d + ReLU
      (model/CANNet.py:14-17, 114-115) as one op.
  cannet::relu_max_pool2x2(x) -> (y, codes)
      the ReLU-fused 2x2 / stride-2 max-pool of an NHWC map: y = max_pool2d(relu(x), 2) (= relu of the window
      max); codes = int32 first-max one-hots (4 bits per channel, 0 where the window max is <= 0).  Backward
      scatters through the codes, so the ReLU's mask is part of the gradient: exactly the gradient of
      max_pool2d(relu(x)), and of a plain max-pool only where the input is already non-negative.
  cannet::sgd_momentum_(param, momentum_buf, grad, lr, momentum, grad_scale) -> ()
      in-place fused SGD with momentum on contiguous fp32 tensors (torch.optim.SGD semantics, weight decay 0,
      dampening 0: buf = momentum * buf + grad_scale * grad; param -= lr * buf), one kernel.

``Conv2dNHWC`` / ``ReluMaxPool2x2`` are nn.Module wrappers with fp32 master parameters.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.nn as nn

from . import _ext
from . import conv as C

_LIB = "cannet"


def _conv_check(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor]) -> Tuple[int, int, int]:
    if x.dim() != 4:
        raise ValueError("x must be NHWC [N,H,W,Ci]")
    if weight.dim() != 4 or weight.shape[2] != weight.shape[3] or weight.shape[2] not in (1, 3):
        raise ValueError("weight must be [Co,Ci,k,k] with k = 1 or 3")
    co, ci, k, _ = weight.shape
    if x.shape[-1] != ci:
        raise ValueError(f"x has {x.shape[-1]} channels, weight expects {ci}")
    if ci % 64 or co % 64:
        raise ValueError("cannet::conv2d_nhwc needs Ci and Co multiples of 64")
    if x.dtype not in C.ACT_DTYPES:
        raise ValueError(f"x must be bf16 or fp16, got {x.dtype}")
    if weight.dtype != torch.float32:
        raise ValueError("weight must be the fp32 master tensor")
    if bias is not None and (bias.dtype != torch.float32 or bias.numel() != co):
        raise ValueError("bias must be fp32 [Co]")
    return ci, co, k


@torch.library.custom_op(f"{_LIB}::conv2d_nhwc", mutates_args=())
def conv2d_nhwc(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor], dilation: int = 1,
                relu: bool = True) -> torch.Tensor:
    ci, co, k = _conv_check(x, weight, bias)
    x = x.contiguous()
    wp = C.pack_weight_fwd(weight, x.dtype)
    if bias is None:
        if relu:
            bias = torch.zeros(co, dtype=torch.float32, device=x.device)
            epi = C.EPI_BIAS_RELU
        else:
            epi = C.EPI_NONE
    else:
        bias = bias.detach().contiguous()
        epi = C.EPI_BIAS_RELU if relu else C.EPI_BIAS
    return C.conv_igemm(x, wp, bias, ksize=k, dil=dilation, epi=epi)


@conv2d_nhwc.register_fake
def _(x, weight, bias, dilation=1, relu=True):
    _conv_check(x, weight, bias)
    return x.new_empty(*x.shape[:3], weight.shape[0])


@torch.library.custom_op(f"{_LIB}::conv2d_nhwc_backward", mutates_args=())
def conv2d_nhwc_backward(dy: torch.Tensor, x: torch.Tensor, y: torch.Tensor, weight: torch.Tensor, dilation: int,
                         relu: bool, need_bias: bool) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """(dx, dweight, dbias) of conv2d_nhwc; dbias is an empty tensor when need_bias is False."""
    co, ci, k, _ = weight.shape
    dz = dy.to(x.dtype)
    if relu:
        dz = torch.where(y > 0, dz, torch.zeros((), dtype=dz.dtype, device=dz.device))
    dz = dz.contiguous()
    dx = C.conv_igemm(dz, C.pack_weight_dgrad(weight, x.dtype), None, ksize=k, dil=dilation, epi=C.EPI_NONE)
    dw = torch.empty(co, ci, k, k, dtype=torch.float32, device=x.device)
    db = torch.empty(co if need_bias else 0, dtype=torch.float32, device=x.device)
    C.conv_wgrad(dz, x.contiguous(), dw, db if need_bias else None, ksize=k, dil=dilation)
    return dx, dw, db


@conv2d_nhwc_backward.register_fake
def _(dy, x, y, weight, dilation, relu, need_bias):
    co = weight.shape[0]
    return (x.new_empty(x.shape), weight.new_empty(weight.shape), weight.new_empty(co if need_bias else 0))


def _conv_setup(ctx, inputs, output):
    x, weight, bias, dilation, relu = inputs
    ctx.save_for_backward(x, weight, output)
    ctx.dilation, ctx.relu, ctx.has_bias = dilation, relu, bias is not None


def _conv_bwd(ctx, dy):
    x, weight, y = ctx.saved_tensors
    dx, dw, db = conv2d_nhwc_backward(dy, x, y, weight, ctx.dilation, ctx.relu, ctx.has_bias)
    return dx, dw, (db if ctx.has_bias else None), None, None


conv2d_nhwc.register_autograd(_conv_bwd, setup_context=_conv_setup)


@torch.library.custom_op(f"{_LIB}::relu_max_pool2x2", mutates_args=())
def relu_max_pool2x2(x: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    y, codes = C.maxpool_codes(x.contiguous())
    return y.clamp_min_(0), codes          # relu(max): a window whose max is <= 0 pools to 0 (its code is 0)


@relu_max_pool2x2.register_fake
def _(x):
    n, h, w, c = x.shape
    if h % 2 or w % 2 or c % 8:
        raise ValueError("max-pool needs even H, W and C % 8 == 0")
    return x.new_empty(n, h // 2, w // 2, c), x.new_empty(n, h // 2, w // 2, c // 8, dtype=torch.int32)


@torch.library.custom_op(f"{_LIB}::relu_max_pool2x2_backward", mutates_args=())
def relu_max_pool2x2_backward(dy: torch.Tensor, codes: torch.Tensor) -> torch.Tensor:
    return C.maxpool_bwd_codes(codes, dy.contiguous())


@relu_max_pool2x2_backward.register_fake
def _(dy, codes):
    n, h, w, c = dy.shape
    return dy.new_empty(n, 2 * h, 2 * w, c)


def _pool_setup(ctx, inputs, output):
    ctx.save_for_backward(output[1])
    ctx.mark_non_differentiable(output[1])


def _pool_bwd(ctx, dy, dcodes):
    (codes,) = ctx.saved_tensors
    return relu_max_pool2x2_backward(dy, codes)


relu_max_pool2x2.register_autograd(_pool_bwd, setup_context=_pool_setup)


@torch.library.custom_op(f"{_LIB}::sgd_momentum_", mutates_args=("param", "momentum_buf"))
def sgd_momentum_(param: torch.Tensor, momentum_buf: torch.Tensor, grad: torch.Tensor, lr: float, momentum: float,
                  grad_scale: float = 1.0) -> None:
    for t, name in ((param, "param"), (momentum_buf, "momentum_buf"), (grad, "grad")):
        if t.dtype != torch.float32 or not t.is_contiguous() or not t.is_cuda:
            raise ValueError(f"{name} must be a contiguous fp32 GPU tensor")
    if not (param.numel() == momentum_buf.numel() == grad.numel()):
        raise ValueError("param / momentum_buf / grad sizes differ")
    n = param.numel()
    if n == 0:
        return
    if any(t.data_ptr() % 16 for t in (param, momentum_buf, grad)):
        momentum_buf.mul_(momentum).add_(grad, alpha=grad_scale)      # float4 kernel needs 16-B alignment
        param.add_(momentum_buf, alpha=-lr)
        return
    Cx = _ext.require()
    # the arena kernel works on float4 groups; a ragged tail (n % 4) goes through ATen
    n4 = n - n % 4
    if n4:
        Cx.sgd_momentum(param.data_ptr(), momentum_buf.data_ptr(), grad.data_ptr(), n4, float(lr), float(momentum),
                        float(grad_scale), 0, 0, 0, _ext.stream_ptr(param.device))
    if n4 < n:
        b, g, p = momentum_buf.view(-1)[n4:], grad.view(-1)[n4:], param.view(-1)[n4:]
        b.mul_(momentum).add_(g, alpha=grad_scale)
        p.add_(b, alpha=-lr)


@sgd_momentum_.register_fake
def _(param, momentum_buf, grad, lr, momentum, grad_scale=1.0):
    return None


class Conv2dNHWC(nn.Module):
    """nn.Conv2d(ci, co, k, padding=dilation*(k//2), dilation=dilation) [+ ReLU] on NHWC 16-bit activations, run
    by the native MFMA kernels (``torch.ops.cannet.conv2d_nhwc``).  Parameters are fp32 in the PyTorch layout, so
    ``state_dict`` is interchangeable with nn.Conv2d's."""

    def __init__(self, in_channels: int, out_channels: int, kernel_size: int = 3, dilation: int = 1,
                 bias: bool = True, relu: bool = True):
        super().__init__()
        if kernel_size not in (1, 3):
            raise ValueError("kernel_size must be 1 or 3")
        self.dilation, self.relu = dilation, relu
        self.weight = nn.Parameter(torch.empty(out_channels, in_channels, kernel_size, kernel_size))
        self.bias = nn.Parameter(torch.zeros(out_channels)) if bias else None
        nn.init.normal_(self.weight, std=0.01)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return torch.ops.cannet.conv2d_nhwc(x, self.weight, self.bias, self.dilation, self.relu)


class ReluMaxPool2x2(nn.Module):
    """ReLU followed by a 2x2 / stride-2 max-pool of an NHWC map, as one op (``torch.ops.cannet.relu_max_pool2x2``);
    after a ReLU (Conv2dNHWC(relu=True)) it is the plain max-pool."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return torch.ops.cannet.relu_max_pool2x2(x)[0]
