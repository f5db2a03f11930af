"""fp32 training on the native MFMA kernels: split-bf16 ("bf16x3") convolutions.

The reference trains in fp32 (train.py:126, no autocast).  gfx950's fp32 matrix rate is a small fraction of
its bf16 rate, so an fp32 operand is split into two bf16 parts, x = hi + lo (hi = bf16(x), lo = bf16(x - hi):
16 significant bits together), and every conv GEMM is computed as

    x * w  ~=  hi(x) hi(w) + hi(x) lo(w) + lo(x) hi(w)          (the lo*lo term is below fp32 rounding of the sum)

with fp32 accumulation, in ONE launch of the bf16 kernels:

* forward / data gradient: the three products are concatenated along K — the activation becomes
  [hi | hi | lo] (3*Cin channels, csrc/elementwise.hip split_x3 mode 0), the packed weight [W_hi | W_lo | W_hi]
  — and the LDS-DMA conv kernel stores its fp32 accumulator (EPI_F32) instead of a 16-bit rounding;
* weight gradient: the reduction runs over pixels, so the parts are stacked along M (batch 3N:
  dY = [hi; hi; lo], X = [hi; lo; hi], split_x3 mode 1) into the existing weight-gradient kernels, which
  accumulate and reduce in fp32; the bias gradient is an fp32 column sum of dY (bias_rows_reduce).

Relative error of a product term is ~2^-16..2^-17 (vs fp32's 2^-24 and TF32's 2^-11): the operands carry about
16 significant bits (lo is itself rounded to bf16) and lo*lo is dropped, so this is APPROXIMATELY fp32 — gradients
can differ from true fp32 by ~1e-5 relative — not the reference's fp32 numerics bit for bit (parity unpinned).  Everything between the
convolutions (ReLU, max-pool, the context module's pooling / upsampling / sigmoid weighting, the loss) stays
fp32 in ATen, on channels-last (NHWC) tensors so the conv operands need no layout copies.

``conv2d_x3`` is the autograd op; ``cannet_forward_fp32`` runs CANNet with it (model backend
``"hip_fp32"``; engine/trainer.Fp32Stepper is the step).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

from . import _ext
from .conv import BF16, pack_weight_dgrad, pack_weight_fwd

EPI_F32 = 7
HI_HI_LO = 0b100       # block pattern: bit b set -> block b is the lo part
HI_LO_HI = 0b010


def split_x3(x: torch.Tensor, mode: int, pattern: int, stride: Optional[int] = None) -> torch.Tensor:
    """fp32 NHWC [N,H,W,C] -> bf16 split operand (see module doc).  mode 0: [N,H,W,stride] (>= 3C, zero padded);
    mode 1: [3N,H,W,stride] (>= C, zero padded)."""
    C = _ext.require()
    if x.dtype != torch.float32 or not x.is_cuda or not x.is_contiguous() or x.dim() != 4:
        raise ValueError("split_x3 takes a contiguous fp32 NHWC GPU tensor")
    n, h, w, c = x.shape
    if mode == 0:
        stride = stride or 3 * c
        out = torch.empty(n, h, w, stride, dtype=BF16, device=x.device)
    else:
        stride = stride or c
        out = torch.empty(3 * n, h, w, stride, dtype=BF16, device=x.device)
    C.split_x3(x.data_ptr(), out.data_ptr(), n * h * w, c, stride, mode, pattern, _ext.stream_ptr(x.device))
    return out


def split_weight(w: torch.Tensor):
    hi = w.detach().to(BF16).float()
    lo = (w.detach().float() - hi).to(BF16).float()
    return hi, lo


def colsum(dy: torch.Tensor) -> torch.Tensor:
    """fp32 [M, C] (C % 64 == 0) -> [C]: the bias gradient, two deterministic row-block passes."""
    C = _ext.require()
    m, c = dy.shape
    st = _ext.stream_ptr(dy.device)
    part = torch.empty(512, c, dtype=torch.float32, device=dy.device)
    g = C.bias_rows_reduce(dy.data_ptr(), part.data_ptr(), m, c, 512, st)
    out = torch.empty(1, c, dtype=torch.float32, device=dy.device)
    C.bias_rows_reduce(part.data_ptr(), out.data_ptr(), g, c, 1, st)
    return out[0]


def _pad_to(n: int, q: int = 64) -> int:
    return -(-n // q) * q


def _as_pixels(t: torch.Tensor) -> torch.Tensor:
    """1x1 conv operands with a spatial side < 2 (the context module's 1x1 / 2x2 cells): the LDS-DMA kernels
    take H, W >= 2, and a 1x1 conv does not care about the pixel layout, so lay the M pixels out as a zero-padded
    [1, 2, P, C] map."""
    n, h, w, c = t.shape
    m = n * h * w
    p = max(2, -(-m // 2))
    out = torch.zeros(1, 2, p, c, dtype=t.dtype, device=t.device)
    out.view(-1, c)[:m] = t.reshape(m, c)
    return out


def _from_pixels(t: torch.Tensor, shape) -> torch.Tensor:
    n, h, w, _ = shape
    c = t.shape[-1]
    return t.reshape(-1, c)[:n * h * w].reshape(n, h, w, c)


class _ConvX3(torch.autograd.Function):
    """y[N,H,W,Co] fp32 = conv(x[N,H,W,Ci] fp32, weight[Co,Ci,k,k]) + bias, stride 1, 'same' padding.
    Ci is padded to a multiple of 64 for the first layer (Ci = 3: the 9 split channels of [hi|hi|lo] fit one
    64-channel block); Co is padded to 64 for the 1-channel head."""

    @staticmethod
    def forward(ctx, x, weight, bias, dil: int):
        co, _, k, _ = weight.shape
        flat = k == 1 and min(x.shape[1], x.shape[2]) < 2
        ctx.flat, ctx.xshape = flat, tuple(x.shape)
        if flat:
            x = _as_pixels(x.detach())
        y = _ConvX3._fwd(ctx, x, weight, bias, dil)
        return _from_pixels(y, ctx.xshape[:3] + (co,)).contiguous() if flat else y

    @staticmethod
    def _fwd(ctx, x, weight, bias, dil: int):
        C = _ext.require()
        n, h, w, ci = x.shape
        co, _, k, _ = weight.shape
        cop = _pad_to(co)
        small = 3 * ci < 64 and ci % 64 != 0            # first layer: the whole split operand in 64 channels
        if not small and ci % 64:
            raise ValueError(f"Cin={ci} must be a multiple of 64 (or 3 * Cin <= 64)")
        whi, wlo = split_weight(weight)
        if small:
            w3 = torch.zeros(cop, 64, k, k, device=x.device)
            w3[:co, 0:ci], w3[:co, ci:2 * ci], w3[:co, 2 * ci:3 * ci] = whi, wlo, whi
            x3 = split_x3(x, 0, HI_HI_LO, stride=64)
        else:
            w3 = torch.zeros(cop, 3 * ci, k, k, device=x.device)
            w3[:co] = torch.cat([whi, wlo, whi], dim=1)
            x3 = split_x3(x, 0, HI_HI_LO)
        b = None
        if bias is not None:
            b = torch.zeros(cop, device=x.device)
            b[:co] = bias.detach().float()
        y = torch.empty(n, h, w, cop, dtype=torch.float32, device=x.device)
        # the fp32 output buffer goes through the kernel's 16-bit `y` argument (EPI_F32 reinterprets it)
        C.conv_igemm(x3.data_ptr(), pack_weight_fwd(w3).data_ptr(), b.data_ptr() if b is not None else 0, 0,
                     y.data_ptr(), n, h, w, x3.shape[-1], cop, k, dil, EPI_F32, 0, 0, 0, _ext.stream_ptr(x.device),
                     0, 0)
        ctx.save_for_backward(x, weight)
        ctx.dil, ctx.small, ctx.has_bias = dil, small, bias is not None
        return y if cop == co else y[..., :co].contiguous()

    @staticmethod
    def backward(ctx, dy):
        C = _ext.require()
        x, weight = ctx.saved_tensors
        n, h, w, ci = x.shape
        co, _, k, _ = weight.shape
        cop = _pad_to(co)
        dy = dy.contiguous().float()
        if ctx.flat:
            dy = _as_pixels(dy)
        if cop != co:
            dyp = torch.zeros(n, h, w, cop, dtype=torch.float32, device=dy.device)
            dyp[..., :co] = dy
            dy = dyp
        st = _ext.stream_ptr(dy.device)
        dx = dw = db = None
        whi, wlo = split_weight(weight)
        if ctx.needs_input_grad[0]:
            if ctx.small:
                raise RuntimeError("no data gradient for the first (3-channel) layer")
            # dX = conv_transpose(dY, W): K-concatenated [dY_hi | dY_hi | dY_lo] x [W_hi; W_lo; W_hi]
            w3 = torch.zeros(3 * cop, ci, k, k, device=dy.device)
            w3[0:co], w3[cop:cop + co], w3[2 * cop:2 * cop + co] = whi, wlo, whi
            dy3 = split_x3(dy, 0, HI_HI_LO)
            dx = torch.empty(n, h, w, ci, dtype=torch.float32, device=dy.device)
            C.conv_igemm(dy3.data_ptr(), pack_weight_dgrad(w3).data_ptr(), 0, 0, dx.data_ptr(), n, h, w, 3 * cop, ci,
                         k, ctx.dil, EPI_F32, 0, 0, 0, st, 0, 0)
        if ctx.needs_input_grad[1]:
            from .conv import conv_wgrad
            cis = 64 if ctx.small else ci
            dys = split_x3(dy, 1, HI_HI_LO)                       # [3N,H,W,Cop]
            xs = split_x3(x, 1, HI_LO_HI, stride=cis)             # [3N,H,W,Cis]
            dwf = torch.empty(cop, cis, k, k, dtype=torch.float32, device=dy.device)
            conv_wgrad(dys, xs, dwf, None, ksize=k, dil=ctx.dil)
            dw = dwf[:co, :ci].contiguous()
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = colsum(dy.view(-1, cop))[:co].contiguous()
        if ctx.flat and dx is not None:
            dx = _from_pixels(dx, ctx.xshape).contiguous()
        return dx, dw, db, None


def conv2d_x3(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor], dil: int = 1) -> torch.Tensor:
    """NHWC fp32 conv (3x3 'same' with dilation, or 1x1) on the bf16 MFMA kernels, split-bf16 accurate."""
    return _ConvX3.apply(x, weight, bias, dil)


def _nchw(t):      # NHWC tensor -> NCHW view (channels-last strides) for ATen's spatial ops
    return t.permute(0, 3, 1, 2)


def _nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def _run_seq(seq, y):
    for m in seq:
        if isinstance(m, torch.nn.Conv2d):
            y = conv2d_x3(y, m.weight, m.bias, m.dilation[0])
        elif isinstance(m, torch.nn.ReLU):
            y = F.relu(y)
        elif isinstance(m, torch.nn.MaxPool2d):
            y = _nhwc(F.max_pool2d(_nchw(y), 2, 2))
        else:
            raise TypeError(f"fp32 path: unsupported layer {type(m).__name__}")
    return y


_AXIS_CACHE = {}


def _pool_matrix(S: int, L: int, device) -> torch.Tensor:
    """[S, L] adaptive-average-pool weights (ATen bins: floor(i*L/S) .. ceil((i+1)*L/S))."""
    key = ("pool", S, L, str(device))
    if key not in _AXIS_CACHE:
        m = torch.zeros(S, L, dtype=torch.float64)
        for i in range(S):
            st, en = (i * L) // S, -(-((i + 1) * L) // S)
            m[i, st:en] = 1.0 / (en - st)
        _AXIS_CACHE[key] = m.float().to(device)
    return _AXIS_CACHE[key]


def _interp_matrix(S: int, L: int, device) -> torch.Tensor:
    """[L, S] bilinear (align_corners=True) weights of output position x over the S input cells."""
    key = ("up", S, L, str(device))
    if key not in _AXIS_CACHE:
        m = torch.zeros(L, S, dtype=torch.float64)
        scale = (S - 1) / (L - 1) if L > 1 else 0.0
        for x in range(L):
            src = scale * x
            x0 = int(src)
            x1 = x0 + (1 if x0 < S - 1 else 0)
            lam = src - x0
            m[x, x0] += 1.0 - lam
            m[x, x1] += lam
        _AXIS_CACHE[key] = m.float().to(device)
    return _AXIS_CACHE[key]


def _adaptive_pool_nhwc(x: torch.Tensor, S: int) -> torch.Tensor:
    """adaptive_avg_pool2d on NHWC as two fp32 GEMMs (their backward is GEMMs too); ATen's NHWC kernels for a
    96 x 128 -> 1..6 pooling and its bilinear backward took 17 ms of the fp32 step."""
    n, h, w, c = x.shape
    t = torch.matmul(_pool_matrix(S, w, x.device), x)                       # [n, h, S, c]
    return torch.matmul(_pool_matrix(S, h, x.device), t.reshape(n, h, S * c)).reshape(n, S, S, c)


def _upsample_nhwc(a: torch.Tensor, h: int, w: int) -> torch.Tensor:
    """bilinear upsample (align_corners=True) of NHWC [n, S, S, c] to [n, h, w, c] as two fp32 GEMMs."""
    n, S, _, c = a.shape
    t = torch.matmul(_interp_matrix(S, w, a.device), a)                     # [n, S, w, c]
    return torch.matmul(_interp_matrix(S, h, a.device), t.reshape(n, S, w * c)).reshape(n, h, w, c)


def cannet_forward_fp32(model, img: torch.Tensor) -> torch.Tensor:
    """CANNet forward (model/CANNet.py:39-91 math) with every convolution on conv2d_x3; img [N,3,H,W] fp32 ->
    density [N,1,H/8,W/8] fp32."""
    from ..models.cannet import CONTEXT_SCALES, FUSE_EPS
    x = _nhwc(img.float())
    fv = _run_seq(model.frontend, x)                             # [N,h,w,512]
    n, h, w, c = fv.shape
    num = den = None
    for s in CONTEXT_SCALES:
        c1, c2 = getattr(model, f"conv{s}_1"), getattr(model, f"conv{s}_2")
        ave = conv2d_x3(_adaptive_pool_nhwc(fv, s), c1.weight, None)
        up = _upsample_nhwc(ave, h, w)
        wgt = torch.sigmoid(conv2d_x3(up - fv, c2.weight, None))
        num = wgt * up if num is None else num + wgt * up
        den = wgt if den is None else den + wgt
    fi = num / (den + FUSE_EPS)
    y = _run_seq(model._modules["backend"], torch.cat((fv, fi), dim=-1))
    et = conv2d_x3(y, model.output_layer.weight, model.output_layer.bias)
    return _nchw(et).contiguous()
