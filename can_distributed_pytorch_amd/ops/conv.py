"""Python front-end of the gfx950 implicit-GEMM convolution kernels.

Replaces the nn.Conv2d calls of the reference (model/CANNet.py:14-17,114-115)
with NHWC 16-bit MFMA kernels (csrc/conv_igemm.hip forward + data-gradient,
csrc/conv_wgrad.hip weight-gradient).  All shape / dtype / layout checks are
done here, on the host, before anything is launched.

Element type: bf16 (default) or fp16, taken from the activation tensor; every
16-bit operand of one call must share it (v_mfma_f32_16x16x32_{bf16,f16},
fp32 accumulation either way).

Weight layouts (packed from the fp32 master weights [Co][Ci][kh][kw]):
  * forward  : [Co][kh][kw][Ci]        (K = 9*Ci contiguous per output channel)
  * dgrad    : [Ci][kh'][kw'][Co] with kh' = 2-kh, kw' = 2-kw (flipped)
  * first    : [64][64], k = tap*4 + c (c < 3), zero padded (Cin=3 layer)
"""
from __future__ import annotations

from typing import Optional

import torch

from . import _ext
from . import dispatch

EPI_BIAS_RELU, EPI_MASK, EPI_NONE, EPI_BIAS, EPI_SIGMOID, EPI_POOLBWD = 0, 1, 2, 3, 4, 5
BF16 = torch.bfloat16
ACT_DTYPES = {torch.bfloat16: 0, torch.float16: 1}   # -> kernel element-type code (csrc/common.h DT_*)


def dt_code(dtype: torch.dtype) -> int:
    if dtype not in ACT_DTYPES:
        raise ValueError(f"native kernels take bf16 or fp16 activations, got {dtype}")
    return ACT_DTYPES[dtype]


def pack_weight_fwd(w: torch.Tensor, dtype: torch.dtype = BF16) -> torch.Tensor:
    co = w.shape[0]
    return w.detach().permute(0, 2, 3, 1).reshape(co, -1).to(dtype).contiguous()


def pack_weight_dgrad(w: torch.Tensor, dtype: torch.dtype = BF16) -> torch.Tensor:
    ci = w.shape[1]
    return w.detach().flip(2, 3).permute(1, 2, 3, 0).reshape(ci, -1).to(dtype).contiguous()


def pack_weight_first(w: torch.Tensor, dtype: torch.dtype = BF16) -> torch.Tensor:
    co, ci, kh, kw = w.shape
    assert ci == 3 and kh == 3 and kw == 3
    wp = torch.zeros(co, 64, dtype=torch.float32, device=w.device)
    wp[:, :36].view(co, 9, 4)[:, :, :3] = w.detach().float().permute(0, 2, 3, 1).reshape(co, 9, 3)
    return wp.to(dtype).contiguous()


def to_nhwc4(img: torch.Tensor, dtype: torch.dtype = BF16) -> torch.Tensor:
    """[N,3,H,W] float -> [N,H,W,4] 16-bit (channel 3 = 0): the first layer's input layout."""
    n, c, h, w = img.shape
    assert c == 3
    out = torch.zeros(n, h, w, 4, dtype=dtype, device=img.device)
    out[..., :3] = img.permute(0, 2, 3, 1)
    return out


# Largest element count one conv launch addresses in any operand: the kernels index pixels x channels with 32-bit
# offsets and read activations through 32-bit buffer resources (the v2 weight gradient needs M * Cout * 2 < 2^31).
# A batch beyond it runs as consecutive launches over image chunks (images are independent in every conv; weight
# gradients accumulate over the chunks with beta = 1), so batch size is bounded by HBM, not by the index width.
MAX_ELEMS_PER_LAUNCH = 1 << 30


def image_chunks(n: int, elems_per_image: int, limit: Optional[int] = None):
    """[(i0, i1)] image ranges whose operands stay within ``limit`` (default MAX_ELEMS_PER_LAUNCH) elements."""
    limit = limit or MAX_ELEMS_PER_LAUNCH
    if elems_per_image > limit:
        raise ValueError(f"one image needs {elems_per_image} elements per operand (> {limit}): too large for one launch")
    per = max(1, limit // elems_per_image)
    return [(i, min(n, i + per)) for i in range(0, n, per)]


def _check_act(x: torch.Tensor, name: str, c: Optional[int] = None, dtype: Optional[torch.dtype] = None):
    if not x.is_cuda:
        raise ValueError(f"{name} must be a GPU tensor")
    if x.dtype not in ACT_DTYPES:
        raise ValueError(f"{name} must be bf16 or fp16, got {x.dtype}")
    if dtype is not None and x.dtype != dtype:
        raise ValueError(f"{name} is {x.dtype}, the other operands are {dtype}")
    if not x.is_contiguous():
        raise ValueError(f"{name} must be contiguous NHWC")
    if c is not None and x.shape[-1] != c:
        raise ValueError(f"{name} has {x.shape[-1]} channels, expected {c}")


def conv_igemm(x: torch.Tensor, wpack: torch.Tensor, bias: Optional[torch.Tensor], *, ksize: int, dil: int = 1,
               epi: int = EPI_BIAS_RELU, mask: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
               first: bool = False, tile: int = 0, bias_part: Optional[torch.Tensor] = None):
    """y[N,H,W,Co] = epi(conv(x[N,H,W,Ci], W) ...), stride 1, 'same' padding = dil*(ksize//2).

    epi=EPI_POOLBWD: the conv result is d(maxpool output); ``mask`` is the pool's max-pool codes
    (int32 [N,H,W,Co/8], see ``maxpool_codes``) and the result is written as d(pool input) (ReLU mask of the
    pool input included) into [N,2H,2W,Co].

    bias_part (EPI_MASK / EPI_POOLBWD): fp32 [cap, Co] buffer; the epilogue writes the bias-gradient partials
    of its output into its first rows and (out, bias_part[:rows] or None) is returned instead of out."""
    C = _ext.require()
    if x.dim() != 4:
        raise ValueError("x must be [N,H,W,C]")
    n, h, w, ci = x.shape
    _check_act(x, "x")
    co, k = wpack.shape
    dt = x.dtype
    if wpack.dtype != dt or not wpack.is_contiguous():
        raise ValueError(f"wpack must be contiguous {dt}")
    if first:
        if ci != 4 or ksize != 3 or k != 64:
            raise ValueError("first-layer conv expects x[...,4], 3x3, packed weight [Co,64]")
    else:
        if ci % 64 != 0:
            raise ValueError(f"Cin={ci} must be a multiple of 64")
        if k != ksize * ksize * ci:
            raise ValueError(f"packed weight K={k} != {ksize}*{ksize}*{ci}")
    if co % 64 != 0:
        raise ValueError(f"Cout={co} must be a multiple of 64")
    if ksize not in (1, 3):
        raise ValueError("ksize must be 1 or 3")
    if epi in (EPI_BIAS_RELU, EPI_BIAS):
        if bias is None or bias.dtype != torch.float32 or bias.numel() != co or not bias.is_contiguous():
            raise ValueError("bias must be contiguous fp32 [Cout]")
    oshape = (n, 2 * h, 2 * w, co) if epi == EPI_POOLBWD else (n, h, w, co)
    if epi == EPI_MASK:
        if mask is None or tuple(mask.shape) != oshape:
            raise ValueError(f"mask must be {list(oshape)}")
        _check_act(mask, "mask", dtype=dt)
    if epi == EPI_POOLBWD:
        _check_codes(mask, (n, h, w, co))
        if first or tile not in (0, 21, 22, 23, 25, 27, 28, 29):
            raise ValueError("EPI_POOLBWD runs on the LDS-DMA kernels only")
    if out is None:
        out = torch.empty(*oshape, dtype=dt, device=x.device)
    else:
        if tuple(out.shape) != oshape:
            raise ValueError("out has the wrong shape")
        _check_act(out, "out", dtype=dt)
    bp_ptr, bp_cap = 0, 0
    if bias_part is not None:
        if epi not in (EPI_MASK, EPI_POOLBWD):
            raise ValueError("bias partials come from data-gradient epilogues (EPI_MASK / EPI_POOLBWD)")
        if bias_part.dtype != torch.float32 or not bias_part.is_contiguous() or bias_part.dim() != 2 or \
                bias_part.shape[1] != co:
            raise ValueError(f"bias_part must be a contiguous fp32 [rows, {co}] tensor")
        bp_ptr, bp_cap = bias_part.data_ptr(), bias_part.shape[0]
    chunks = image_chunks(n, h * w * max(ci, co) * (4 if epi == EPI_POOLBWD else 1))
    if len(chunks) > 1:
        # consecutive launches over image chunks; bias partial rows are written back to back
        r0, none_rows = 0, False
        for i0, i1 in chunks:
            res = conv_igemm(x[i0:i1], wpack, bias, ksize=ksize, dil=dil, epi=epi,
                             mask=mask[i0:i1] if mask is not None else None, out=out[i0:i1], first=first, tile=tile,
                             bias_part=bias_part[r0:] if bias_part is not None else None)
            if bias_part is not None:
                part = res[1]
                if part is None:
                    none_rows = True
                else:
                    r0 += part.shape[0]
        if bias_part is not None:
            return out, (None if none_rows or r0 == 0 else bias_part[:r0])
        return out
    rows = C.conv_igemm(x.data_ptr(), wpack.data_ptr(), bias.data_ptr() if bias is not None else 0,
                        mask.data_ptr() if mask is not None else 0, out.data_ptr(), n, h, w, ci, co, ksize, dil,
                        epi, int(first), tile, dt_code(dt), _ext.stream_ptr(x.device), bp_ptr, bp_cap)
    if bias_part is not None:
        return out, (bias_part[:rows] if rows > 0 else None)
    return out


def conv_igemm_batched(x: torch.Tensor, wpack: torch.Tensor, *, ksize: int, epi: int, dil: int = 1,
                       out: Optional[torch.Tensor] = None, tile: int = 0) -> torch.Tensor:
    """nb independent convs of one shape in one launch: x [nb,N,H,W,Ci], wpack [nb,Co,K] -> [nb,N,H,W,Co];
    epi EPI_NONE or EPI_SIGMOID (no bias).  Same kernel and tile config as nb conv_igemm calls (bitwise)."""
    C = _ext.require()
    if x.dim() != 5 or wpack.dim() != 3 or x.shape[0] != wpack.shape[0]:
        raise ValueError("x must be [nb,N,H,W,C] and wpack [nb,Co,K] with the same nb")
    if epi not in (EPI_NONE, EPI_SIGMOID):
        raise ValueError("batched convs take EPI_NONE or EPI_SIGMOID")
    nb, n, h, w, ci = x.shape
    _check_act(x, "x")
    _, co, k = wpack.shape
    if wpack.dtype != x.dtype or not wpack.is_contiguous():
        raise ValueError(f"wpack must be contiguous {x.dtype}")
    if ci % 64 or co % 64 or k != ksize * ksize * ci or ksize not in (1, 3):
        raise ValueError("Cin / Cout must be multiples of 64 and K = ksize^2 * Cin")
    if h < 2 or w < 2:
        raise ValueError("H and W must be >= 2")
    oshape = (nb, n, h, w, co)
    if out is None:
        out = torch.empty(*oshape, dtype=x.dtype, device=x.device)
    elif tuple(out.shape) != oshape:
        raise ValueError("out has the wrong shape")
    else:
        _check_act(out, "out", dtype=x.dtype)
    C.conv_igemm_batched(x.data_ptr(), wpack.data_ptr(), 0, out.data_ptr(), nb, n * h * w * ci, co * k,
                         n * h * w * co, n, h, w, ci, co, ksize, dil, epi, tile, dt_code(x.dtype),
                         _ext.stream_ptr(x.device))
    return out


BIAS_ROWS = 512     # bias partial rows the weight-gradient reduce kernels take directly (kBiasParts)


def bias_part_capacity(n: int, h: int, w: int) -> int:
    """Rows a data-gradient epilogue may write for an output of n x h x w pixels (pooled resolution for
    EPI_POOLBWD): LDS-DMA kernels one row per (pixel tile, wave slot) = ceil(M / 64) at most, the halo
    kernel one per (4 x 64 tile, wave slot), the row ring one per (per-image 2- or 4-row x 128-column tile, wave
    slot) (ragged tiles included)."""
    cb = -(-w // 128)
    return max(-(-n * h * w // 64) + 64, n * (-(-h // 4)) * (-(-w // 64)) * 8,
               n * (-(-h // 2)) * cb * 4, n * (-(-h // 4)) * cb * 8)


def conv_dgrad_with_bias(dy: torch.Tensor, wpack: torch.Tensor, *, ksize: int, dil: int = 1, epi: int = EPI_MASK,
                         mask: torch.Tensor, tile: int = 0, out: Optional[torch.Tensor] = None):
    """Data gradient (EPI_MASK / EPI_POOLBWD) whose epilogue also sums the bias gradient of the gradient it
    writes (the next layer's dY): returns (dX, partials [rows, Cin] fp32 or None when the kernel path does not
    produce them).  conv_wgrad(bias_partials=...) reduces them into db instead of re-reading dY."""
    n, h, w, _ = dy.shape
    co = wpack.shape[0]
    bp = torch.empty(bias_part_capacity(n, h, w), co, dtype=torch.float32, device=dy.device)
    # long partial lists are folded by conv_wgrad on the weight-gradient stream after its GEMM (folded here, on the
    # producer's critical-path stream, the short launch waited 85-345 us for CUs, profiles/r3/ab_bias_prereduce.txt)
    return conv_igemm(dy, wpack, None, ksize=ksize, dil=dil, epi=epi, mask=mask, tile=tile, bias_part=bp, out=out)


def _check_codes(codes: Optional[torch.Tensor], pooled_shape) -> None:
    n, h, w, c = pooled_shape
    if codes is None or codes.dtype != torch.int32 or not codes.is_cuda or not codes.is_contiguous() or \
            tuple(codes.shape) != (n, h, w, c // 8):
        raise ValueError(f"max-pool codes must be a contiguous int32 GPU tensor [{n},{h},{w},{c // 8}]")


def maxpool_codes(x: torch.Tensor):
    """2x2/s2 max-pool of x [N,H,W,C] -> (pooled [N,H/2,W/2,C], codes int32 [N,H/2,W/2,C/8]).

    codes: per pooled pixel and channel a 4-bit one-hot of the FIRST max of its window (ATen scan order
    (0,0),(0,1),(1,0),(1,1) = bits 0..3), 0 when that max is not > 0 (the ReLU mask of the pool input);
    channel c sits in word c // 8, nibble c % 8.  The backward (``maxpool_bwd_codes``, EPI_POOLBWD) needs
    nothing else, so the pool input need not be kept."""
    C = _ext.require()
    _check_act(x, "x")
    n, h, w, c = x.shape
    if h % 2 or w % 2 or c % 8:
        raise ValueError("max-pool needs even H, W and C % 8 == 0")
    y = torch.empty(n, h // 2, w // 2, c, dtype=x.dtype, device=x.device)
    codes = torch.empty(n, h // 2, w // 2, c // 8, dtype=torch.int32, device=x.device)
    C.maxpool_fwd(x.data_ptr(), y.data_ptr(), n, h, w, c, dt_code(x.dtype), _ext.stream_ptr(x.device),
                  codes.data_ptr())
    return y, codes


def maxpool_bwd_codes(codes: torch.Tensor, dy: torch.Tensor) -> torch.Tensor:
    """d(pool input) [N,2H,2W,C] from d(pool output) dy [N,H,W,C] and the pool's codes."""
    C = _ext.require()
    _check_act(dy, "dy")
    n, h, w, c = dy.shape
    _check_codes(codes, (n, h, w, c))
    dx = torch.empty(n, 2 * h, 2 * w, c, dtype=dy.dtype, device=dy.device)
    C.maxpool_bwd_codes(codes.data_ptr(), dy.data_ptr(), dx.data_ptr(), n, 2 * h, 2 * w, c, dt_code(dy.dtype),
                        _ext.stream_ptr(dy.device))
    return dx


class WgradWorkspace:
    """One fp32 scratch buffer for the split-pixel partial slabs, grown on demand
    (allocated outside any captured region, never inside a launch function)."""

    def __init__(self, device, target_blocks: int = 1024):
        self.device = torch.device(device)
        self.target_blocks = target_blocks
        self.buf = torch.empty(0, dtype=torch.float32, device=self.device)

    def plan(self, m: int, ci: int, co: int, ksize: int, first: bool, dil: int = 1, w: int = 0):
        """(slices, pixels per slice, kernel config, workspace floats) of one weight gradient; w (the map width, 0 =
        unknown) lets the planner pick the width-dependent tap-ring kernel."""
        C = _ext.require()
        s, mslice, cfg = C.wgrad_plan(m, ci, co, ksize, int(first), self.target_blocks, dil, w)
        ktot = 64 if first else ksize * ksize * ci
        need = s * ktot * co + max(s, 512) * co      # slabs + bias partials (v2 path: 512 column-sum parts)
        return s, mslice, cfg, need

    def reserve(self, need: int) -> torch.Tensor:
        if self.buf.numel() < need:
            self.buf = torch.empty(need, dtype=torch.float32, device=self.device)
        return self.buf


def conv_wgrad(dy: torch.Tensor, x: torch.Tensor, dw: torch.Tensor, db: Optional[torch.Tensor], *, ksize: int,
               dil: int = 1, first: bool = False, ws: Optional[WgradWorkspace] = None, beta: float = 0.0,
               scale: float = 1.0, dscale: Optional[torch.Tensor] = None,
               bias_partials: Optional[torch.Tensor] = None) -> None:
    """dw[Co,Ci,kh,kw] (fp32, PyTorch layout) = scale * [dscale[0]] * sum_m dY[m,co] Xcol[m,k] (+ beta*dw);
    db likewise.  dscale: optional fp32 device scalar read at run time (1 / loss scale of the fp16 step).
    bias_partials: [rows, Co] fp32 per-slice sums of dY written by the data-gradient epilogue that produced it
    (conv_dgrad_with_bias): db is reduced from them and dY is not re-read for the bias."""
    C = _ext.require()
    _check_act(dy, "dy")
    _check_act(x, "x", dtype=dy.dtype)
    if dscale is not None and (dscale.dtype != torch.float32 or not dscale.is_cuda):
        raise ValueError("dscale must be an fp32 GPU tensor")
    n, h, w, ci = x.shape
    co = dy.shape[-1]
    if tuple(dy.shape[:3]) != (n, h, w):
        raise ValueError("dy/x spatial mismatch")
    if first:
        if ci != 4 or ksize != 3 or tuple(dw.shape) != (co, 3, 3, 3):
            raise ValueError("first-layer wgrad expects x[...,4] and dw[Co,3,3,3]")
    else:
        if ci % 64 or co % 64:
            raise ValueError("Cin/Cout must be multiples of 64")
        if tuple(dw.shape) != (co, ci, ksize, ksize):
            raise ValueError(f"dw shape {tuple(dw.shape)} != {(co, ci, ksize, ksize)}")
    if dw.dtype != torch.float32 or not dw.is_contiguous():
        raise ValueError("dw must be contiguous fp32")
    if db is not None and (db.dtype != torch.float32 or db.numel() != co or not db.is_contiguous()):
        raise ValueError("db must be contiguous fp32 [Co]")
    ws = ws or WgradWorkspace(x.device)
    chunks = image_chunks(n, h * w * max(ci, co))
    if len(chunks) > 1:
        # dW (and db) accumulate over image chunks: the first launch applies beta, the others add (beta = 1); bias
        # partials of the whole dY (one list) are reduced by the first launch only
        for c, (i0, i1) in enumerate(chunks):
            use_bp = bias_partials is not None and db is not None
            conv_wgrad(dy[i0:i1], x[i0:i1], dw, db if (c == 0 or not use_bp) else None, ksize=ksize, dil=dil,
                       first=first, ws=ws, beta=beta if c == 0 else 1.0, scale=scale, dscale=dscale,
                       bias_partials=bias_partials if c == 0 else None)
        return
    s, mslice, cfg, need = ws.plan(n * h * w, ci, co, ksize, first, dil, w)
    buf = ws.reserve(need)
    ktot = 64 if first else ksize * ksize * ci
    wsb_ptr = buf.data_ptr() + 4 * s * ktot * co
    bx, brows = 0, 0
    if bias_partials is not None and db is not None:
        if bias_partials.dtype != torch.float32 or not bias_partials.is_contiguous() or bias_partials.dim() != 2 or \
                bias_partials.shape[1] != co or co > 1024:
            raise ValueError(f"bias_partials must be a contiguous fp32 [rows, {co}] tensor (Cout <= 1024)")
        bx, brows = bias_partials.data_ptr(), bias_partials.shape[0]
    C.conv_wgrad(dy.data_ptr(), x.data_ptr(), buf.data_ptr(), wsb_ptr, dw.data_ptr(),
                 db.data_ptr() if db is not None else 0, n, h, w, ci, co, ksize, dil, int(first), s, mslice, cfg,
                 float(beta), float(scale), dscale.data_ptr() if dscale is not None else 0, dt_code(dy.dtype),
                 _ext.stream_ptr(x.device), bx, brows)


def _ctx_wgrad_cus() -> int:
    """CUs the batched context 1x1 weight gradient is planned for.  It runs on the weight-gradient stream while the
    critical-path context backward (bilinear-transpose row / cell passes, ctx_bwd_final) runs on the compute stream;
    a grid of one 512-thread, 256-VGPR block per CU leaves those memory-bound kernels no CU until it drains.
    224 of 256 measured best (profiles/r2/ab_ctx_wgrad_cus.txt: 441.7-442.4 img/s vs 438.9-440.9 for 256,
    worse at 192 / 160); dispatch ctx_wgrad_cus selects."""
    return dispatch.current().ctx_wgrad_cus


def wgrad_1x1_batched_plan(m: int, nb: int, ci: int, co: int, ncu: int = 0):
    """(S, mslice, workspace floats) of the batched 1x1 weight gradient: one round of 256x256 tiles over ncu CUs
    (0: ``_ctx_wgrad_cus()``)."""
    ncu = ncu or _ctx_wgrad_cus()
    ntile = (co // 256) * (ci // 256) * nb
    s = max(1, ncu // ntile)
    mslice = -(-m // s)
    mslice = -(-mslice // 64) * 64
    s = -(-m // mslice)
    return s, mslice, nb * s * ci * co


def wgrad_1x1_batched_ok(dy: torch.Tensor, x: torch.Tensor, dws) -> bool:
    """Shapes / layouts the batched kernel takes: [nb,N,H,W,C] operands with W % 64 == 0, channels % 256 == 0,
    and the nb fp32 [Co,Ci,1,1] outputs laid out back to back (consecutive slots of the gradient arena)."""
    if dy.dim() != 5 or x.dim() != 5 or not (dy.is_contiguous() and x.is_contiguous()):
        return False
    nb, n, h, w, co = dy.shape
    ci = x.shape[-1]
    if tuple(x.shape[:4]) != (nb, n, h, w) or w % 64 or co % 256 or ci % 256 or (n * h * w) % 64:
        return False
    if n * h * w * max(ci, co) * 2 >= 2 ** 31:
        return False                       # 32-bit operand addressing: the per-item launches chunk instead
    if len(dws) != nb or any(d.dtype != torch.float32 or not d.is_contiguous() or tuple(d.shape) != (co, ci, 1, 1)
                             for d in dws):
        return False
    step = co * ci * 4
    return all(d.data_ptr() == dws[0].data_ptr() + i * step for i, d in enumerate(dws))


def conv_wgrad_1x1_batched(dy: torch.Tensor, x: torch.Tensor, dws, *, ws: "WgradWorkspace", beta: float = 0.0,
                           scale: float = 1.0, dscale: Optional[torch.Tensor] = None) -> None:
    """dws[b][co,ci,0,0] = scale * [dscale] * sum_m dy[b,m,co] x[b,m,ci]  for b < nb, in ONE GEMM launch
    (+ nb deterministic slab reductions).  Caller checks wgrad_1x1_batched_ok first."""
    C = _ext.require()
    _check_act(dy, "dy")
    _check_act(x, "x", dtype=dy.dtype)
    if not wgrad_1x1_batched_ok(dy, x, dws):
        raise ValueError("batched 1x1 wgrad: unsupported shapes / output layout")
    nb, n, h, w, co = dy.shape
    ci = x.shape[-1]
    m = n * h * w
    s, mslice, need = wgrad_1x1_batched_plan(m, nb, ci, co)
    buf = ws.reserve(need)
    C.conv_wgrad_1x1_batched(dy.data_ptr(), x.data_ptr(), buf.data_ptr(), dws[0].data_ptr(), m, w, ci, co, nb,
                             m * co, m * ci, co * ci, s, mslice, float(beta), float(scale),
                             dscale.data_ptr() if dscale is not None else 0, dt_code(dy.dtype),
                             _ext.stream_ptr(x.device))


def conv_pool_fwd_ok(x: torch.Tensor, cout: int, ksize: int, tile: int = 0) -> bool:
    """Whether conv_pool_fwd covers this layer: H even and W a multiple of half the kernel's pixel tile."""
    n, h, w, ci = x.shape
    if ci % 64 or cout % 64 or h % 2 or h < 2 or w < 2:
        return False
    if ci == 64 and cout == 64 and ksize == 3 and tile == 0 and h % 4:
        return False                       # conv1_2's halo kernel pools whole 4-row tiles
    tp = _ext.require().conv_pool_tp(ci, cout, ksize, tile)
    return tp > 0 and w % (tp // 2) == 0


def conv_pool_fwd(x: torch.Tensor, wpack: torch.Tensor, bias: torch.Tensor, *, ksize: int, dil: int = 1,
                  out: Optional[torch.Tensor] = None, pooled: Optional[torch.Tensor] = None, tile: int = 0,
                  keep_full: bool = True, codes: bool = False):
    """relu(conv(x, W) + b) -> (y [N,H,W,Co] or None, maxpool2x2(y) [N,H/2,W/2,Co], codes or None) in one kernel:
    the pool runs in the conv epilogue on the rounded outputs, so the tensors equal conv_igemm(EPI_BIAS_RELU) +
    maxpool_codes bitwise.  keep_full=False skips the full-resolution store (the training step keeps only the
    pooled map and the max-pool codes its backward needs)."""
    C = _ext.require()
    _check_act(x, "x")
    n, h, w, ci = x.shape
    co, k = wpack.shape
    dt = x.dtype
    if wpack.dtype != dt or not wpack.is_contiguous() or k != ksize * ksize * ci:
        raise ValueError("wpack must be the contiguous packed forward weight of this layer")
    if bias is None or bias.dtype != torch.float32 or bias.numel() != co or not bias.is_contiguous():
        raise ValueError("bias must be contiguous fp32 [Cout]")
    if not conv_pool_fwd_ok(x, co, ksize, tile):
        raise ValueError(f"fused pool needs H even and W a multiple of the tile half-width ({list(x.shape)})")
    if not keep_full and out is not None:
        raise ValueError("out given with keep_full=False")
    for t, shp, name in ((out, (n, h, w, co), "out"), (pooled, (n, h // 2, w // 2, co), "pooled")):
        if t is not None:
            if tuple(t.shape) != shp:
                raise ValueError(f"{name} must be {list(shp)}")
            _check_act(t, name, dtype=dt)
    if out is None and keep_full:
        out = torch.empty(n, h, w, co, dtype=dt, device=x.device)
    if pooled is None:
        pooled = torch.empty(n, h // 2, w // 2, co, dtype=dt, device=x.device)
    cd = torch.empty(n, h // 2, w // 2, co // 8, dtype=torch.int32, device=x.device) if codes else None
    chunks = image_chunks(n, h * w * max(ci, co))
    if len(chunks) > 1:
        for i0, i1 in chunks:
            xs = x[i0:i1]
            C.conv_pool_fwd(xs.data_ptr(), wpack.data_ptr(), bias.data_ptr(),
                            out[i0:i1].data_ptr() if out is not None else 0, pooled[i0:i1].data_ptr(),
                            cd[i0:i1].data_ptr() if cd is not None else 0, i1 - i0, h, w, ci, co, ksize, dil, tile,
                            dt_code(dt), _ext.stream_ptr(x.device))
        return out, pooled, cd
    C.conv_pool_fwd(x.data_ptr(), wpack.data_ptr(), bias.data_ptr(), out.data_ptr() if out is not None else 0,
                    pooled.data_ptr(), cd.data_ptr() if cd is not None else 0, n, h, w, ci, co, ksize, dil, tile,
                    dt_code(dt), _ext.stream_ptr(x.device))
    return out, pooled, cd


def w1g_slab_cap(device) -> int:
    """Slab rows conv_dgrad_w1g may write: 2 per block of the one-block-per-CU ws64 grid."""
    return 2 * torch.cuda.get_device_properties(device).multi_processor_count


def conv_dgrad_w1g(dy: torch.Tensor, wpack: torch.Tensor, mask: torch.Tensor, img: torch.Tensor, dw1: torch.Tensor,
                   db1: torch.Tensor, *, slabs: torch.Tensor, bslabs: torch.Tensor, store_dx: bool = False,
                   beta: float = 0.0, scale: float = 1.0, dscale: Optional[torch.Tensor] = None):
    """conv1_2's data gradient with conv1_1's weight gradient fused into it (weight-stationary ws64 kernel).

    dX = conv(dy, flipped conv1_2 wpack) * (mask > 0) with mask = conv1_1's output; every produced 4 x 64 tile
    is multiplied on the MFMA with the matching image patches (img = NHWC4 network input) into per-block fp32
    partials, so conv1_1's weight gradient never re-reads dX from memory; one deterministic slab reduction
    writes dw1 [64,3,3,3] / db1 [64] (beta / scale / dscale as conv_wgrad).  dX (conv1_1's dY, never needed
    again) is returned only with store_dx.  slabs / bslabs: fp32 [w1g_slab_cap, 36*64] / [w1g_slab_cap, 64].
    """
    C = _ext.require()
    dt = dy.dtype
    n, h, w, c = dy.shape
    if c != 64 or tuple(mask.shape) != (n, h, w, 64) or tuple(img.shape) != (n, h, w, 4):
        raise ValueError(f"conv_dgrad_w1g: dy/mask [N,H,W,64], img [N,H,W,4]; got {tuple(dy.shape)}, "
                         f"{tuple(mask.shape)}, {tuple(img.shape)}")
    for t, nm in ((dy, "dy"), (mask, "mask"), (img, "img")):
        _check_act(t, nm, dtype=dt)
    if tuple(wpack.shape) != (64, 576) or wpack.dtype != dt or not wpack.is_contiguous():
        raise ValueError("wpack must be the packed [64, 9*64] conv1_2 data-gradient weight")
    if tuple(dw1.shape) != (64, 3, 3, 3) or tuple(db1.shape) != (64,):
        raise ValueError("dw1 / db1 must be conv1_1's [64,3,3,3] / [64] gradients")
    for t, nm in ((dw1, "dw1"), (db1, "db1"), (slabs, "slabs"), (bslabs, "bslabs")):
        if t.dtype != torch.float32 or not t.is_contiguous() or t.device != dy.device:
            raise ValueError(f"{nm} must be a contiguous fp32 tensor on {dy.device}")
    cap = slabs.shape[0]
    if slabs.dim() != 2 or slabs.shape[1] != 36 * 64 or tuple(bslabs.shape) != (cap, 64):
        raise ValueError("slabs / bslabs must be [cap, 36*64] / [cap, 64]")
    out = torch.empty_like(dy) if store_dx else None
    chunks = image_chunks(n, h * w * 64)
    if len(chunks) > 1:
        for c, (i0, i1) in enumerate(chunks):
            o = conv_dgrad_w1g(dy[i0:i1], wpack, mask[i0:i1], img[i0:i1], dw1, db1, slabs=slabs, bslabs=bslabs,
                               store_dx=store_dx, beta=beta if c == 0 else 1.0, scale=scale, dscale=dscale)
            if out is not None:
                out[i0:i1].copy_(o)
        return out
    st = _ext.stream_ptr(dy.device)
    s = C.conv_ws64_dgrad_w1g(dy.data_ptr(), wpack.data_ptr(), mask.data_ptr(), img.data_ptr(),
                              out.data_ptr() if out is not None else 0, slabs.data_ptr(), bslabs.data_ptr(), cap,
                              n, h, w, dt_code(dt), st)
    C.wgrad_reduce_first(slabs.data_ptr(), bslabs.data_ptr(), dw1.data_ptr(), db1.data_ptr(), s, float(beta),
                         float(scale), dscale.data_ptr() if dscale is not None else 0, st)
    return out


# ---------------------------------------------------------------------------------------------------------------------
# Linearised context module (csrc/conv_igemm.hip "Linearised context module", csrc/context.hip ctx_bwd_lin)
# ---------------------------------------------------------------------------------------------------------------------
def ctx_linear_ok(fv: torch.Tensor) -> bool:
    """The one-GEMM context module needs 256-channel tiles and a 256-pixel tile spanning <= 5 image rows (W >= 64)."""
    return fv.dim() == 4 and fv.shape[-1] % 256 == 0 and fv.shape[2] >= 64


def _check_cells(t: torch.Tensor, n: int, c: int, name: str):
    if t.dtype != torch.float32 or not t.is_contiguous() or tuple(t.shape) != (n, 50, c) or not t.is_cuda:
        raise ValueError(f"{name} must be a contiguous fp32 GPU tensor [{n}, 50, {c}]")


def conv_ctx_fwd(fv: torch.Tensor, wcat: torch.Tensor, t: torch.Tensor, u: torch.Tensor):
    """fv [N,h,w,C] -> (w maps [N,h,w,4C] (sigmoid of the four scales, columns 4c + si), cat [N,h,w,2C] = fv | fi).
    wcat: [4C, C] interleaved conv{S}_2 pack; t = W2 u, u = W1 ave: fp32 cell tables [N, 50, C]."""
    C = _ext.require()
    _check_act(fv, "fv")
    n, h, w, c = fv.shape
    if not ctx_linear_ok(fv):
        raise ValueError("conv_ctx_fwd needs C % 256 == 0 and w >= 64")
    if wcat.dtype != fv.dtype or not wcat.is_contiguous() or tuple(wcat.shape) != (4 * c, c):
        raise ValueError(f"wcat must be a contiguous {fv.dtype} [{4 * c}, {c}] pack")
    _check_cells(t, n, c, "t")
    _check_cells(u, n, c, "u")
    wts = torch.empty(n, h, w, 4 * c, dtype=fv.dtype, device=fv.device)
    cat = torch.empty(n, h, w, 2 * c, dtype=fv.dtype, device=fv.device)
    for i0, i1 in image_chunks(n, h * w * 4 * c):
        C.conv_ctx(1, fv[i0:i1].data_ptr(), wcat.data_ptr(), t[i0:i1].data_ptr(), u[i0:i1].data_ptr(),
                   fv[i0:i1].data_ptr(), cat[i0:i1].data_ptr(), wts[i0:i1].data_ptr(), i1 - i0, h, w, c,
                   dt_code(fv.dtype), _ext.stream_ptr(fv.device))
    return wts, cat


def ctx_bwd_lin(dcat: torch.Tensor, wts: torch.Tensor, u: torch.Tensor):
    """(dG [N,h,w,4C] = -dz, row partials [2, N, h, 12, C] of up^T(dz) and up^T(ds)) from dcat [N,h,w,2C]."""
    C = _ext.require()
    _check_act(wts, "wts")
    n, h, w, c4 = wts.shape
    c = c4 // 4
    _check_act(dcat, "dcat", dtype=wts.dtype)
    if tuple(dcat.shape) != (n, h, w, 2 * c) or c % 128:
        raise ValueError("dcat / wts shapes")
    _check_cells(u, n, c, "u")
    dg = torch.empty_like(wts)
    rowacc = torch.empty(2, n, h, 12, c, dtype=torch.float32, device=wts.device)
    C.ctx_bwd_lin(dcat.data_ptr(), wts.data_ptr(), u.data_ptr(), dg.data_ptr(), rowacc.data_ptr(), n, h, w, c,
                  dt_code(wts.dtype), _ext.stream_ptr(wts.device))
    return dg, rowacc


def conv_ctx_bwd(dg: torch.Tensor, wcat_dgr: torch.Tensor, dave: torch.Tensor, dcat: torch.Tensor,
                 fv: torch.Tensor) -> torch.Tensor:
    """dfv [N,h,w,C] = (dG . W2cat + dcat[..., :C] + pool^T(dave)) * (fv > 0)."""
    C = _ext.require()
    _check_act(fv, "fv")
    n, h, w, c = fv.shape
    if not ctx_linear_ok(fv):
        raise ValueError("conv_ctx_bwd needs C % 256 == 0 and w >= 64")
    _check_act(dg, "dg", 4 * c, dtype=fv.dtype)
    _check_act(dcat, "dcat", 2 * c, dtype=fv.dtype)
    if tuple(dg.shape[:3]) != (n, h, w) or tuple(dcat.shape[:3]) != (n, h, w):
        raise ValueError("dg / dcat spatial shape")
    if wcat_dgr.dtype != fv.dtype or not wcat_dgr.is_contiguous() or tuple(wcat_dgr.shape) != (c, 4 * c):
        raise ValueError(f"wcat_dgr must be a contiguous {fv.dtype} [{c}, {4 * c}] pack")
    _check_cells(dave, n, c, "dave")
    dfv = torch.empty_like(fv)
    for i0, i1 in image_chunks(n, h * w * 4 * c):
        C.conv_ctx(0, dg[i0:i1].data_ptr(), wcat_dgr.data_ptr(), dave[i0:i1].data_ptr(), 0, fv[i0:i1].data_ptr(),
                   dcat[i0:i1].data_ptr(), dfv[i0:i1].data_ptr(), i1 - i0, h, w, c, dt_code(fv.dtype),
                   _ext.stream_ptr(fv.device))
    return dfv
