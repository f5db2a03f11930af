"""Numerics of the MFMA implicit-GEMM conv kernels vs a plain fp32 PyTorch reference."""
import pytest
import torch
import torch.nn.functional as F
from numerics import check, check_out16

pytestmark = pytest.mark.gpu


def _ref(x_nhwc, w, b, dil, relu=True):
    x = x_nhwc.float().permute(0, 3, 1, 2)
    pad = dil * (w.shape[-1] // 2)
    y = F.conv2d(x, w.float(), b, padding=pad, dilation=dil)
    if relu:
        y = torch.relu(y)
    return y.permute(0, 2, 3, 1)


def _close(a, b):
    """Tight elementwise check (tests/numerics.py): 16-bit outputs to 8e-3 relative + 2e-3 rms, fp32 weight
    gradients to 1e-3 of (max + |value|)."""
    check(a, b)


@pytest.mark.parametrize("n,h,w,ci,co,k,dil,tile", [
    (2, 24, 40, 64, 64, 3, 1, 0), (1, 17, 33, 128, 128, 3, 1, 0), (2, 32, 32, 256, 512, 3, 2, 0),
    (1, 12, 16, 1024, 512, 3, 2, 0), (2, 16, 24, 512, 512, 1, 1, 0),
    (1, 20, 20, 128, 256, 3, 1, 1), (1, 20, 20, 128, 256, 3, 1, 2), (1, 20, 20, 128, 256, 3, 1, 3),
    (1, 20, 20, 128, 256, 3, 1, 4),
    (1, 20, 20, 128, 256, 3, 1, 11), (1, 20, 20, 128, 256, 3, 1, 12), (1, 20, 20, 128, 256, 3, 1, 13),
    (2, 9, 13, 64, 128, 3, 2, 0), (1, 7, 5, 512, 1024, 3, 2, 0), (3, 11, 17, 64, 64, 3, 1, 0),
    # v2 pipelined LDS-DMA kernel: every tile, 1x1 (nk = Cin/64), nk = 1, nk = 2, dilation 2, ragged M
    (1, 20, 20, 128, 256, 3, 1, 21), (1, 20, 20, 128, 256, 3, 1, 22), (1, 20, 20, 128, 256, 3, 1, 23),
    (2, 16, 24, 512, 512, 1, 1, 21), (1, 9, 13, 64, 256, 1, 1, 21), (1, 9, 13, 128, 128, 1, 1, 22),
    (2, 32, 32, 256, 512, 3, 2, 21), (3, 11, 17, 64, 64, 3, 1, 23), (2, 9, 13, 64, 128, 3, 2, 22),
    # halo-tiled Cin = 64 kernel: full tiles, ragged rows / columns, Cout 64 and 128
    (1, 4, 128, 64, 64, 3, 1, 31), (2, 10, 200, 64, 64, 3, 1, 31), (1, 9, 130, 64, 128, 3, 1, 31),
    (2, 3, 7, 64, 128, 3, 1, 31),
    # 128 x 512 tile (160 KB LDS)
    (1, 20, 40, 128, 128, 3, 1, 25), (2, 9, 13, 256, 128, 3, 2, 25), (1, 5, 7, 128, 384, 1, 1, 25),
])
def test_conv_fwd(n, h, w, ci, co, k, dil, tile):
    from can_distributed_pytorch_amd.ops import conv as C
    torch.manual_seed(0)
    dev = "cuda"
    x = torch.randn(n, h, w, ci, device=dev).to(torch.bfloat16)
    wt = (torch.randn(co, ci, k, k, device=dev) * 0.05).to(torch.bfloat16).float()
    b = torch.randn(co, device=dev)
    y = C.conv_igemm(x, C.pack_weight_fwd(wt), b, ksize=k, dil=dil, tile=tile)
    torch.cuda.synchronize()
    _close(y, _ref(x, wt, b, dil))


@pytest.mark.parametrize("pf", [0, 1])
@pytest.mark.parametrize("n,h,w,tile", [(2, 40, 56, 0), (1, 37, 150, 0), (2, 8, 256, 0), (2, 40, 56, 32)])
def test_conv_first_layer(n, h, w, tile, pf, dispatch_cfg):
    """tile 0 (auto) / 32: halo-tiled first-layer kernel (pf: persistent, prefetching the next tile's halo)."""
    from can_distributed_pytorch_amd.ops import conv as C
    dispatch_cfg(first_pf=pf)
    torch.manual_seed(1)
    img = torch.randn(n, 3, h, w, device="cuda")
    wt = (torch.randn(64, 3, 3, 3, device="cuda") * 0.2).to(torch.bfloat16).float()
    b = torch.randn(64, device="cuda")
    x4 = C.to_nhwc4(img)
    y = C.conv_igemm(x4, C.pack_weight_first(wt), b, ksize=3, first=True, tile=tile)
    ref = _ref(x4[..., :3].contiguous(), wt, b, 1)
    _close(y, ref)


@pytest.mark.parametrize("n,h,w,ci,co,dil,tile", [
    (2, 24, 40, 64, 128, 1, 0), (1, 16, 16, 512, 1024, 2, 0), (1, 9, 13, 64, 64, 1, 0),
    (1, 16, 16, 512, 1024, 2, 21), (2, 24, 40, 128, 64, 1, 22), (1, 9, 13, 64, 64, 1, 23),
    (2, 9, 140, 64, 64, 1, 31), (1, 12, 256, 128, 64, 1, 31)])
def test_conv_dgrad_mask(n, h, w, ci, co, dil, tile):
    """dX = conv_transpose(dY, W) * (mask > 0) via the same kernel with the flipped pack."""
    from can_distributed_pytorch_amd.ops import conv as C
    torch.manual_seed(2)
    dev = "cuda"
    wt = (torch.randn(co, ci, 3, 3, device=dev) * 0.05).to(torch.bfloat16).float()
    dy = torch.randn(n, h, w, co, device=dev).to(torch.bfloat16)
    mask = torch.randn(n, h, w, ci, device=dev).to(torch.bfloat16)
    dx = C.conv_igemm(dy, C.pack_weight_dgrad(wt), None, ksize=3, dil=dil, epi=C.EPI_MASK, mask=mask, tile=tile)
    xr = torch.zeros(n, ci, h, w, device=dev, requires_grad=True)
    y = F.conv2d(xr, wt, None, padding=dil, dilation=dil)
    (gx,) = torch.autograd.grad(y, xr, dy.float().permute(0, 3, 1, 2))
    ref = gx.permute(0, 2, 3, 1) * (mask.float() > 0)
    _close(dx, ref)


@pytest.mark.parametrize("n,h,w,ci,co,k,dil", [
    (2, 24, 40, 64, 64, 3, 1), (1, 17, 33, 128, 128, 3, 1), (2, 16, 16, 256, 512, 3, 2),
    (1, 12, 16, 128, 64, 3, 2), (2, 16, 24, 512, 512, 1, 1), (1, 40, 40, 64, 128, 3, 1),
    (1, 7, 9, 256, 256, 3, 2), (2, 13, 11, 64, 64, 3, 1), (1, 9, 10, 1024, 512, 3, 2), (1, 6, 8, 128, 256, 3, 1),
])
def test_conv_wgrad(n, h, w, ci, co, k, dil):
    from can_distributed_pytorch_amd.ops import conv as C
    torch.manual_seed(3)
    dev = "cuda"
    x = torch.randn(n, h, w, ci, device=dev).to(torch.bfloat16)
    dy = torch.randn(n, h, w, co, device=dev).to(torch.bfloat16)
    dw = torch.empty(co, ci, k, k, device=dev)
    db = torch.empty(co, device=dev)
    C.conv_wgrad(dy, x, dw, db, ksize=k, dil=dil)
    wr = torch.zeros(co, ci, k, k, device=dev, requires_grad=True)
    br = torch.zeros(co, device=dev, requires_grad=True)
    y = F.conv2d(x.float().permute(0, 3, 1, 2), wr, br, padding=dil * (k // 2), dilation=dil)
    gw, gb = torch.autograd.grad(y, (wr, br), dy.float().permute(0, 3, 1, 2))
    _close(dw, gw)
    _close(db, gb)


@pytest.mark.parametrize("n,h,w,ci,co,dil,bias", [
    (1, 6, 64, 256, 256, 1, True), (2, 5, 128, 512, 256, 2, True), (1, 3, 64, 1024, 512, 2, True),
    (3, 4, 64, 256, 512, 1, False), (1, 2, 64, 512, 512, 2, True),
    # ragged widths (W % 64 != 0, odd H): virtual 64-pixel stages per row, the padding pixels read zeros
    (2, 7, 100, 256, 256, 1, True), (1, 9, 120, 512, 256, 2, True), (3, 5, 30, 256, 512, 1, False),
    (1, 4, 135, 1024, 512, 2, True)])
def test_conv_wgrad_v2_row_aligned(n, h, w, ci, co, dil, bias, dispatch_cfg):
    """W % 64 == 0, Cin % 256 == 0 layers take the v2 pipelined wgrad (cfg 9) with bias column-sum blocks (with the
    tap-ring kernel off: it takes these layers by default)."""
    from can_distributed_pytorch_amd.ops import _ext
    from can_distributed_pytorch_amd.ops import conv as C
    dispatch_cfg(wgrad_tap=0)
    assert _ext.require().wgrad_plan(n * h * w, ci, co, 3, 0, 1024, dil, w)[2] == 9
    torch.manual_seed(6)
    x = torch.randn(n, h, w, ci, device="cuda").to(torch.bfloat16)
    dy = torch.randn(n, h, w, co, device="cuda").to(torch.bfloat16)
    dw = torch.empty(co, ci, 3, 3, device="cuda")
    db = torch.empty(co, device="cuda") if bias else None
    C.conv_wgrad(dy, x, dw, db, ksize=3, dil=dil)
    wr = torch.zeros(co, ci, 3, 3, device="cuda", requires_grad=True)
    br = torch.zeros(co, device="cuda", requires_grad=True)
    y = F.conv2d(x.float().permute(0, 3, 1, 2), wr, br, padding=dil, dilation=dil)
    gw, gb = torch.autograd.grad(y, (wr, br), dy.float().permute(0, 3, 1, 2))
    _close(dw, gw)
    if bias:
        _close(db, gb)


@pytest.mark.parametrize("n,h,w,ci,co,dil,dtype", [
    (1, 6, 64, 64, 128, 1, torch.bfloat16), (2, 7, 128, 128, 256, 1, torch.bfloat16),
    (1, 9, 120, 256, 128, 2, torch.bfloat16), (2, 5, 200, 64, 256, 2, torch.float16),
    (1, 12, 96, 512, 512, 2, torch.bfloat16), (3, 4, 64, 128, 128, 1, torch.float16),
    (1, 1, 64, 64, 128, 1, torch.bfloat16), (1, 3, 40, 64, 128, 2, torch.bfloat16),
    # 1024 -> 512: 64 tiles, 4 slices over 36 stages -> slices that span chains (several segments each)
    (2, 9, 128, 1024, 512, 2, torch.bfloat16),
    # Cout = 64: the 64-channel tile (4 waves, two blocks per CU, 2-stage DMA lead)
    (1, 6, 64, 64, 64, 1, torch.bfloat16), (2, 9, 120, 128, 64, 2, torch.bfloat16),
    (1, 5, 200, 64, 64, 1, torch.float16), (3, 16, 256, 64, 64, 1, torch.bfloat16)])
@pytest.mark.parametrize("adb", [0, 1])
def test_wgrad_tap_ring(n, h, w, ci, co, dil, dtype, adb, dispatch_cfg):
    """Tap-ring weight gradient (cfg 12: 128 output channels x 9 taps of a 64-channel input slice, input rows in an
    LDS ring walked down 64-column chains, one chain per row phase for dilation 2) == the fp32 reference: ragged
    widths (W % 64 != 0) and heights, single-row maps, slices spanning several chains, bias through the column-sum
    path."""
    from can_distributed_pytorch_amd.ops import _ext
    from can_distributed_pytorch_amd.ops import conv as C
    dispatch_cfg(wgrad_tap=3, wgrad_tap_adb=adb)
    assert _ext.require().wgrad_plan(n * h * w, ci, co, 3, 0, 1024, dil, w)[2] == 12
    torch.manual_seed(16)
    x = torch.randn(n, h, w, ci, device="cuda").to(dtype)
    dy = torch.randn(n, h, w, co, device="cuda").to(dtype)
    dw = torch.empty(co, ci, 3, 3, device="cuda")
    db = torch.empty(co, device="cuda")
    C.conv_wgrad(dy, x, dw, db, ksize=3, dil=dil)
    torch.cuda.synchronize()
    wr = torch.zeros(co, ci, 3, 3, device="cuda", requires_grad=True)
    br = torch.zeros(co, device="cuda", requires_grad=True)
    y = F.conv2d(x.float().permute(0, 3, 1, 2), wr, br, padding=dil, dilation=dil)
    gw, gb = torch.autograd.grad(y, (wr, br), dy.float().permute(0, 3, 1, 2))
    _close(dw, gw)
    _close(db, gb)


def test_conv_wgrad_first_layer():
    from can_distributed_pytorch_amd.ops import conv as C
    torch.manual_seed(4)
    img = torch.randn(2, 3, 40, 56, device="cuda")
    x4 = C.to_nhwc4(img)
    dy = torch.randn(2, 40, 56, 64, device="cuda").to(torch.bfloat16)
    dw = torch.empty(64, 3, 3, 3, device="cuda")
    db = torch.empty(64, device="cuda")
    C.conv_wgrad(dy, x4, dw, db, ksize=3, first=True)
    wr = torch.zeros(64, 3, 3, 3, device="cuda", requires_grad=True)
    br = torch.zeros(64, device="cuda", requires_grad=True)
    y = F.conv2d(x4[..., :3].float().permute(0, 3, 1, 2), wr, br, padding=1)
    gw, gb = torch.autograd.grad(y, (wr, br), dy.float().permute(0, 3, 1, 2))
    _close(dw, gw)
    _close(db, gb)


@pytest.mark.parametrize("ring", ["1", "0"])
@pytest.mark.parametrize("n,h,w,ci,co", [(1, 256, 1024, 64, 64), (2, 181, 733, 128, 128), (1, 301, 900, 64, 128)])
def test_conv_wgrad_halo_path(n, h, w, ci, co, ring, dispatch_cfg):
    """Large-M, small-channel layers take the halo-tiled wgrad kernel (odd H, W not a multiple of 64 included).
    ring=1 (default): row-ring kernel, 4-row tiles down 64-column strips; the last two shapes have slices that
    cross strip boundaries (full-halo reload mid-slice) and a ragged last tile row."""
    from can_distributed_pytorch_amd.ops import _ext
    from can_distributed_pytorch_amd.ops import conv as C
    dispatch_cfg(wgrad_halo_ring=int(ring), wgrad_tap=0)
    assert _ext.require().wgrad_plan(n * h * w, ci, co, 3, 0, 1024, 1, w)[2] == 8
    torch.manual_seed(5)
    x = torch.randn(n, h, w, ci, device="cuda").to(torch.bfloat16)
    dy = torch.randn(n, h, w, co, device="cuda").to(torch.bfloat16)
    dw = torch.empty(co, ci, 3, 3, device="cuda")
    db = torch.empty(co, device="cuda")
    C.conv_wgrad(dy, x, dw, db, ksize=3, dil=1)
    wr = torch.zeros(co, ci, 3, 3, device="cuda", requires_grad=True)
    br = torch.zeros(co, device="cuda", requires_grad=True)
    y = F.conv2d(x.float().permute(0, 3, 1, 2), wr, br, padding=1)
    gw, gb = torch.autograd.grad(y, (wr, br), dy.float().permute(0, 3, 1, 2))
    _close(dw, gw)
    _close(db, gb)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("n,h,w,ci,co", [(2, 128, 1024, 64, 64), (1, 512, 576, 128, 128), (4, 96, 704, 64, 128)])
def test_ring_wgrad_fast_addressing_bitwise(n, h, w, ci, co, dtype, dispatch_cfg):
    """Row-ring weight gradient with the hoisted DMA addressing (H % 4 == 0, W % 64 == 0: per-lane offsets from the
    tile / row origins, edge slots zeroed per lane) == the general per-piece addressing (ring_fast = 0),
    bitwise: several strips per image, several images, 2 ci / co tiles, slices crossing strips."""
    from can_distributed_pytorch_amd.ops import _ext
    from can_distributed_pytorch_amd.ops import conv as C
    dispatch_cfg(wgrad_tap=0)
    assert _ext.require().wgrad_plan(n * h * w, ci, co, 3, 0, 1024, 1, w)[2] == 8
    torch.manual_seed(21)
    x = torch.randn(n, h, w, ci, device="cuda").to(dtype)
    dy = torch.randn(n, h, w, co, device="cuda").to(dtype)
    dw0, db0 = torch.empty(co, ci, 3, 3, device="cuda"), torch.empty(co, device="cuda")
    dw1, db1 = torch.empty_like(dw0), torch.empty_like(db0)
    ws = C.WgradWorkspace("cuda")
    C.conv_wgrad(dy, x, dw0, db0, ksize=3, dil=1, ws=ws)             # FAST + SKEW (default)
    dw2, db2 = torch.empty_like(dw0), torch.empty_like(db0)
    dispatch_cfg(ring_skew=0)                                          # FAST, every wave issues DMA
    C.conv_wgrad(dy, x, dw2, db2, ksize=3, dil=1, ws=ws)
    dispatch_cfg(ring_fast=0)
    C.conv_wgrad(dy, x, dw1, db1, ksize=3, dil=1, ws=ws)
    torch.cuda.synchronize()
    assert torch.equal(dw0, dw1) and torch.equal(db0, db1)
    assert torch.equal(dw2, dw1) and torch.equal(db2, db1)
    if n * h * w <= 300000:
        wr = torch.zeros(co, ci, 3, 3, device="cuda", requires_grad=True)
        br = torch.zeros(co, device="cuda", requires_grad=True)
        y = F.conv2d(x.float().permute(0, 3, 1, 2), wr, br, padding=1)
        gw, gb = torch.autograd.grad(y, (wr, br), dy.float().permute(0, 3, 1, 2))
        _close(dw0, gw)
        _close(db0, gb)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_conv_wgrad_1x1_batched(dtype):
    """The four context-module 1x1 weight gradients in one batched launch == fp32 reference, per item."""
    from can_distributed_pytorch_amd.ops import conv as C
    torch.manual_seed(7)
    nb, n, h, w, c = 4, 2, 12, 128, 512
    dy = torch.randn(nb, n, h, w, c, device="cuda").to(dtype)
    x = torch.randn(nb, n, h, w, c, device="cuda").to(dtype)
    arena = torch.full((nb * c * c,), float("nan"), device="cuda")
    dws = [arena[i * c * c:(i + 1) * c * c].view(c, c, 1, 1) for i in range(nb)]
    assert C.wgrad_1x1_batched_ok(dy, x, dws)
    ws = C.WgradWorkspace("cuda")
    C.conv_wgrad_1x1_batched(dy, x, dws, ws=ws, scale=0.5)
    for b in range(nb):
        ref = 0.5 * dy[b].float().reshape(-1, c).t() @ x[b].float().reshape(-1, c)
        _close(dws[b].view(c, c), ref)


@pytest.mark.parametrize("n,h,w,ci,co,dil,cfg,bias", [
    (1, 6, 64, 128, 256, 1, 10, True), (2, 5, 128, 128, 512, 2, 10, False), (1, 9, 64, 256, 128, 2, 11, True),
    (2, 4, 64, 512, 128, 1, 11, True),
    # ragged widths (W % 64 != 0): virtual 64-pixel stages per row, padding pixels zero
    (1, 6, 90, 128, 256, 1, 10, True), (2, 5, 100, 512, 128, 2, 11, True)])
def test_conv_wgrad_v2_half_tiles(n, h, w, ci, co, dil, cfg, bias, dispatch_cfg):
    """v2 pipelined wgrad with 256co x 128k (Cin = 128, cfg 10) and 128co x 256k (Cout = 128, cfg 11) tiles (tap-ring
    kernel off)."""
    from can_distributed_pytorch_amd.ops import _ext
    from can_distributed_pytorch_amd.ops import conv as C
    dispatch_cfg(wgrad_tap=0)
    assert _ext.require().wgrad_plan(n * h * w, ci, co, 3, 0, 1024, dil, w)[2] == cfg
    torch.manual_seed(8)
    x = torch.randn(n, h, w, ci, device="cuda").to(torch.bfloat16)
    dy = torch.randn(n, h, w, co, device="cuda").to(torch.bfloat16)
    dw = torch.empty(co, ci, 3, 3, device="cuda")
    db = torch.empty(co, device="cuda") if bias else None
    C.conv_wgrad(dy, x, dw, db, ksize=3, dil=dil)
    wr = torch.zeros(co, ci, 3, 3, device="cuda", requires_grad=True)
    br = torch.zeros(co, device="cuda", requires_grad=True)
    y = F.conv2d(x.float().permute(0, 3, 1, 2), wr, br, padding=dil, dilation=dil)
    gw, gb = torch.autograd.grad(y, (wr, br), dy.float().permute(0, 3, 1, 2))
    _close(dw, gw)
    if bias:
        _close(db, gb)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("n,h,w,ci,co,dil", [(2, 8, 512, 128, 128, 1), (1, 6, 256, 256, 256, 1),
                                             (2, 4, 256, 256, 128, 2), (1, 4, 512, 128, 64, 1),
                                             (2, 8, 128, 64, 64, 1), (1, 12, 320, 64, 64, 1)])
def test_conv_pool_fwd_fused(n, h, w, ci, co, dil, dtype):
    """conv + bias + ReLU with the 2x2 max-pool in the epilogue == conv_igemm(EPI_BIAS_RELU) + max_pool2d, bitwise
    (both outputs; the 2-row pixel tiling must not change any conv value)."""
    from can_distributed_pytorch_amd.ops import conv as C
    torch.manual_seed(12)
    x = torch.randn(n, h, w, ci, device="cuda").to(dtype)
    wt = torch.randn(co, ci, 3, 3, device="cuda") * (2.0 / (9 * ci)) ** 0.5
    b = torch.randn(co, device="cuda") * 0.1
    wp = C.pack_weight_fwd(wt, dtype)
    assert C.conv_pool_fwd_ok(x, co, 3)
    y, yp, codes = C.conv_pool_fwd(x, wp, b, ksize=3, dil=dil, codes=True)
    _, yp2, codes2 = C.conv_pool_fwd(x, wp, b, ksize=3, dil=dil, keep_full=False, codes=True)
    y_ref = C.conv_igemm(x, wp, b, ksize=3, dil=dil)
    yp_ref = F.max_pool2d(y_ref.permute(0, 3, 1, 2), 2).permute(0, 2, 3, 1).contiguous()
    yp_ref2, codes_ref = C.maxpool_codes(y_ref)
    torch.cuda.synchronize()
    assert torch.equal(y, y_ref)
    assert torch.equal(yp, yp_ref) and torch.equal(yp_ref2, yp_ref)
    assert torch.equal(codes, codes_ref)
    assert torch.equal(yp2, yp) and torch.equal(codes2, codes)       # without the full-resolution store
    assert not C.conv_pool_fwd_ok(x[:, :h - 1].contiguous(), co, 3)     # odd H: not covered
    if ci == 64 and co == 64:                                            # halo kernel: whole 4-row tiles
        assert not C.conv_pool_fwd_ok(x[:, :h - 2].contiguous(), co, 3)
        assert not C.conv_pool_fwd_ok(x[:, :, :w - 32].contiguous(), co, 3)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("n,h,w,ci,co,tile", [(2, 8, 256, 128, 128, 29), (1, 6, 128, 256, 256, 27),
                                              (2, 4, 384, 64, 128, 29), (1, 10, 256, 128, 256, 0),
                                              (2, 6, 256, 128, 128, 0)])
def test_conv_pool_fwd_rring(n, h, w, ci, co, tile, dtype, dispatch_cfg):
    """Row-ring conv with the max-pool in the epilogue (2-row tiles, both rows per wave; tile 0 = dispatch
    rring_pool) == conv_igemm(EPI_BIAS_RELU) + max-pool codes, bitwise, with and without the full-size store."""
    from can_distributed_pytorch_amd.ops import conv as C
    dispatch_cfg(rring_pool=1)
    torch.manual_seed(13)
    x = torch.randn(n, h, w, ci, device="cuda").to(dtype)
    wt = torch.randn(co, ci, 3, 3, device="cuda") * (2.0 / (9 * ci)) ** 0.5
    b = torch.randn(co, device="cuda") * 0.1
    wp = C.pack_weight_fwd(wt, dtype)
    assert C.conv_pool_fwd_ok(x, co, 3, tile)
    y, yp, codes = C.conv_pool_fwd(x, wp, b, ksize=3, tile=tile, codes=True)
    _, yp2, codes2 = C.conv_pool_fwd(x, wp, b, ksize=3, tile=tile, keep_full=False, codes=True)
    y_ref = C.conv_igemm(x, wp, b, ksize=3)
    yp_ref, codes_ref = C.maxpool_codes(y_ref)
    torch.cuda.synchronize()
    assert torch.equal(y, y_ref)
    assert torch.equal(yp, yp_ref) and torch.equal(codes, codes_ref)
    assert torch.equal(yp2, yp) and torch.equal(codes2, codes)
    assert torch.equal(yp_ref, F.max_pool2d(y_ref.permute(0, 3, 1, 2), 2).permute(0, 2, 3, 1))


@pytest.mark.parametrize("n,h,w,ci,co,dil,beta", [(2, 8, 64, 512, 256, 2, 0.0), (1, 6, 128, 1024, 512, 1, 1.0),
                                                    (2, 5, 64, 256, 512, 2, 0.5)])
def test_wgrad_tiled_reduction_matches_grid_stride(n, h, w, ci, co, dil, beta, dispatch_cfg):
    """The LDS-transposing slab reduction (coalesced dW writes) == the grid-stride one, bitwise, beta included."""
    from can_distributed_pytorch_amd.ops import conv as C
    torch.manual_seed(11)
    x = torch.randn(n, h, w, ci, device="cuda").to(torch.bfloat16)
    dy = torch.randn(n, h, w, co, device="cuda").to(torch.bfloat16)
    dw0 = torch.randn(co, ci, 3, 3, device="cuda")
    db0 = torch.randn(co, device="cuda")
    out = []
    for tiled in (0, 1):
        dispatch_cfg(reduce_tiled=tiled)
        dw, db = dw0.clone(), db0.clone()
        C.conv_wgrad(dy, x, dw, db, ksize=3, dil=dil, beta=beta, scale=0.25)
        torch.cuda.synchronize()
        out.append((dw, db))
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])
    wr = torch.zeros(co, ci, 3, 3, device="cuda", requires_grad=True)
    y = F.conv2d(x.float().permute(0, 3, 1, 2), wr, None, padding=dil, dilation=dil)
    (gw,) = torch.autograd.grad(y, (wr,), dy.float().permute(0, 3, 1, 2))
    _close(out[1][0], beta * dw0 + 0.25 * gw)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("n,h,w,ci,co", [(2, 12, 20, 128, 64), (1, 9, 13, 256, 128), (2, 6, 8, 512, 256)])
def test_conv_dgrad_pool_backward_fused(n, h, w, ci, co, dtype):
    """EPI_POOLBWD (dgrad + max-pool backward + ReLU mask in one epilogue, driven by the max-pool codes) ==
    EPI_NONE + maxpool_bwd_codes == EPI_NONE + maxpool_bwd_relu on the pool input itself, bitwise."""
    from can_distributed_pytorch_amd.ops import _ext
    from can_distributed_pytorch_amd.ops import conv as C
    torch.manual_seed(9)
    wt = (torch.randn(ci, co, 3, 3, device="cuda") * 0.05).to(dtype).float()   # layer co -> ci (dgrad maps ci -> co)
    dy = torch.randn(n, h, w, ci, device="cuda").to(dtype)
    full = torch.relu(torch.randn(n, 2 * h, 2 * w, co, device="cuda")).to(dtype)
    full[:, ::3, ::2] = 0                                          # ties and all-zero windows
    _, codes = C.maxpool_codes(full)
    pack = C.pack_weight_dgrad(wt, dtype)
    fused = C.conv_igemm(dy, pack, None, ksize=3, epi=C.EPI_POOLBWD, mask=codes)
    dp = C.conv_igemm(dy, pack, None, ksize=3, epi=C.EPI_NONE)
    via_codes = C.maxpool_bwd_codes(codes, dp)
    ref = torch.empty_like(full)
    _ext.require().maxpool_bwd_relu(full.data_ptr(), dp.data_ptr(), ref.data_ptr(), n, 2 * h, 2 * w, co,
                                    C.dt_code(dtype), _ext.stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(via_codes, ref)
    assert torch.equal(fused, ref)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("n,h,w,ci,co,dil,epi", [
    (2, 12, 20, 128, 64, 1, "pool"), (1, 9, 13, 256, 128, 1, "pool"), (2, 6, 64, 512, 256, 1, "pool"),
    (2, 16, 96, 64, 64, 1, "mask"), (1, 10, 70, 128, 64, 1, "mask"), (2, 12, 128, 128, 128, 1, "mask"),
    (2, 8, 64, 512, 512, 2, "mask"), (1, 5, 40, 256, 128, 2, "mask"), (2, 8, 128, 64, 128, 1, "mask"),
    # > 512 partial rows: folded by the short launch conv_wgrad queues after its GEMM
    (8, 96, 128, 256, 512, 2, "mask"), (4, 48, 128, 128, 256, 1, "pool")])
def test_dgrad_bias_partials_feed_wgrad(n, h, w, ci, co, dil, epi, dtype):
    """The data-gradient epilogue's bias partials (EPI_MASK on the LDS-DMA and halo kernels, EPI_POOLBWD through
    the max-pool codes) reduce to the bias gradient of the tensor it writes: db from the partials == db from
    re-reading dY (bias_colsum / in-GEMM), and dW is untouched by the switch.  Here the conv maps co -> ci
    (dgrad of a ci -> co layer), so dX has ci channels."""
    from can_distributed_pytorch_amd.ops import conv as C
    torch.manual_seed(21)
    wt = (torch.randn(co, ci, 3, 3, device="cuda") * 0.05).to(dtype).float()   # layer ci -> co
    pack = C.pack_weight_dgrad(wt, dtype)                                         # dgrad: co -> ci
    dy = torch.randn(n, h, w, co, device="cuda").to(dtype)
    if epi == "pool":
        full = torch.relu(torch.randn(n, 2 * h, 2 * w, ci, device="cuda")).to(dtype)
        _, mask = C.maxpool_codes(full)
        e = C.EPI_POOLBWD
    else:
        mask = torch.randn(n, h, w, ci, device="cuda").to(dtype)
        e = C.EPI_MASK
    dx, bp = C.conv_dgrad_with_bias(dy, pack, ksize=3, dil=dil, epi=e, mask=mask)
    dx_plain = C.conv_igemm(dy, pack, None, ksize=3, dil=dil, epi=e, mask=mask)
    assert bp is not None and bp.shape[1] == ci
    torch.cuda.synchronize()
    assert torch.equal(dx, dx_plain)                       # the partials do not change the written gradient
    # dX is the dY of the previous layer (ci channels): its weight gradient against some input
    xin = torch.randn(*dx.shape[:3], 64, device="cuda").to(dtype)
    dw1, db1 = torch.empty(ci, 64, 3, 3, device="cuda"), torch.empty(ci, device="cuda")
    dw2, db2 = torch.empty_like(dw1), torch.empty_like(db1)
    C.conv_wgrad(dx, xin, dw1, db1, ksize=3)
    C.conv_wgrad(dx, xin, dw2, db2, ksize=3, bias_partials=bp)
    torch.cuda.synchronize()
    assert torch.equal(dw1, dw2)
    ref = dx.float().sum(dim=(0, 1, 2))
    # partials sum the unrounded fp32 values: equal to the rounded-dY column sums to rounding
    assert torch.allclose(db2, ref, rtol=2e-2, atol=2e-2 * ref.abs().mean().item())
    assert torch.allclose(db1, ref, rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("epi", ["fwd", "bias", "none", "dgrad", "pool"])
@pytest.mark.parametrize("n,h,w", [(2, 64, 640), (1, 61, 600), (3, 8, 1024), (1, 4, 64)])
def test_ws64_matches_halo_kernel(n, h, w, epi, dispatch_cfg):
    """Cin = Cout = 64 convs: the weight-stationary persistent kernel (several tiles per block, ragged tiles)
    == the per-tile halo kernel (ws64 = 0) bitwise — the same MFMA k order per output — and both == the
    fp32 reference."""
    from can_distributed_pytorch_amd.ops import conv as C
    torch.manual_seed(13)
    dev = "cuda"
    x = torch.randn(n, h, w, 64, device=dev).to(torch.bfloat16)
    wt = (torch.randn(64, 64, 3, 3, device=dev) * 0.05).to(torch.bfloat16).float()
    b = torch.randn(64, device=dev)
    mask = torch.randn(n, h, w, 64, device=dev).to(torch.bfloat16)
    if epi == "pool" and (h % 4 or w % 64):
        pytest.skip("fused pool: whole 4 x 64 tiles only")

    def run():
        if epi == "fwd":
            return (C.conv_igemm(x, C.pack_weight_fwd(wt), b, ksize=3),)
        if epi == "bias":
            return (C.conv_igemm(x, C.pack_weight_fwd(wt), b, ksize=3, epi=C.EPI_BIAS),)
        if epi == "none":
            return (C.conv_igemm(x, C.pack_weight_fwd(wt), None, ksize=3, epi=C.EPI_NONE),)
        if epi == "dgrad":
            return (C.conv_igemm(x, C.pack_weight_dgrad(wt), None, ksize=3, epi=C.EPI_MASK, mask=mask),)
        y, yp, codes = C.conv_pool_fwd(x, C.pack_weight_fwd(wt), b, ksize=3, codes=True)
        return y, yp, codes

    dispatch_cfg(ws64=1)
    new = run()
    dispatch_cfg(ws64=0)
    old = run()
    torch.cuda.synchronize()
    for a_, b_ in zip(new, old):
        assert torch.equal(a_, b_)
    if epi in ("fwd", "pool"):
        _close(new[0], _ref(x, wt, b, 1))
    elif epi == "dgrad":
        xr = torch.zeros(n, 64, h, w, device=dev, requires_grad=True)
        (gx,) = torch.autograd.grad(F.conv2d(xr, wt, None, padding=1), xr, x.float().permute(0, 3, 1, 2))
        _close(new[0], gx.permute(0, 2, 3, 1) * (mask.float() > 0))


@pytest.mark.parametrize("epi", [2, 4])
@pytest.mark.parametrize("n,h,w,ci,co,k", [(2, 12, 16, 512, 512, 1), (1, 9, 13, 128, 256, 3)])
def test_conv_igemm_batched_matches_per_item(n, h, w, ci, co, k, epi):
    """nb convs in one launch (grid.y = item) == nb single launches, bitwise (context module conv{S}_2)."""
    from can_distributed_pytorch_amd.ops import conv as C
    torch.manual_seed(15)
    nb = 4
    x = torch.randn(nb, n, h, w, ci, device="cuda").to(torch.bfloat16)
    wp = torch.stack([C.pack_weight_fwd(torch.randn(co, ci, k, k, device="cuda") * 0.05) for _ in range(nb)])
    y = C.conv_igemm_batched(x, wp, ksize=k, epi=epi)
    ref = torch.stack([C.conv_igemm(x[i], wp[i], None, ksize=k, epi=epi) for i in range(nb)])
    torch.cuda.synchronize()
    assert torch.equal(y, ref)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("n,h,w,beta", [(2, 40, 128, 0.0), (1, 37, 150, 0.0), (2, 13, 70, 1.0), (1, 256, 512, 0.0)])
def test_conv_dgrad_w1g_fused(n, h, w, beta, dtype):
    """conv1_2's data gradient with conv1_1's weight gradient fused (ws64 W1G): dX bitwise equal to the plain ws64
    data gradient; dW1 / db1 vs fp32 PyTorch of conv1_1's weight gradient from that dX (ragged tiles, beta)."""
    from can_distributed_pytorch_amd.ops import conv as C
    torch.manual_seed(11)
    dev = "cuda"
    wt = (torch.randn(64, 64, 3, 3, device=dev) * 0.05).to(dtype).float()
    dgr = C.pack_weight_dgrad(wt, dtype)
    dy = torch.randn(n, h, w, 64, device=dev).to(dtype)
    mask = torch.randn(n, h, w, 64, device=dev).to(dtype)
    img = torch.randn(n, 3, h, w, device=dev)
    x4 = C.to_nhwc4(img, dtype)
    dx_ref = C.conv_igemm(dy, dgr, None, ksize=3, epi=C.EPI_MASK, mask=mask)
    cap = C.w1g_slab_cap(dev)
    sl = torch.full((cap, 36 * 64), float("nan"), device=dev)
    bsl = torch.full((cap, 64), float("nan"), device=dev)
    dw0 = torch.randn(64, 3, 3, 3, device=dev)
    db0 = torch.randn(64, device=dev)
    dw, db = dw0.clone(), db0.clone()
    dx = C.conv_dgrad_w1g(dy, dgr, mask, x4, dw, db, slabs=sl, bslabs=bsl, store_dx=True, beta=beta)
    torch.cuda.synchronize()
    assert torch.equal(dx, dx_ref)
    wr = torch.zeros(64, 3, 3, 3, device=dev, requires_grad=True)
    br = torch.zeros(64, device=dev, requires_grad=True)
    y = F.conv2d(x4[..., :3].float().permute(0, 3, 1, 2), wr, br, padding=1)
    gw, gb = torch.autograd.grad(y, (wr, br), dx_ref.float().permute(0, 3, 1, 2))
    _close(dw, gw + beta * dw0)
    _close(db, gb + beta * db0)
    # against the unfused first-layer weight gradient of the same dX
    dw2, db2 = dw0.clone(), db0.clone()
    C.conv_wgrad(dx_ref, x4, dw2, db2, ksize=3, first=True, beta=beta)
    _close(dw, dw2)
    _close(db, db2)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("n,h,w,ci,co,dil", [(2, 8, 128, 256, 256, 1), (1, 12, 128, 1024, 512, 2),
                                             (1, 6, 256, 128, 256, 1), (2, 10, 384, 64, 256, 2),
                                             (1, 4, 256, 512, 512, 2), (1, 2, 128, 192, 256, 1),
                                             # cfg 28: 64-channel 4-row tiles (8 row slots, 2-stage lead)
                                             (2, 8, 128, 128, 64, 1), (1, 8, 512, 128, 64, 1), (1, 4, 256, 256, 64, 2),
                                             # cfg 29: 128-channel 2-row tiles (the wave tile of cfg 22)
                                             (2, 6, 128, 256, 128, 1), (1, 4, 256, 384, 128, 2),
                                             # ragged: masked last column block (W % 128 != 0) / tile row (odd H)
                                             (2, 9, 240, 256, 256, 1), (1, 7, 200, 512, 512, 2),
                                             (1, 10, 240, 128, 64, 1), (2, 9, 120, 256, 128, 1),
                                             (1, 5, 480, 256, 256, 2), (1, 3, 104, 64, 64, 2)])
def test_row_ring_conv_bitwise(n, h, w, ci, co, dil, dtype, dispatch_cfg):
    """Row-ring 3x3 conv (cfg 27 / 28: activation rows staged once per 64-channel chunk, taps read shifted windows
    of the row slots) == the LDS-DMA kernel of the same tile (cfg 21 256 x 256 / cfg 23 64 x 512, rring = 0)
    bitwise for every epilogue it takes:
    bias + ReLU, plain, bias, ReLU-mask data gradient with bias partials, pool-backward data gradient, fp32 store;
    one- and multi-block-wide maps (zero guards / neighbour-pixel guards), dilation 1 and 2, top/bottom padding."""
    from can_distributed_pytorch_amd.ops import conv as C
    from can_distributed_pytorch_amd.ops import _ext
    torch.manual_seed(37)
    x = torch.randn(n, h, w, ci, device="cuda").to(dtype)
    wt = (torch.randn(co, ci, 3, 3, device="cuda") * (2.0 / (9 * ci)) ** 0.5).to(dtype).float()
    b = torch.randn(co, device="cuda") * 0.1
    wf = C.pack_weight_fwd(wt, dtype)
    wdt = (torch.randn(ci, co, 3, 3, device="cuda") * 0.05).to(dtype).float()     # a co -> ci layer: dgrad ci -> co
    wd = C.pack_weight_dgrad(wdt, dtype)
    mask = torch.randn(n, h, w, co, device="cuda").to(dtype)
    full = torch.relu(torch.randn(n, 2 * h, 2 * w, co, device="cuda")).to(dtype)
    full[:, ::3, ::2] = 0
    _, codes = C.maxpool_codes(full)
    ext = _ext.require()

    def run():
        r = [C.conv_igemm(x, wf, b, ksize=3, dil=dil),
             C.conv_igemm(x, wf, None, ksize=3, dil=dil, epi=C.EPI_NONE),
             C.conv_igemm(x, wf, b, ksize=3, dil=dil, epi=C.EPI_BIAS)]
        r += list(C.conv_dgrad_with_bias(x, wd, ksize=3, dil=dil, epi=C.EPI_MASK, mask=mask))
        r += list(C.conv_dgrad_with_bias(x, wd, ksize=3, dil=dil, epi=C.EPI_POOLBWD, mask=codes))
        y32 = torch.empty(n, h, w, co, dtype=torch.float32, device="cuda")
        ext.conv_igemm(x.data_ptr(), wf.data_ptr(), b.data_ptr(), 0, y32.data_ptr(), n, h, w, ci, co, 3, dil, 7, 0, 0,
                       C.dt_code(dtype), _ext.stream_ptr(x.device), 0, 0)
        r.append(y32)
        torch.cuda.synchronize()
        return r

    dispatch_cfg(rring=0)
    ref = run()
    dispatch_cfg(rring=2, rring64=1, rring128=3)   # every dilation, 64-channel 4-row and 128-channel 2-row tiles
    assert ext.conv_plan(h, w, ci, co, 3, dil, C.EPI_BIAS_RELU) in (27, 28, 29)    # the row ring really runs
    got = run()
    assert len(got) == len(ref)
    for i, (g, r) in enumerate(zip(got, ref)):
        assert g is not None
        if i in (4, 6) and (w > 128 or h % (4 if co == 64 else 2)):
            # bias partials: one row per (tile, wave row); a multi-block-wide map groups the pixels of a row-ring
            # tile (2 rows x 128 columns) differently from a 256-pixel run, so only the column sums agree
            torch.testing.assert_close(g.sum(0), r.sum(0), rtol=1e-4, atol=1e-3)
        else:
            assert torch.equal(g, r), f"output {i} differs"
    # and against the fp32 reference (the cfg-21 path is covered there already; one direct check here)
    yref = torch.relu(torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), wt, b, padding=dil,
                                                 dilation=dil)).permute(0, 2, 3, 1)
    check_out16(got[0], yref)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_image_chunked_launches(dtype, monkeypatch):
    """Batches beyond the 32-bit per-launch operand size run as consecutive launches over image chunks (forced
    here with a tiny limit): forward / data gradient / fused pool / context GEMMs bitwise equal to one launch,
    weight gradients accumulated over the chunks equal to the fp32 reference."""
    from can_distributed_pytorch_amd.ops import conv as C
    torch.manual_seed(31)
    n, h, w = 5, 16, 128
    x64 = torch.randn(n, h, w, 64, device="cuda").to(dtype)
    x256 = torch.randn(n, h, w, 256, device="cuda").to(dtype)
    w1 = (torch.randn(256, 64, 3, 3, device="cuda") * 0.05).to(dtype).float()
    w2 = (torch.randn(256, 256, 3, 3, device="cuda") * 0.03).to(dtype).float()
    b = torch.randn(256, device="cuda")
    mask = torch.randn(n, h, w, 64, device="cuda").to(dtype)

    def run():
        y = C.conv_igemm(x64, C.pack_weight_fwd(w1, dtype), b, ksize=3)
        dx, part = C.conv_dgrad_with_bias(x256, C.pack_weight_dgrad(w1, dtype), ksize=3, mask=mask)
        _, yp, cd = C.conv_pool_fwd(x256, C.pack_weight_fwd(w2, dtype), b, ksize=3, keep_full=False, codes=True)
        dw = torch.empty(256, 64, 3, 3, device="cuda")
        db = torch.empty(256, device="cuda")
        C.conv_wgrad(x256, x64, dw, db, ksize=3)
        torch.cuda.synchronize()
        return y, dx, None if part is None else part.sum(0), yp, cd, dw, db

    one = run()
    monkeypatch.setattr(C, "MAX_ELEMS_PER_LAUNCH", 2 * h * w * 256)     # 2 images per launch -> 3 launches
    assert len(C.image_chunks(n, h * w * 256)) == 3
    many = run()
    for i in (0, 1, 3, 4):
        assert torch.equal(one[i], many[i]), i
    if one[2] is not None:
        torch.testing.assert_close(many[2], one[2], rtol=1e-5, atol=1e-3)
    xr = x64.float().permute(0, 3, 1, 2)
    wr = torch.zeros(256, 64, 3, 3, device="cuda", requires_grad=True)
    br = torch.zeros(256, device="cuda", requires_grad=True)
    gw, gb = torch.autograd.grad(F.conv2d(xr, wr, br, padding=1), (wr, br), x256.float().permute(0, 3, 1, 2))
    _close(many[5], gw)
    _close(many[6], gb)
