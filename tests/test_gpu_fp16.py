"""fp16 variants of the native kernels and the fp16 native step (dynamic loss scaling on the device).

Every kernel family is instantiated for bf16 and fp16 (csrc/common.h DT_*);
the fp16 path is checked against plain fp32 PyTorch references of the same
op, like the bf16 tests in test_gpu_conv.py / test_gpu_components.py.
"""
import copy

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

F16 = torch.float16


def _close(a, b, tol=1e-2):
    err = (a.float() - b.float()).abs().max().item()
    scale = b.float().abs().max().item() + 1e-6
    assert err <= tol * scale, f"max err {err} vs scale {scale}"


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("n,h,w,ci,co,k,dil,tile", [
    (2, 24, 40, 64, 64, 3, 1, 0), (1, 17, 33, 128, 128, 3, 1, 0), (2, 32, 32, 256, 512, 3, 2, 0),
    (2, 16, 24, 512, 512, 1, 1, 0), (1, 20, 20, 128, 256, 3, 1, 21), (2, 9, 13, 64, 128, 3, 2, 22),
    (3, 11, 17, 64, 64, 3, 1, 23), (1, 20, 40, 128, 128, 3, 1, 25), (2, 10, 200, 64, 64, 3, 1, 31),
    (1, 9, 130, 64, 128, 3, 1, 31), (1, 20, 20, 128, 256, 3, 1, 1), (1, 20, 20, 128, 256, 3, 1, 11),
])
def test_fp16_conv_fwd(n, h, w, ci, co, k, dil, tile):
    from can_distributed_pytorch_amd.ops import conv as C
    torch.manual_seed(0)
    x = torch.randn(n, h, w, ci, device="cuda").to(F16)
    wt = (torch.randn(co, ci, k, k, device="cuda") * 0.05).to(F16).float()
    b = torch.randn(co, device="cuda")
    y = C.conv_igemm(x, C.pack_weight_fwd(wt, F16), b, ksize=k, dil=dil, tile=tile)
    assert y.dtype == F16
    ref = torch.relu(F.conv2d(x.float().permute(0, 3, 1, 2), wt, b, padding=dil * (k // 2), dilation=dil))
    _close(y, ref.permute(0, 2, 3, 1), 5e-3)


@pytest.mark.parametrize("tile", [0, 32])
def test_fp16_first_layer(tile):
    from can_distributed_pytorch_amd.ops import conv as C
    torch.manual_seed(1)
    img = torch.randn(2, 3, 40, 136, device="cuda")
    wt = (torch.randn(64, 3, 3, 3, device="cuda") * 0.2).to(F16).float()
    b = torch.randn(64, device="cuda")
    x4 = C.to_nhwc4(img, F16)
    y = C.conv_igemm(x4, C.pack_weight_first(wt, F16), b, ksize=3, first=True, tile=tile)
    ref = torch.relu(F.conv2d(x4[..., :3].float().permute(0, 3, 1, 2), wt, b, padding=1))
    _close(y, ref.permute(0, 2, 3, 1), 5e-3)


@pytest.mark.parametrize("n,h,w,ci,co,dil,tile", [
    (2, 24, 40, 64, 128, 1, 0), (1, 16, 16, 512, 1024, 2, 0), (2, 9, 140, 64, 64, 1, 31), (1, 9, 13, 64, 64, 1, 23)])
def test_fp16_dgrad_mask(n, h, w, ci, co, dil, tile):
    from can_distributed_pytorch_amd.ops import conv as C
    torch.manual_seed(2)
    wt = (torch.randn(co, ci, 3, 3, device="cuda") * 0.05).to(F16).float()
    dy = torch.randn(n, h, w, co, device="cuda").to(F16)
    mask = torch.randn(n, h, w, ci, device="cuda").to(F16)
    dx = C.conv_igemm(dy, C.pack_weight_dgrad(wt, F16), None, ksize=3, dil=dil, epi=C.EPI_MASK, mask=mask, tile=tile)
    xr = torch.zeros(n, ci, h, w, device="cuda", requires_grad=True)
    (gx,) = torch.autograd.grad(F.conv2d(xr, wt, None, padding=dil, dilation=dil), xr, dy.float().permute(0, 3, 1, 2))
    _close(dx, gx.permute(0, 2, 3, 1) * (mask.float() > 0), 5e-3)


@pytest.mark.parametrize("n,h,w,ci,co,k,dil,first", [
    (2, 24, 40, 64, 64, 3, 1, False), (2, 16, 16, 256, 512, 3, 2, False), (2, 16, 24, 512, 512, 1, 1, False),
    (2, 5, 128, 512, 256, 3, 2, False),
    (1, 256, 1024, 64, 64, 3, 1, False), (2, 40, 56, 4, 64, 3, 1, True)])
def test_fp16_wgrad(n, h, w, ci, co, k, dil, first):
    """Generic, v2 row-aligned (cfg 9), halo (cfg 8) and first-layer weight-gradient paths in fp16."""
    from can_distributed_pytorch_amd.ops import conv as C
    torch.manual_seed(3)
    if first:
        x = C.to_nhwc4(torch.randn(n, 3, h, w, device="cuda"), F16)
        xin = x[..., :3].float().permute(0, 3, 1, 2)
        cin = 3
    else:
        x = torch.randn(n, h, w, ci, device="cuda").to(F16)
        xin = x.float().permute(0, 3, 1, 2)
        cin = ci
    dy = torch.randn(n, h, w, co, device="cuda").to(F16)
    dw = torch.empty(co, cin, k, k, device="cuda")
    db = torch.empty(co, device="cuda")
    C.conv_wgrad(dy, x, dw, db, ksize=k, dil=dil, first=first)
    wr = torch.zeros(co, cin, k, k, device="cuda", requires_grad=True)
    br = torch.zeros(co, device="cuda", requires_grad=True)
    y = F.conv2d(xin, wr, br, padding=dil * (k // 2), dilation=dil)
    gw, gb = torch.autograd.grad(y, (wr, br), dy.float().permute(0, 3, 1, 2))
    _close(dw, gw, 5e-3)
    _close(db, gb, 5e-3)


def test_fp16_wgrad_device_scale():
    """dscale (1 / loss scale, a device scalar) multiplies the weight and bias gradients."""
    from can_distributed_pytorch_amd.ops import conv as C
    torch.manual_seed(4)
    x = torch.randn(1, 12, 64, 256, device="cuda").to(F16)
    dy = torch.randn(1, 12, 64, 256, device="cuda").to(F16)
    d1, b1 = torch.empty(256, 256, 3, 3, device="cuda"), torch.empty(256, device="cuda")
    d2, b2 = torch.empty_like(d1), torch.empty_like(b1)
    C.conv_wgrad(dy, x, d1, b1, ksize=3)
    C.conv_wgrad(dy, x, d2, b2, ksize=3, dscale=torch.tensor([0.125], device="cuda"))
    assert torch.equal(d2, d1 * 0.125) and torch.equal(b2, b1 * 0.125)


def test_fp16_maxpool():
    from can_distributed_pytorch_amd.ops import _ext
    C = _ext.require()
    n, h, w, c = 2, 16, 24, 64
    x = torch.relu(torch.randn(n, h, w, c, device="cuda")).to(F16)
    y = torch.empty(n, h // 2, w // 2, c, dtype=F16, device="cuda")
    C.maxpool_fwd(x.data_ptr(), y.data_ptr(), n, h, w, c, 1, _ext.stream_ptr())
    ref = F.max_pool2d(x.float().permute(0, 3, 1, 2), 2).permute(0, 2, 3, 1)
    assert torch.equal(y.float(), ref)


def _models(seed):
    from can_distributed_pytorch_amd.models import CANNet
    torch.manual_seed(seed)
    ref = CANNet(backend="torch")
    for m in ref.modules():
        if isinstance(m, torch.nn.Conv2d):
            fan_in = m.in_channels * m.kernel_size[0] * m.kernel_size[1]
            torch.nn.init.normal_(m.weight, std=(2.0 / fan_in) ** 0.5)
            if m.bias is not None:
                torch.nn.init.uniform_(m.bias, -0.05, 0.05)
    return ref.cuda()


def test_fp16_executor_grads_vs_fp32():
    """fp16 executor forward + backward against fp32 autograd; at least as close as the bf16 executor."""
    from can_distributed_pytorch_amd.ops.executor import CANNetExecutor
    ref = _models(1)
    n, h, w = 2, 64, 96
    x = torch.randn(n, 3, h, w, device="cuda")
    gt = torch.rand(n, 1, h // 8, w // 8, device="cuda") * 4
    crit = torch.nn.MSELoss(reduction="sum")
    crit(ref(x), gt).backward()
    errs = {}
    for dt in (torch.bfloat16, F16):
        m = copy.deepcopy(ref)
        m.zero_grad(set_to_none=True)
        m.exec_backend = "hip"
        m._executor = CANNetExecutor(m, dtype=dt)
        crit(m(x), gt).backward()
        errs[dt] = max(_rel(pn.grad, pr.grad) for pn, pr in zip(m.parameters(), ref.parameters()))
    assert errs[F16] < max(1.5 * errs[torch.bfloat16], 0.02), errs


def test_fp16_native_step_loss_scaling():
    """Overflowing loss scale -> update skipped and scale backed off; clean steps -> update and growth."""
    from can_distributed_pytorch_amd.engine.native import NativeStepper
    m = _models(2)
    m.exec_backend = "hip"
    x = torch.randn(1, 3, 64, 64, device="cuda")
    gt = torch.rand(1, 1, 8, 8, device="cuda")
    st = NativeStepper("cuda", dtype="fp16", lr=1e-6, graph=False, model=m, init_scale=2.0 ** 40, scale_interval=2)
    w0 = st.arena.data.clone()
    st.step(x, gt)
    torch.cuda.synchronize()
    assert st.skipped_last() and not st.nonfinite()
    assert torch.equal(st.arena.data, w0)                       # no update on overflow
    assert st.loss_scale() == 2.0 ** 39
    st.scaler.copy_(torch.tensor([1024.0, 1 / 1024.0, 0.0, 0.0], device="cuda"))
    st.step(x, gt)
    st.step(x, gt)
    torch.cuda.synchronize()
    assert not st.skipped_last()
    assert not torch.equal(st.arena.data, w0)
    assert st.loss_scale() == 2048.0                             # grew after 2 clean steps


def test_fp16_native_step_matches_bf16_and_graph():
    """fp16 native step (eager and hipGraph) tracks the bf16 native step; graph replay == eager."""
    from can_distributed_pytorch_amd.engine.native import NativeStepper
    ref = _models(3)
    x = torch.randn(2, 3, 64, 64, device="cuda")
    gt = torch.rand(2, 1, 8, 8, device="cuda")
    runs = {}
    for key, dt, graph in (("bf16", "bf16", False), ("fp16", "fp16", False), ("fp16g", "fp16", True)):
        m = copy.deepcopy(ref)
        m.exec_backend = "hip"
        st = NativeStepper("cuda", dtype=dt, lr=1e-6, graph=graph, model=m, init_scale=256.0)
        w0 = st.arena.data.clone()
        losses = [float(st.step(x, gt)) for _ in range(3)]
        torch.cuda.synchronize()
        runs[key] = (st.arena.data - w0, losses)
    d16, l16 = runs["fp16"]
    dg, lg = runs["fp16g"]
    assert torch.allclose(d16, dg, rtol=1e-5, atol=1e-10) and l16 == pytest.approx(lg, rel=1e-6)
    db, lb = runs["bf16"]
    assert _rel(d16, db) < 0.1, _rel(d16, db)
    assert l16 == pytest.approx(lb, rel=0.05)
