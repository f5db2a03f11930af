"""torch.ops.cannet.* custom operators (ops/library.py): registration, fake-tensor shape propagation (CPU) and,
on the GPU, numerics of forward / backward against fp32 ATen and torch.library.opcheck."""
import pytest
import torch
import torch.nn.functional as F

from can_distributed_pytorch_amd.ops import library as L  # noqa: F401  (registers the ops)


def test_ops_registered():
    for name in ("conv2d_nhwc", "conv2d_nhwc_backward", "relu_max_pool2x2", "relu_max_pool2x2_backward", "sgd_momentum_"):
        assert hasattr(torch.ops.cannet, name)


def test_fake_shapes_cpu():
    from torch._subclasses.fake_tensor import FakeTensorMode
    with FakeTensorMode():
        x = torch.empty(2, 24, 32, 128, dtype=torch.bfloat16)
        w = torch.empty(64, 128, 3, 3)
        b = torch.empty(64)
        y = torch.ops.cannet.conv2d_nhwc(x, w, b, 2, True)
        assert y.shape == (2, 24, 32, 64) and y.dtype == torch.bfloat16
        p, codes = torch.ops.cannet.relu_max_pool2x2(y)
        assert p.shape == (2, 12, 16, 64) and codes.shape == (2, 12, 16, 8) and codes.dtype == torch.int32
        dx, dw, db = torch.ops.cannet.conv2d_nhwc_backward(y, x, y, w, 2, True, True)
        assert dx.shape == x.shape and dw.shape == w.shape and db.shape == (64,)


def test_conv_shape_checks_cpu():
    from torch._subclasses.fake_tensor import FakeTensorMode
    with FakeTensorMode():
        with pytest.raises(ValueError):
            torch.ops.cannet.conv2d_nhwc(torch.empty(1, 8, 8, 3, dtype=torch.bfloat16), torch.empty(64, 3, 3, 3),
                                         None, 1, True)
        with pytest.raises(ValueError):
            torch.ops.cannet.conv2d_nhwc(torch.empty(1, 8, 8, 64), torch.empty(64, 64, 3, 3), None, 1, True)


def test_module_state_dict_matches_conv2d():
    m = L.Conv2dNHWC(64, 128, 3, dilation=2)
    ref = torch.nn.Conv2d(64, 128, 3, padding=2, dilation=2)
    assert {k: v.shape for k, v in m.state_dict().items()} == {k: v.shape for k, v in ref.state_dict().items()}


def _rel(a, b):
    return ((a.double() - b.double()).norm() / (b.double().norm() + 1e-30)).item()


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("n,h,w,ci,co,k,dil,relu,bias", [
    (2, 20, 36, 64, 128, 3, 1, True, True), (1, 17, 29, 128, 64, 3, 2, True, False),
    (2, 16, 64, 256, 256, 3, 2, False, True), (3, 9, 11, 128, 192, 1, 1, True, True)])
def test_conv2d_nhwc_vs_aten(n, h, w, ci, co, k, dil, relu, bias, dtype):
    torch.manual_seed(0)
    x = torch.randn(n, h, w, ci, device="cuda").to(dtype)
    m = L.Conv2dNHWC(ci, co, k, dilation=dil, bias=bias, relu=relu).cuda()
    with torch.no_grad():
        m.weight.normal_(0, 0.05)
        if bias:
            m.bias.normal_(0, 0.1)
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    wr = m.weight.detach().clone().requires_grad_(True)
    br = m.bias.detach().clone().requires_grad_(True) if bias else None
    z = F.conv2d(xr, wr, br, padding=dil * (k // 2), dilation=dil)
    yr = F.relu(z) if relu else z
    xg = x.clone().requires_grad_(True)
    y = m(xg)
    assert y.dtype == dtype and y.shape == (n, h, w, co)
    assert _rel(y.float().permute(0, 3, 1, 2), yr) < 1e-2
    g = torch.randn_like(yr)
    y.backward(g.permute(0, 2, 3, 1).to(dtype))
    # the reference backward through the SAME ReLU mask (the op's own 16-bit y: a near-zero output whose sign
    # differs from the fp32 reference would otherwise dominate the comparison) and the same 16-bit dY
    dz = g.to(dtype).float()
    if relu:
        dz = dz * (y.float().permute(0, 3, 1, 2) > 0)
    refs = torch.autograd.grad(z, [xr, wr] + ([br] if bias else []), dz)
    assert _rel(xg.grad.float().permute(0, 3, 1, 2), refs[0]) < 1e-2
    assert _rel(m.weight.grad, refs[1]) < 1e-2
    if bias:
        assert _rel(m.bias.grad, refs[2]) < 1e-2


@pytest.mark.gpu
def test_maxpool_op_vs_aten():
    torch.manual_seed(1)
    x = F.relu(torch.randn(2, 16, 24, 64, device="cuda")).to(torch.bfloat16)
    xg = x.clone().requires_grad_(True)
    y = L.ReluMaxPool2x2()(xg)
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    yr = F.relu(F.max_pool2d(xr, 2, 2))
    assert torch.equal(y.float().permute(0, 3, 1, 2), yr)
    g = torch.randn_like(yr)
    yr.backward(g)
    y.backward(g.permute(0, 2, 3, 1).to(torch.bfloat16))
    assert _rel(xg.grad.float().permute(0, 3, 1, 2), xr.grad) < 1e-2


@pytest.mark.gpu
def test_relu_maxpool_op_signed_input_vs_aten():
    """Signed input (no ReLU before the op): values and gradient are those of max_pool2d(relu(x))."""
    torch.manual_seed(3)
    x = torch.randn(2, 10, 14, 64, device="cuda").to(torch.bfloat16)
    x[0, :2, :2, :8] = -1.0                       # whole windows <= 0
    xg = x.clone().requires_grad_(True)
    y = L.ReluMaxPool2x2()(xg)
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    yr = F.max_pool2d(F.relu(xr), 2, 2)
    assert torch.equal(y.float().permute(0, 3, 1, 2), yr)
    g = torch.randn_like(yr)
    yr.backward(g)
    y.backward(g.permute(0, 2, 3, 1).to(torch.bfloat16))
    assert _rel(xg.grad.float().permute(0, 3, 1, 2), xr.grad) < 1e-2
    assert torch.count_nonzero(xg.grad[0, :2, :2, :8]) == 0


@pytest.mark.gpu
def test_sgd_op_matches_torch_optim():
    torch.manual_seed(2)
    p0 = torch.randn(1003, device="cuda")
    p, q = p0.clone(), p0.clone().requires_grad_(True)
    buf = torch.zeros_like(p)
    opt = torch.optim.SGD([q], lr=0.1, momentum=0.95)
    for _ in range(3):
        g = torch.randn_like(p)
        torch.ops.cannet.sgd_momentum_(p, buf, g, 0.1, 0.95, 1.0)
        q.grad = g.clone()
        opt.step()
    torch.cuda.synchronize()
    assert torch.allclose(p, q.detach(), rtol=1e-6, atol=1e-6)


@pytest.mark.gpu
def test_opcheck_conv():
    x = torch.randn(1, 8, 16, 64, device="cuda").to(torch.bfloat16)
    w = torch.randn(64, 64, 3, 3, device="cuda") * 0.05
    b = torch.randn(64, device="cuda")
    torch.library.opcheck(torch.ops.cannet.conv2d_nhwc.default, (x, w, b, 1, True),
                          test_utils=("test_schema", "test_faketensor", "test_autograd_registration"))


@pytest.mark.gpu
def test_compile_fullgraph():
    m = torch.nn.Sequential(L.Conv2dNHWC(64, 64), L.ReluMaxPool2x2(), L.Conv2dNHWC(64, 128)).cuda()
    x = torch.randn(2, 16, 32, 64, device="cuda").to(torch.bfloat16)
    ref = m(x)
    out = torch.compile(m, fullgraph=True, backend="aot_eager")(x)
    assert torch.equal(out, ref)
