"""fp32 training path (ops/fp32.py): split-bf16 convolutions on the MFMA kernels vs ATen fp32 and fp64.

Tolerance rule: the split-bf16 result's error against an fp64 reference must be within a small factor of ATen
fp32's own error (and far below bf16's), for forward, data and weight gradients."""
import copy

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, ref):
    return ((a.double() - ref).abs().max() / ref.abs().max()).item()


def _fro(a, ref):
    return ((a.double() - ref).norm() / ref.norm()).item()


@pytest.mark.parametrize("n,h,w,ci,co,k,dil", [
    (2, 24, 40, 3, 64, 3, 1),       # first layer (3 channels: split operand in one 64-channel block)
    (2, 24, 40, 64, 64, 3, 1), (1, 17, 33, 128, 256, 3, 1), (2, 16, 16, 512, 512, 3, 2),
    (2, 12, 20, 512, 512, 1, 1), (2, 12, 20, 64, 1, 1, 1),     # context 1x1, head (Cout 1 padded to 64)
    (2, 1, 1, 512, 512, 1, 1), (3, 2, 2, 512, 512, 1, 1),      # conv1_1 / conv2_1 on the pooled cells
])
def test_conv2d_x3_matches_fp64(n, h, w, ci, co, k, dil):
    from can_distributed_pytorch_amd.ops.fp32 import conv2d_x3
    torch.backends.cudnn.allow_tf32 = False
    torch.manual_seed(0)
    dev = "cuda"
    x = torch.randn(n, ci, h, w, device=dev)
    wt = torch.randn(co, ci, k, k, device=dev) / (ci * k * k) ** 0.5
    b = torch.randn(co, device=dev)
    dy = torch.randn(n, co, h, w, device=dev)
    pad = dil * (k // 2)

    def ref(dtype, dev_):
        xr = x.to(dev_, dtype).requires_grad_(ci != 3)
        wr = wt.to(dev_, dtype).requires_grad_()
        br = b.to(dev_, dtype).requires_grad_()
        y = F.conv2d(xr, wr, br, padding=pad, dilation=dil)
        gs = torch.autograd.grad(y, [t for t in (xr, wr, br) if t.requires_grad], dy.to(dev_, dtype))
        return [y] + list(gs)

    r64 = [t.double().cpu() for t in ref(torch.float64, "cpu")]
    r32 = ref(torch.float32, dev)
    rbf = ref(torch.bfloat16, dev)
    xn = x.permute(0, 2, 3, 1).contiguous().requires_grad_(ci != 3)
    wn = wt.clone().requires_grad_()
    bn = b.clone().requires_grad_()
    y = conv2d_x3(xn, wn, bn, dil)
    gs = torch.autograd.grad(y, [t for t in (xn, wn, bn) if t.requires_grad], dy.permute(0, 2, 3, 1).contiguous())
    ours = [y.permute(0, 3, 1, 2)] + ([gs[0].permute(0, 3, 1, 2)] if ci != 3 else []) + list(gs[-2:])
    names = ["y"] + (["dx"] if ci != 3 else []) + ["dw", "db"]
    for name, o, a32, abf, a64 in zip(names, ours, r32, rbf, r64):
        e_ours, e32, ebf = _rel(o.cpu(), a64), _rel(a32.cpu(), a64), _rel(abf.float().cpu(), a64)
        assert e_ours <= max(8 * e32, 2e-5), f"{name}: split-bf16 err {e_ours:.2e} vs ATen fp32 {e32:.2e}"
        assert e_ours < ebf / 20, f"{name}: split-bf16 err {e_ours:.2e} not well below bf16 {ebf:.2e}"


def test_fp32_stepper_matches_torch_fp32_step():
    """One full training step (forward, MSE(sum), backward) of Fp32Stepper and of the ATen fp32 TorchStepper
    from the same weights, both against an fp64 CPU reference: the loss and every parameter gradient of the
    split-bf16 step are within a small factor of ATen fp32's own error."""
    from can_distributed_pytorch_amd.engine.trainer import Fp32Stepper, TorchStepper
    from can_distributed_pytorch_amd.models import CANNet
    from can_distributed_pytorch_amd.data.synthetic import make_synthetic_batch
    torch.backends.cudnn.allow_tf32 = False
    torch.manual_seed(1)
    dev = torch.device("cuda", 0)
    base = CANNet(backend="torch")
    for m in base.modules():
        if isinstance(m, torch.nn.Conv2d):
            torch.nn.init.normal_(m.weight, std=(2.0 / (m.in_channels * m.kernel_size[0] ** 2)) ** 0.5)
    img, gt = make_synthetic_batch(2, 128, 192, seed=3, device=dev)
    m64 = copy.deepcopy(base).double()
    l64 = torch.nn.functional.mse_loss(m64(img.cpu().double()), gt.cpu().double(), reduction="sum")
    l64.backward()
    ref = TorchStepper(dev, dtype="fp32", lr=1e-9, model=copy.deepcopy(base))
    amp = TorchStepper(dev, dtype="bf16", lr=1e-9, model=copy.deepcopy(base))
    ours = Fp32Stepper(dev, lr=1e-9, model=copy.deepcopy(base))
    l_ref = float(ref.step(img, gt))
    amp.step(img, gt)
    l_ours = float(ours.step(img, gt))
    e_ref, e_ours = abs(l_ref - l64.item()) / l64.item(), abs(l_ours - l64.item()) / l64.item()
    assert e_ours <= max(4 * e_ref, 1e-5), (l_ours, l_ref, l64.item())
    rows = []
    for (name, p64), p_ref, p_amp, p_ours in zip(m64.named_parameters(), ref.model.parameters(),
                                                 amp.model.parameters(), ours.model.parameters()):
        # the step leaves this step's gradients in .grad (zero_grad runs at the start of the next one)
        g = p64.grad
        e = [(_rel(q.float().cpu(), g), _fro(q.float().cpu(), g)) for q in (p_ours.grad, p_ref.grad, p_amp.grad)]
        rows.append((name, e))
    for name, e in rows:
        print(f"{name:22s} max-rel / fro-rel  split-bf16 {e[0][0]:.1e} {e[0][1]:.1e}  aten-fp32 {e[1][0]:.1e} "
              f"{e[1][1]:.1e}  autocast-bf16 {e[2][0]:.1e} {e[2][1]:.1e}")
    for name, e in rows:
        # ~17 significant bits per product (ops/fp32.py): a handful of ReLU units near 0 flip against fp64 where
        # ATen fp32 (24 bits) flips none, so the bound is against autocast bf16 (8 bits) plus a fixed floor
        (mo, fo), (m32, f32), (mbf, fbf) = e
        assert fo <= max(fbf / 8, 16 * f32), f"{name}: split-bf16 grad fro err {fo:.2e} (bf16 {fbf:.2e})"
        assert mo <= max(mbf / 3, 16 * m32), f"{name}: split-bf16 grad max err {mo:.2e} (bf16 {mbf:.2e})"
