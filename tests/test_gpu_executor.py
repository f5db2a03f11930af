"""Native executor (HIP kernels end to end) vs the fp32 ATen reference graph of the reference model."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _models(seed=0):
    from can_distributed_pytorch_amd.models import CANNet
    torch.manual_seed(seed)
    ref = CANNet(backend="torch")
    # larger-than-default init so the signal survives 16 ReLU layers in a short test
    for m in ref.modules():
        if isinstance(m, torch.nn.Conv2d):
            fan_in = m.in_channels * m.kernel_size[0] * m.kernel_size[1]
            torch.nn.init.normal_(m.weight, std=(2.0 / fan_in) ** 0.5)
            if m.bias is not None:
                torch.nn.init.uniform_(m.bias, -0.05, 0.05)
    nat = copy.deepcopy(ref)
    nat.exec_backend = "hip"
    # the reference sees what the native path sees: bf16 conv weights, bf16 activations
    with torch.no_grad():
        for m in ref.modules():
            if isinstance(m, torch.nn.Conv2d) and m.kernel_size == (3, 3):
                m.weight.copy_(m.weight.to(torch.bfloat16).float())
    for m in list(ref.frontend) + list(ref._modules["backend"]):
        if isinstance(m, (torch.nn.ReLU, torch.nn.MaxPool2d)):
            m.register_forward_hook(lambda mod, inp, out: out.to(torch.bfloat16).float())
    return ref.cuda(), nat.cuda()


@pytest.mark.parametrize("n,h,w", [(2, 64, 96), (1, 72, 120)])
def test_executor_forward(n, h, w):
    ref, nat = _models()
    x = torch.randn(n, 3, h, w, device="cuda")
    with torch.no_grad():
        yr = ref(x.to(torch.bfloat16).float())
        yn = nat(x)
    assert yn.shape == yr.shape == (n, 1, h // 8, w // 8)
    assert _rel(yn, yr) < 0.03, _rel(yn, yr)


def test_executor_backward_grads():
    ref, nat = _models(1)
    n, h, w = 2, 64, 96
    x = torch.randn(n, 3, h, w, device="cuda")
    gt = torch.rand(n, 1, h // 8, w // 8, device="cuda")
    crit = torch.nn.MSELoss(reduction="sum")
    lr_ = crit(ref(x.to(torch.bfloat16).float()), gt)
    lr_.backward()
    ln = crit(nat(x), gt)
    ln.backward()
    assert abs(ln.item() - lr_.item()) / abs(lr_.item()) < 0.05
    bad = []
    for (name, pr), pn in zip(ref.named_parameters(), nat.parameters()):
        e = _rel(pn.grad, pr.grad)
        if e > 0.08:
            bad.append((name, e))
    assert not bad, bad


def test_native_stepper_matches_torch_sgd():
    """One fused native step (head+loss fused, flat arena, fused SGD) == torch SGD on the same grads."""
    from can_distributed_pytorch_amd.engine.native import NativeStepper
    ref, nat = _models(2)
    n, h, w = 2, 64, 64
    x = torch.randn(n, 3, h, w, device="cuda")
    gt = torch.rand(n, 1, h // 8, w // 8, device="cuda")
    lr = 1e-5
    opt = torch.optim.SGD(ref.parameters(), lr=lr, momentum=0.95)
    for _ in range(2):
        opt.zero_grad()
        torch.nn.MSELoss(reduction="sum")(ref(x.to(torch.bfloat16).float()), gt).backward()
        opt.step()
    st = NativeStepper("cuda", lr=lr, graph=False, model=nat)
    for _ in range(2):
        st.step(x, gt)
    torch.cuda.synchronize()
    assert not st.nonfinite()
    bad = []
    p0 = dict(_models(2)[0].named_parameters())
    for (name, pr), pn in zip(ref.named_parameters(), nat.parameters()):
        d_ref = pr.detach() - p0[name].detach()
        d_nat = pn.detach() - p0[name].detach()
        e = _rel(d_nat, d_ref)
        if e > 0.1:
            bad.append((name, e))
    assert not bad, bad


def test_native_stepper_graph_replay_equals_eager():
    from can_distributed_pytorch_amd.engine.native import NativeStepper
    _, nat_a = _models(3)
    nat_b = copy.deepcopy(nat_a)
    n, h, w = 1, 64, 64
    x = torch.randn(n, 3, h, w, device="cuda")
    gt = torch.rand(n, 1, h // 8, w // 8, device="cuda")
    a = NativeStepper("cuda", lr=1e-4, graph=False, model=nat_a)
    b = NativeStepper("cuda", lr=1e-4, graph=True, model=nat_b)
    for _ in range(3):
        la = a.step(x, gt)
        lb = b.step(x, gt)
    torch.cuda.synchronize()
    for pa, pb in zip(nat_a.parameters(), nat_b.parameters()):
        assert torch.equal(pa, pb)
    assert float(la) == float(lb)
