"""Per-parameter gradients: fused native step (arena) vs the executor's autograd path, same weights/input."""
import copy
import sys
import torch
sys.path.insert(0, ".")
from can_distributed_pytorch_amd.models import CANNet
from can_distributed_pytorch_amd.engine.native import NativeStepper

torch.manual_seed(2)
ref = CANNet(backend="torch")
for m in ref.modules():
    if isinstance(m, torch.nn.Conv2d):
        fan_in = m.in_channels * m.kernel_size[0] * m.kernel_size[1]
        torch.nn.init.normal_(m.weight, std=(2.0 / fan_in) ** 0.5)
        if m.bias is not None:
            torch.nn.init.uniform_(m.bias, -0.05, 0.05)
nat = copy.deepcopy(ref).cuda()
nat.exec_backend = "hip"
n, h, w = 2, 64, 64
x = torch.randn(n, 3, h, w, device="cuda")
gt = torch.rand(n, 1, h // 8, w // 8, device="cuda")
ag = []
for rep in range(2):
    nat2 = copy.deepcopy(nat)
    et = nat2(x)
    torch.nn.MSELoss(reduction="sum")(et, gt).backward()
    ag.append(([p.grad.clone() for p in nat2.parameters()], et.detach().clone()))
names = [nm for nm, _ in nat.named_parameters()]
d = max(((a - b).norm() / (b.norm() + 1e-30)).item() for a, b in zip(ag[0][0], ag[1][0]))
print("autograd rep-to-rep max rel diff", d)
st = NativeStepper("cuda", lr=0.0, graph=False, model=copy.deepcopy(nat))
b6, sv = st.ex.forward_features(x, save=True)
st.ex.workspace(*st.ex.input_hw(x))
loss, et_f, d_b6 = st.ex.head_train(b6, gt, st.grads, flags=st.flags)
torch.cuda.synchronize()
print("et fused vs autograd max abs", (et_f - ag[0][1]).abs().max().item())
g = 2 * (ag[0][1] - gt)
nn_, hh, ww, c = b6.shape
hw_ = st.ex.head.weight.detach().view(1, c)
d_ref = (g.reshape(nn_, hh, ww, 1) * hw_ * (b6.float() > 0)).to(torch.bfloat16)
print("d_b6 fused vs torch-formula: mismatching elements", (d_b6 != d_ref).sum().item(), "of", d_b6.numel())
st.ex.backward_features(sv, d_b6, st.grads)
torch.cuda.synchronize()
worst = sorted((((gg - a).norm() / (a.norm() + 1e-30)).item(), nm) for nm, gg, a in zip(names, st.grads, ag[0][0]))[::-1]
print("fused vs autograd", worst[:6])
