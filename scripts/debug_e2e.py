#!/usr/bin/env python
"""E2E forward/grad error of native / autocast-bf16 / GPU-fp32 against a CPU float64 oracle."""
import copy, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from can_distributed_pytorch_amd.models import CANNet  # noqa

def rel(a, b):
    return ((a.double().cpu() - b.double().cpu()).norm() / (b.double().cpu().norm() + 1e-30)).item()

torch.manual_seed(0)
m = CANNet(backend="torch")
for mod in m.modules():
    if isinstance(mod, torch.nn.Conv2d):
        fan = mod.in_channels * mod.kernel_size[0] * mod.kernel_size[1]
        torch.nn.init.normal_(mod.weight, std=(2.0 / fan) ** 0.5)
        if mod.bias is not None:
            torch.nn.init.uniform_(mod.bias, -0.05, 0.05)
x = torch.randn(2, 3, 64, 96)
gt = torch.rand(2, 1, 8, 12) * 4
crit = torch.nn.MSELoss(reduction="sum")
m64 = copy.deepcopy(m).double()
y64 = m64(x.double()); crit(y64, gt.double()).backward()
g64 = [p.grad for p in m64.parameters()]
res = {}
for tf32 in (True, False):
    torch.backends.cudnn.allow_tf32 = tf32
    torch.backends.cuda.matmul.allow_tf32 = tf32
    mg = copy.deepcopy(m).cuda()
    y = mg(x.cuda()); crit(y, gt.cuda()).backward()
    res[f"gpu_fp32_tf32={tf32}"] = (rel(y, y64), [rel(p.grad, g) for p, g in zip(mg.parameters(), g64)])
ma = copy.deepcopy(m).cuda().to(memory_format=torch.channels_last)
with torch.autocast("cuda", dtype=torch.bfloat16):
    ya = ma(x.cuda().contiguous(memory_format=torch.channels_last)).float()
crit(ya, gt.cuda()).backward()
res["autocast_bf16"] = (rel(ya, y64), [rel(p.grad, g) for p, g in zip(ma.parameters(), g64)])
mn = copy.deepcopy(m).cuda(); mn.exec_backend = "hip"
yn = mn(x.cuda()); crit(yn, gt.cuda()).backward()
res["native_bf16"] = (rel(yn, y64), [rel(p.grad, g) for p, g in zip(mn.parameters(), g64)])
names = [n for n, _ in m.named_parameters()]
for k, (fe, ge) in res.items():
    print(f"{k:22s} fwd {fe:.3e}  grad median {sorted(ge)[len(ge)//2]:.3e} max {max(ge):.3e} ({names[ge.index(max(ge))]})")
print("per-param grad err (native / autocast):")
for i, n in enumerate(names):
    print(f"  {n:22s} {res['native_bf16'][1][i]:.3e} {res['autocast_bf16'][1][i]:.3e}")
