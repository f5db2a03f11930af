import copy, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from can_distributed_pytorch_amd.models import CANNet  # noqa
torch.manual_seed(0)
m = CANNet(backend="hip").cuda()
for mod in m.modules():
    if isinstance(mod, torch.nn.Conv2d):
        fan = mod.in_channels * mod.kernel_size[0] * mod.kernel_size[1]
        torch.nn.init.normal_(mod.weight, std=(2.0 / fan) ** 0.5)
x = torch.randn(2, 3, 64, 96, device="cuda")
y_grad = m(x).detach()
with torch.no_grad():
    y_eval = m(x)
    ex = m._executor
    b6, sv = ex.forward_features(x, save=True)
    y_save = ex.head_forward(b6)
    b6b, _ = ex.forward_features(x, save=False)
    y_nosave = ex.head_forward(b6b)
torch.cuda.synchronize()
print("grad vs eval", (y_grad - y_eval).abs().max().item())
print("save vs nosave", (y_save - y_nosave).abs().max().item(), "b6", (b6.float() - b6b.float()).abs().max().item())
print("grad vs save", (y_grad - y_save).abs().max().item())
