import copy, os, sys
import torch, torch.nn.functional as F
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_gpu_executor import _models, _rel  # noqa
ref, nat = _models(2)
g = torch.Generator(device="cuda").manual_seed(102)
x = torch.randn(2, 3, 64, 96, device="cuda", generator=g)
cap = {}
last_relu = list(ref._modules["backend"])[-1]
last_relu.register_forward_hook(lambda m, i, o: cap.__setitem__("b6", o.detach().clone()))
fvmod = list(ref.frontend)[-1]
fvmod.register_forward_hook(lambda m, i, o: cap.__setitem__("fv", o.detach().clone()))
with torch.no_grad():
    yr = ref(x)
    yn = nat(x)
    ex = nat._executor
    b6n, sv = ex.forward_features(x, save=True)
    yn2 = ex.head_forward(b6n)
nchw = lambda t: t.float().permute(0, 3, 1, 2)
print("y rel", _rel(yn, yr), "y2 rel", _rel(yn2, yr))
print("fv rel", _rel(nchw(sv["fv"]), cap["fv"]))
print("b6 rel", _rel(nchw(b6n), cap["b6"]))
hr = F.conv2d(cap["b6"], ref.output_layer.weight, ref.output_layer.bias)
hn = F.conv2d(nchw(b6n), ref.output_layer.weight, ref.output_layer.bias)
print("head(ref b6) vs yr", _rel(hr, yr), " head(nat b6) vs yn", _rel(hn, yn), " head(nat b6) vs yr", _rel(hn, yr))
d = (nchw(b6n) - cap["b6"])
print("per-channel b6 err (top 8):", sorted([(round((d[:, c].norm() / (cap['b6'][:, c].norm() + 1e-9)).item(), 4), c) for c in range(64)], reverse=True)[:8])
print("w.dot per-channel err contribution:", (ref.output_layer.weight.view(64, 1, 1) * d[0]).sum(0).abs().mean().item(), "vs |y|", yr.abs().mean().item())
print("nat head w vs ref head w", (nat.output_layer.weight - ref.output_layer.weight).abs().max().item(), (nat.output_layer.bias - ref.output_layer.bias).abs().max().item())
for (n1, p1), p2 in zip(ref.named_parameters(), nat.parameters()):
    dd = (p1 - p2).abs().max().item()
    if dd > 0: print("param differs", n1, dd)
