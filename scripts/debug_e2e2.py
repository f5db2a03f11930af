import copy, os, sys
import torch, torch.nn.functional as F
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_gpu_executor import _models, _rel  # noqa
ref, nat = _models()
x = torch.randn(2, 3, 64, 96, device="cuda")
r64 = copy.deepcopy(ref).cpu().double()
with torch.no_grad():
    y64 = r64(x.cpu().double())
    yr = ref(x); yn = nat(x)
print("ref vs fp64", _rel(yr.cpu().double(), y64), "nat vs fp64", _rel(yn.cpu().double(), y64), "nat vs ref", _rel(yn, yr))
print("max|yn-yr|", (yn - yr).abs().max().item(), "argmax", (yn - yr).abs().argmax().item(), "absmax y", yr.abs().max().item())
d = (yn - yr).abs()[0, 0]
print((d > 0.05).nonzero()[:20].tolist())
