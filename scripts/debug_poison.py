import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_gpu_executor import _models, _rel  # noqa

def poison(val_bits):
    t = torch.empty(512 * 1024 * 1024 // 4, dtype=torch.int32, device="cuda")
    t.fill_(val_bits)
    del t
    torch.cuda.synchronize()

for name, bits in (("zeros", 0), ("ones_bf16", 0x3f803f80), ("big", 0x7f007f00), ("nan", 0x7fc07fc0)):
    ref, nat = _models(2)
    g = torch.Generator(device="cuda").manual_seed(102)
    x = torch.randn(2, 3, 64, 96, device="cuda", generator=g)
    with torch.no_grad():
        yr = ref(x)
        poison(bits)
        yn = nat(x)
    torch.cuda.synchronize()
    print(f"poison={name:10s} native vs ref {_rel(yn, yr):.3e}  nan={bool(torch.isnan(yn).any())}")
