import copy, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_gpu_executor import _models, _rel  # noqa
for seed in range(6):
    ref, nat = _models(seed)
    g = torch.Generator(device="cuda").manual_seed(100 + seed)
    x = torch.randn(2, 3, 64, 96, device="cuda", generator=g)
    r64 = copy.deepcopy(ref).cpu().double()
    am = copy.deepcopy(ref).to(memory_format=torch.channels_last)
    with torch.no_grad():
        y64 = r64(x.cpu().double())
        yn = nat(x)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            ya = am(x.contiguous(memory_format=torch.channels_last))
        # bf16 emulation: round every conv output (post-ReLU) like the native path
        em = copy.deepcopy(ref)
        hooks = [mm.register_forward_hook(lambda mod, i, o: o.to(torch.bfloat16).float())
                 for mm in list(em.frontend) + list(em._modules["backend"]) if isinstance(mm, torch.nn.ReLU)]
        with torch.no_grad():
            for mm in em.modules():
                if isinstance(mm, torch.nn.Conv2d) and mm.kernel_size == (3, 3):
                    mm.weight.copy_(mm.weight.to(torch.bfloat16).float())
        ye = em(x.to(torch.bfloat16).float())
    print(f"seed {seed}: native {_rel(yn.cpu().double(), y64):.3e}  autocast {_rel(ya.float().cpu().double(), y64):.3e} "
          f"(dtype {ya.dtype})  emulated-bf16 {_rel(ye.cpu().double(), y64):.3e}  native-vs-emul {_rel(yn, ye):.3e}")
