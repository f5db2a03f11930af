"""Cumulative divergence of native activations from the fp32 reference chain (same x)."""
import os, sys
import torch, torch.nn.functional as F
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_gpu_executor import _models, _rel  # noqa
seed = int(sys.argv[1]) if len(sys.argv) > 1 else 0
ref, nat = _models(seed)
if seed:
    g = torch.Generator(device="cuda").manual_seed(100 + seed)
    x = torch.randn(2, 3, 64, 96, device="cuda", generator=g)
else:
    x = torch.randn(2, 3, 64, 96, device="cuda")
from can_distributed_pytorch_amd.ops.executor import CANNetExecutor
ex = CANNetExecutor(nat)
nchw = lambda t: t.float().permute(0, 3, 1, 2)
with torch.no_grad():
    b6, sv = ex.forward_features(x, save=True)
    # reference chain with hooks
    acts = []
    h = x
    mods = list(ref.frontend)
    i = 0
    for mod in mods:
        h = mod(h)
        if isinstance(mod, torch.nn.ReLU):
            acts.append(h.clone())
    fvr = h
    convs = [s for s in ex.front]
    k = 0
    for s in convs:
        got = sv["pre_pool"][s.idx] if s.pool_after else (sv["front_in"][s.idx + 1] if s.idx + 1 < len(convs) else sv["fv"])
        inp = sv["front_in"][s.idx]
        xin = nchw(inp[..., :3].contiguous()) if s.first else nchw(inp)
        loc = torch.relu(F.conv2d(xin, s.module.weight.to(torch.bfloat16).float(), s.module.bias, padding=1))
        print(f"front conv{s.idx}: cumulative rel {_rel(nchw(got), acts[k]):.3e} local {_rel(nchw(got), loc):.3e} "
              f"max|ref| {acts[k].abs().max().item():.2f}  min/max native {got.float().min().item():.2f}/{got.float().max().item():.2f}")
        k += 1
    fv = sv["fv"]
    print("fv cumulative", _rel(nchw(fv), fvr))
    # context on reference fv
    hh, ww = fvr.shape[2:]
    num = den = None
    for sc in (1, 2, 3, 6):
        ave = F.conv2d(F.adaptive_avg_pool2d(fvr, (sc, sc)), getattr(ref, f"conv{sc}_1").weight)
        up = F.interpolate(ave, size=(hh, ww), mode="bilinear", align_corners=True)
        wt = torch.sigmoid(F.conv2d(up - fvr, getattr(ref, f"conv{sc}_2").weight))
        num = wt * up if num is None else num + wt * up
        den = wt if den is None else den + wt
    catr = torch.cat((fvr, num / (den + 1e-12)), 1)
    print("cat cumulative", _rel(nchw(sv["back_in"][0]), catr), "fi part", _rel(nchw(sv["back_in"][0])[:, 512:], catr[:, 512:]))
    h = catr
    bmods = list(ref._modules["backend"])
    j = 0
    for mod in bmods:
        h = mod(h)
        if isinstance(mod, torch.nn.ReLU):
            got = sv["back_in"][j + 1] if j + 1 < len(ex.back) else b6
            print(f"back conv{j}: cumulative rel {_rel(nchw(got), h):.3e}")
            j += 1
