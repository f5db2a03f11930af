#!/usr/bin/env python
"""Layer-by-layer check of the native executor's forward: each stage is
recomputed in fp32 PyTorch from the executor's OWN input to that stage, so
errors do not accumulate and the first broken stage stands out."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from can_distributed_pytorch_amd.models import CANNet  # noqa: E402
from can_distributed_pytorch_amd.ops.executor import CANNetExecutor  # noqa: E402


def rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def main():
    n, h, w = 2, int(sys.argv[1]) if len(sys.argv) > 1 else 64, int(sys.argv[2]) if len(sys.argv) > 2 else 96
    if len(sys.argv) > 3 and sys.argv[3] == "test":
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
        from test_gpu_executor import _models
        _, m = _models()
    else:
        torch.manual_seed(0)
        m = CANNet().cuda()
        for mod in m.modules():
            if isinstance(mod, torch.nn.Conv2d):
                fan = mod.in_channels * mod.kernel_size[0] * mod.kernel_size[1]
                torch.nn.init.normal_(mod.weight, std=(2.0 / fan) ** 0.5)
                if mod.bias is not None:
                    torch.nn.init.uniform_(mod.bias, -0.05, 0.05)
    ex = CANNetExecutor(m)
    x = torch.randn(n, 3, h, w, device="cuda")
    with torch.no_grad():
        b6, sv = ex.forward_features(x, save=True)
        nchw = lambda t: t.float().permute(0, 3, 1, 2)  # noqa: E731
        x4 = sv["front_in"][0]
        print("img_to_nhwc4", rel(nchw(x4[..., :3].contiguous()), x.to(torch.bfloat16).float()),
              "pad channel zero:", bool((x4[..., 3] == 0).all()))
        for s in ex.front:
            inp = sv["front_in"][s.idx]
            xin = nchw(inp[..., :3].contiguous()) if s.first else nchw(inp)
            wq = s.module.weight.to(torch.bfloat16).float()
            ref = torch.relu(F.conv2d(xin, wq, s.module.bias, padding=1))
            if s.pool_after:
                got = sv["pre_pool"][s.idx]
                print(f"front conv{s.idx} (pre-pool) rel {rel(nchw(got), ref):.2e}")
                nxt = sv["front_in"][s.idx + 1] if s.idx + 1 < len(ex.front) else sv["fv"]
                print(f"front pool{s.idx}            rel {rel(nchw(nxt), F.max_pool2d(nchw(got), 2)):.2e}")
            else:
                nxt = sv["front_in"][s.idx + 1] if s.idx + 1 < len(ex.front) else sv["fv"]
                print(f"front conv{s.idx}            rel {rel(nchw(nxt), ref):.2e}")
        fv = sv["fv"]
        cat = sv["back_in"][0]
        fvr = nchw(fv)
        num = den = None
        for sc in (1, 2, 3, 6):
            ave = F.conv2d(F.adaptive_avg_pool2d(fvr, (sc, sc)), getattr(m, f"conv{sc}_1").weight)
            up = F.interpolate(ave, size=fvr.shape[2:], mode="bilinear", align_corners=True)
            wt = torch.sigmoid(F.conv2d(up - fvr, getattr(m, f"conv{sc}_2").weight.to(torch.bfloat16).float()))
            num = wt * up if num is None else num + wt * up
            den = wt if den is None else den + wt
        print(f"context cat             rel {rel(nchw(cat), torch.cat((fvr, num / (den + 1e-12)), 1)):.2e}")
        for s in ex.back:
            inp = sv["back_in"][s.idx]
            ref = torch.relu(F.conv2d(nchw(inp), s.module.weight.to(torch.bfloat16).float(), s.module.bias,
                                      padding=s.dil, dilation=s.dil))
            nxt = sv["back_in"][s.idx + 1] if s.idx + 1 < len(ex.back) else b6
            print(f"back conv{s.idx} d{s.dil}          rel {rel(nchw(nxt), ref):.2e}")
        et = ex.head_forward(b6)
        print(f"head                    rel {rel(et, F.conv2d(nchw(b6), m.output_layer.weight, m.output_layer.bias)):.2e}")


if __name__ == "__main__":
    main()
