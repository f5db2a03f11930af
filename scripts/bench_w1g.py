"""Time conv1_2's data gradient at batch 8 x 768 x 1024: plain (ws64, EPI_MASK, dX stored) vs with conv1_1's weight
gradient fused (conv_dgrad_w1g, dX not stored, + its slab reduction), and conv1_1's separate weight gradient."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from can_distributed_pytorch_amd.ops import conv as C


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    torch.manual_seed(0)
    n, h, w = 8, 768, 1024
    dy = torch.randn(n, h, w, 64, device="cuda").to(torch.bfloat16)
    mask = torch.randn(n, h, w, 64, device="cuda").to(torch.bfloat16)
    img = C.to_nhwc4(torch.randn(n, 3, h, w, device="cuda"))
    wt = torch.randn(64, 64, 3, 3, device="cuda") * 0.05
    dgr = C.pack_weight_dgrad(wt)
    dw1 = torch.empty(64, 3, 3, 3, device="cuda")
    db1 = torch.empty(64, device="cuda")
    cap = C.w1g_slab_cap(dy.device)
    sl = torch.empty(cap, 36 * 64, device="cuda")
    bsl = torch.empty(cap, 64, device="cuda")
    x1 = torch.relu(mask)
    for rnd in range(2):
        res = {
            "round": rnd,
            "dgrad_plain_ms": timeit(lambda: C.conv_igemm(dy, dgr, None, ksize=3, epi=C.EPI_MASK, mask=mask)),
            "dgrad_w1g_ms": timeit(lambda: C.conv_dgrad_w1g(dy, dgr, mask, img, dw1, db1, slabs=sl, bslabs=bsl)),
            "conv1_1_wgrad_ms": timeit(lambda: C.conv_wgrad(x1, img, dw1, db1, ksize=3, first=True)),
        }
        print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
