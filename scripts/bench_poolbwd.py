"""Time the pooled layers' data gradients at batch 8 x 768 x 1024: the max-pool backward fused into the epilogue
(EPI_POOLBWD: the full-resolution gradient written, 3 of 4 window positions zero) vs the plain masked data
gradient at the pooled resolution (EPI_MASK), i.e. what the 4x scatter store costs."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from can_distributed_pytorch_amd.ops import conv as C

# name: (pooled H, W, dgrad input channels (the conv's Cout), dgrad output channels (its Cin))
LAYERS = {"F3 conv2_1": (384, 512, 128, 64), "F5 conv3_1": (192, 256, 256, 128), "F8 conv4_1": (96, 128, 512, 256)}


def timeit(fn, iters=20):
    for _ in range(5):
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
    n = 8
    for name, (h, w, ci, co) in LAYERS.items():
        dy = torch.randn(n, h, w, ci, device="cuda").to(torch.bfloat16)
        dgr = C.pack_weight_dgrad(torch.randn(ci, co, 3, 3, device="cuda") * 0.05)
        full = torch.relu(torch.randn(n, 2 * h, 2 * w, co, device="cuda")).to(torch.bfloat16)
        _, codes = C.maxpool_codes(full)
        mask = torch.randn(n, h, w, co, device="cuda").to(torch.bfloat16)
        t_pb = timeit(lambda: C.conv_dgrad_with_bias(dy, dgr, ksize=3, epi=C.EPI_POOLBWD, mask=codes))
        t_mk = timeit(lambda: C.conv_dgrad_with_bias(dy, dgr, ksize=3, epi=C.EPI_MASK, mask=mask))
        print(json.dumps({"layer": name, "poolbwd_ms": round(t_pb, 4), "mask_ms": round(t_mk, 4),
                          "scatter_MB": round(n * 4 * h * w * co * 2 / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
