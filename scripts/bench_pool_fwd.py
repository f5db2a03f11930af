"""Time the conv + bias + ReLU + 2x2 max-pool forward kernels of CANNet's pooled layers (conv1_2, conv2_2, conv3_3 at
batch 8 x 768 x 1024) per kernel config: conv_glds2 / halo defaults (tile 0, dispatch rring_pool 0) vs the row ring
(tiles 27 / 29).  What the training step runs: keep_full=False, max-pool codes on."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from can_distributed_pytorch_amd.ops import conv as C
from can_distributed_pytorch_amd.ops import dispatch

LAYERS = {"F2": (768, 1024, 64, 64), "F4": (384, 512, 128, 128), "F7": (192, 256, 256, 256)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    torch.manual_seed(0)
    out = []
    for name, (h, w, ci, co) in LAYERS.items():
        x = torch.randn(args.batch, h, w, ci, device="cuda").to(torch.bfloat16)
        wp = C.pack_weight_fwd(torch.randn(co, ci, 3, 3, device="cuda") * (2.0 / (9 * ci)) ** 0.5)
        b = torch.randn(co, device="cuda") * 0.1
        flops = 2.0 * args.batch * h * w * ci * co * 9
        tiles = [0] + ([29, 22, 25] if co % 128 == 0 and ci > 64 else []) + ([27] if co % 256 == 0 else [])
        ref = None
        for tile in tiles:
            with dispatch.override(rring_pool=0):
                fn = lambda: C.conv_pool_fwd(x, wp, b, ksize=3, tile=tile, keep_full=False, codes=True)
                _, yp, cd = fn()
                if ref is None:
                    ref = (yp, cd)
                same = torch.equal(ref[0], yp) and torch.equal(ref[1], cd)
                for _ in range(3):
                    fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                for _ in range(args.iters):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / args.iters
            rec = {"layer": name, "tile": tile, "ms": round(ms, 4), "tflops": round(flops / ms / 1e9, 1),
                   "bitwise_vs_tile0": same}
            out.append(rec)
            print(json.dumps(rec), flush=True)
        # the same conv without the pool (full-resolution store), default kernel
        fn = lambda: C.conv_igemm(x, wp, b, ksize=3)
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(args.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.iters
        print(json.dumps({"layer": name, "plain_conv_ms": round(ms, 4)}), flush=True)


if __name__ == "__main__":
    main()
