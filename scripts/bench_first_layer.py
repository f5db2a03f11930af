"""Time conv1_1 (3 -> 64, NHWC4 input, bias + ReLU) at batch 8 x 768 x 1024 under dispatch first_pf 0 / 1 (one tile per
block vs persistent blocks prefetching the next halo); the kernel is output-write bound (805 MB of bf16 per call)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from can_distributed_pytorch_amd.ops import conv as C
from can_distributed_pytorch_amd.ops import dispatch


def main(iters=20):
    torch.manual_seed(0)
    x4 = C.to_nhwc4(torch.randn(8, 3, 768, 1024, device="cuda"))
    wp = C.pack_weight_first(torch.randn(64, 3, 3, 3, device="cuda") * 0.2)
    b = torch.randn(64, device="cuda")
    ref = None
    for rnd in range(2):
        for st in (0, 1):
            with dispatch.override(first_pf=st):
                y = C.conv_igemm(x4, wp, b, ksize=3, first=True)
                ref = y if ref is None else ref
                same = torch.equal(y, ref)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                for _ in range(iters):
                    C.conv_igemm(x4, wp, b, ksize=3, first=True)
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / iters
            print(json.dumps({"round": rnd, "arm": ["one tile per block", "persistent + LDS-staged stores"][st], "ms": round(ms, 4),
                              "write_TBps": round(y.numel() * 2 / ms / 1e9, 2), "bitwise": same}), flush=True)


if __name__ == "__main__":
    main()
