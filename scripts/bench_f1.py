#!/usr/bin/env python
"""conv1_1 + conv1_2 kernels, stored vs recomputed conv1_1 output (batch 8, 768x1024 by default):
forward, data gradient, weight gradient.  Prints ms per pass for both variants."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from can_distributed_pytorch_amd.ops import conv as C  # noqa: E402


def timeit(fn, iters=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--height", type=int, default=768)
    ap.add_argument("--width", type=int, default=1024)
    a = ap.parse_args()
    n, h, w = a.batch, a.height, a.width
    dt = torch.bfloat16
    x4 = C.to_nhwc4(torch.randn(n, 3, h, w, device="cuda"), dt)
    w1p = C.pack_weight_first(torch.randn(64, 3, 3, 3, device="cuda") * 0.2, dt)
    b1 = torch.randn(64, device="cuda") * 0.1
    w2 = torch.randn(64, 64, 3, 3, device="cuda") * 0.05
    b2 = torch.randn(64, device="cuda") * 0.1
    wf, wd = C.pack_weight_fwd(w2, dt), C.pack_weight_dgrad(w2, dt)
    x2 = C.conv_igemm(x4, w1p, b1, ksize=3, first=True)
    dy = torch.randn(n, h, w, 64, device="cuda").to(dt)
    ws = C.WgradWorkspace("cuda")
    dw, db = torch.empty(64, 64, 3, 3, device="cuda"), torch.empty(64, device="cuda")
    res = {
        "fwd conv1_1 (stored path only)": timeit(lambda: C.conv_igemm(x4, w1p, b1, ksize=3, first=True)),
        "fwd conv1_2 stored": timeit(lambda: C.conv_igemm(x2, wf, b2, ksize=3)),
        "fwd conv1_2 recomputed": timeit(lambda: C.conv_f1(None, wf, b2, x4, w1p, b1, epi=C.EPI_BIAS_RELU)),
        "dgrad conv1_2 stored": timeit(lambda: C.conv_igemm(dy, wd, None, ksize=3, epi=C.EPI_MASK, mask=x2)),
        "dgrad conv1_2 recomputed": timeit(lambda: C.conv_f1(dy, wd, None, x4, w1p, b1, epi=C.EPI_MASK)),
        "wgrad conv1_2 stored": timeit(lambda: C.conv_wgrad(dy, x2, dw, db, ksize=3, ws=ws)),
        "wgrad conv1_2 recomputed": timeit(lambda: C.conv_wgrad_f1(dy, x4, w1p, b1, dw, db, ws=ws)),
    }
    for k, v in res.items():
        print(f"{k:34s} {v:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
