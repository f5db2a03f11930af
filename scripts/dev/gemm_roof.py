#!/usr/bin/env python
"""Library-GEMM throughput (torch.matmul -> hipBLASLt) on the GEMM shapes of CANNet's convolutions, as the
attainable-throughput yardstick for the hand-written conv kernels (same FLOPs, no im2col: the library gets
the operands pre-laid-out, so this is an upper reference, not a like-for-like conv).

usage: python scripts/dev/gemm_roof.py
"""
import json

import torch


def t(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    dev = torch.device("cuda", 0)
    px = 8 * 96 * 128          # 1/8-resolution pixels of a batch-8 768x1024 step
    shapes = {
        "backend fwd/dgrad  [px x 4608] @ [4608 x 512]": (px, 4608, 512),
        "backend wgrad      [512 x px] @ [px x 4608]": (512, px, 4608),
        "F9 fwd  (1/4 res) [4px x 2304] @ [2304 x 256]": (4 * px, 2304, 256),
        "F2 fwd  (full res) [64px x 576] @ [576 x 64]": (64 * px, 576, 64),
        "F2 wgrad [64 x 64px] @ [64px x 576]": (64, 64 * px, 576),
        "square 8192": (8192, 8192, 8192),
    }
    for name, (m, k, n) in shapes.items():
        a = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
        b = torch.randn(k, n, device=dev, dtype=torch.bfloat16)
        ms = t(lambda: torch.matmul(a, b))
        print(json.dumps({"gemm": name, "m": m, "k": k, "n": n, "ms": round(ms, 4),
                          "tflops": round(2 * m * n * k / ms / 1e9, 1)}), flush=True)
        del a, b


if __name__ == "__main__":
    main()
