"""Isolated weight-gradient timings of the 256x256-tile layers at the bench shape (batch 8 at 768x1024) for the
v2 kernel and the deeper-ring v3 kernel (CANNET_WGRAD_RING = 4 / 5).  usage: python scripts/bench_wgrad.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, reps=10, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1000.0


def main():
    from can_distributed_pytorch_amd.ops import conv as C
    layers = [("F6", 8, 192, 256, 256, 256, 1, 3), ("F8", 8, 96, 128, 256, 512, 1, 3),
              ("F9", 8, 96, 128, 512, 512, 1, 3), ("B1", 8, 96, 128, 1024, 512, 2, 3),
              ("B2", 8, 96, 128, 512, 512, 2, 3), ("B4", 8, 96, 128, 512, 256, 2, 3),
              ("ctxW2", 8, 96, 128, 512, 2048, 1, 1)]
    ws = C.WgradWorkspace("cuda")
    for name, n, h, w, ci, co, dil, k in layers:
        x = torch.randn(n, h, w, ci, device="cuda").to(torch.bfloat16)
        dy = torch.randn(n, h, w, co, device="cuda").to(torch.bfloat16)
        dw = torch.empty(co, ci, k, k, device="cuda")
        db = torch.empty(co, device="cuda")
        gf = 2.0 * n * h * w * ci * co * k * k / 1e9
        out = []
        for ring in ("0", "4", "5"):
            os.environ["CANNET_WGRAD_RING"] = ring
            t = timeit(lambda: C.conv_wgrad(dy, x, dw, db, ksize=k, dil=dil, ws=ws))
            out.append(f"ring {ring}: {t:7.1f} us {gf / t * 1e3:7.1f} TF/s")
        print(f"{name:6s} " + " | ".join(out), flush=True)


if __name__ == "__main__":
    main()
