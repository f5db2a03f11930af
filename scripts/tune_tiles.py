#!/usr/bin/env python
"""Per-layer tile search for the forward / data-gradient conv kernels of one CANNet training shape.

For every 3x3 conv of the step (forward with its real epilogue: bias+ReLU, or bias+ReLU+2x2 pool for the layers a
pool follows; data gradient with ReLU mask, pool-backward or plain for backend.0) every tile config the kernels
accept is timed in isolation (CUDA events, interleaved rounds, median), next to the config the default dispatch
picks.  Writes a JSON table {key: {"best": cfg, "ms": {cfg: ms}}} that ops/tiles.py can load.

usage: python scripts/tune_tiles.py --batch 8 --height 768 --width 1024 --out gpurun_out/tiles_768x1024.json
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from can_distributed_pytorch_amd.ops import conv as C  # noqa: E402
from can_distributed_pytorch_amd.ops import _ext  # noqa: E402

# name, cin, cout, resolution divisor, dilation, pool after (forward), pool before (data gradient goes through it)
LAYERS = [
    ("conv2_1", 64, 128, 2, 1, False, True), ("conv2_2", 128, 128, 2, 1, True, False),
    ("conv3_1", 128, 256, 4, 1, False, True), ("conv3_2", 256, 256, 4, 1, False, False),
    ("conv3_3", 256, 256, 4, 1, True, False), ("conv4_1", 256, 512, 8, 1, False, True),
    ("conv4_2", 512, 512, 8, 1, False, False), ("conv4_3", 512, 512, 8, 1, False, False),
    ("back0", 1024, 512, 8, 2, False, False), ("back1", 512, 512, 8, 2, False, False),
    ("back3", 512, 256, 8, 2, False, False), ("back4", 256, 128, 8, 2, False, False),
    ("back5", 128, 64, 8, 2, False, False),
]
FWD_CFGS = (21, 22, 23, 25, 27, 28, 29)


def timeit(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
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
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    ext = _ext.require()
    dev = "cuda"
    table = {}
    for name, ci, co, rd, dil, pool_after, pool_before in LAYERS:
        n, h, w = a.batch, a.height // rd, a.width // rd
        torch.manual_seed(0)
        x = torch.relu(torch.randn(n, h, w, ci, device=dev)).to(torch.bfloat16)
        wt = torch.randn(co, ci, 3, 3, device=dev) * (2.0 / (9 * ci)) ** 0.5
        b = torch.zeros(co, device=dev)
        wf, wd = C.pack_weight_fwd(wt), C.pack_weight_dgrad(wt)
        dy = torch.randn(n, h, w, co, device=dev).to(torch.bfloat16)
        passes = {}
        # forward with the step's epilogue
        if pool_after:
            fwd_epi = "poolfwd"
            passes[fwd_epi] = lambda t: C.conv_pool_fwd(x, wf, b, ksize=3, dil=dil, tile=t, keep_full=False,
                                                        codes=True)
        else:
            fwd_epi = "relu"
            passes[fwd_epi] = lambda t: C.conv_igemm(x, wf, b, ksize=3, dil=dil, tile=t)
        # data gradient with the step's epilogue (dX has ci channels)
        if name == "back0":
            passes["none"] = lambda t: C.conv_igemm(dy, wd, None, ksize=3, dil=dil, epi=C.EPI_NONE, tile=t)
        elif pool_before:
            full = torch.relu(torch.randn(n, 2 * h, 2 * w, ci, device=dev)).to(torch.bfloat16)
            _, codes = C.maxpool_codes(full)
            del full
            passes["poolbwd"] = lambda t: C.conv_dgrad_with_bias(dy, wd, ksize=3, dil=dil, epi=C.EPI_POOLBWD,
                                                                 mask=codes, tile=t)
        else:
            passes["mask"] = lambda t: C.conv_dgrad_with_bias(dy, wd, ksize=3, dil=dil, epi=C.EPI_MASK, mask=x,
                                                              tile=t)
        for epi, fn in passes.items():
            cout = ci if epi in ("none", "poolbwd", "mask") else co
            cin = co if epi in ("none", "poolbwd", "mask") else ci
            epi_code = {"relu": 0, "poolfwd": 6, "none": 2, "poolbwd": 5, "mask": 1}[epi]
            default = ext.conv_plan(h, w, cin, cout, 3, dil, epi_code)
            ok = {}
            for cfg in (0,) + FWD_CFGS:
                try:
                    fn(cfg)
                    torch.cuda.synchronize()
                    ok[cfg] = []
                except (RuntimeError, ValueError):
                    pass
            for _ in range(a.rounds):
                for cfg in ok:
                    ok[cfg].append(timeit(lambda: fn(cfg), a.iters))
            med = {cfg: statistics.median(v) for cfg, v in ok.items()}
            best = min((c for c in med if c != 0), key=lambda c: med[c])
            key = f"{n}x{h}x{w}x{cin}x{cout}x{dil}x{epi}"
            table[key] = {"layer": name, "default": default, "best": best,
                          "ms": {str(c): round(v, 4) for c, v in sorted(med.items())}}
            print(f"{name:8s} {epi:8s} default cfg {default:2d} (auto {med[0]:.4f} ms) best cfg {best} "
                  f"{med[best]:.4f} ms  " + " ".join(f"{c}:{v:.4f}" for c, v in sorted(med.items()) if c), flush=True)
        del x, dy
        torch.cuda.empty_cache()
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(table, f, indent=1)


if __name__ == "__main__":
    main()
