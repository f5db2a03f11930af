#!/usr/bin/env python
"""Per-layer conv kernel micro-benchmark: our gfx950 MFMA kernels vs MIOpen
(torch conv2d, channels_last bf16), CANNet layer shapes at batch B, HxW input.

Prints one line per (layer, pass) with ms and TF/s; --json writes a summary.
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from can_distributed_pytorch_amd.ops import conv as C  # noqa: E402

LAYERS = [  # name, cin, cout, res_div, dil
    ("F2", 64, 64, 1, 1), ("F3", 64, 128, 2, 1), ("F4", 128, 128, 2, 1), ("F5", 128, 256, 4, 1),
    ("F6", 256, 256, 4, 1), ("F8", 256, 512, 8, 1), ("F9", 512, 512, 8, 1), ("B1", 1024, 512, 8, 2),
    ("B2", 512, 512, 8, 2), ("B4", 512, 256, 8, 2), ("B5", 256, 128, 8, 2), ("B6", 128, 64, 8, 2),
]


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
    ap.add_argument("--layers", default="")
    ap.add_argument("--no-ref", action="store_true")
    ap.add_argument("--json", default="")
    ap.add_argument("--halo", action="store_true", help="halo-tiled kernel for the Cin=64 fwd / Cout=64 dgrad layers")
    ap.add_argument("--tile", type=int, default=0, help="forced fwd/dgrad tile config (0 = auto)")
    ap.add_argument("--passes", default="fwd,dgrad,wgrad", help="subset of fwd,dgrad,wgrad")
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dev = "cuda"
    out = []
    ws = C.WgradWorkspace(dev)
    for name, ci, co, rd, dil in LAYERS:
        if a.layers and name not in a.layers.split(","):
            continue
        n, h, w = a.batch, a.height // rd, a.width // rd
        fl = 2.0 * n * h * w * ci * co * 9
        x = torch.randn(n, h, w, ci, device=dev).to(torch.bfloat16)
        dy = torch.randn(n, h, w, co, device=dev).to(torch.bfloat16)
        wt = torch.randn(co, ci, 3, 3, device=dev) * 0.02
        b = torch.zeros(co, device=dev)
        wf, wd = C.pack_weight_fwd(wt), C.pack_weight_dgrad(wt)
        dw = torch.empty_like(wt)
        db = torch.empty(co, device=dev)
        res = {"layer": name, "shape": [n, h, w, ci, co, dil], "gflop": fl / 1e9}
        # --tile >= 20: the v2 kernel with the tile that fits the channel count
        pick = (lambda c: (21 if c % 256 == 0 else (25 if a.tile == 25 else 22) if c % 128 == 0 else 23)
                if a.tile >= 20 else a.tile)
        t, td = pick(co), pick(ci)
        if a.halo and ci == 64 and dil == 1 and co in (64, 128):
            t = 31
        if a.halo and co == 64 and dil == 1 and ci in (64, 128):
            td = 31
        passes = a.passes.split(",")
        it = a.iters
        res["fwd_ms"] = timeit(lambda: C.conv_igemm(x, wf, b, ksize=3, dil=dil, tile=t), it) if "fwd" in passes \
            else float("nan")
        res["dgrad_ms"] = timeit(lambda: C.conv_igemm(dy, wd, None, ksize=3, dil=dil, epi=C.EPI_MASK, mask=x, tile=td),
                                 it) if "dgrad" in passes else float("nan")
        res["wgrad_ms"] = timeit(lambda: C.conv_wgrad(dy, x, dw, db, ksize=3, dil=dil, ws=ws), it) \
            if "wgrad" in passes else float("nan")
        if not a.no_ref:
            xr = x.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
            wr = wt.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
            dyr = dy.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
            res["ref_fwd_ms"] = timeit(lambda: F.conv2d(xr, wr, None, padding=dil, dilation=dil))
            res["ref_dgrad_ms"] = timeit(lambda: torch.ops.aten.convolution_backward(
                dyr, xr, wr, None, (1, 1), (dil, dil), (dil, dil), False, (0, 0), 1, (True, False, False)))
            res["ref_wgrad_ms"] = timeit(lambda: torch.ops.aten.convolution_backward(
                dyr, xr, wr, None, (1, 1), (dil, dil), (dil, dil), False, (0, 0), 1, (False, True, False)))
        for k in ("fwd", "dgrad", "wgrad"):
            if k not in passes:
                continue
            line = f"{name:4s} {k:6s} ours {res[k + '_ms']:7.3f} ms {fl / res[k + '_ms'] / 1e9:7.1f} TF/s"
            if not a.no_ref:
                r = res["ref_" + k + "_ms"]
                line += f" | MIOpen {r:7.3f} ms {fl / r / 1e9:7.1f} TF/s | speedup {r / res[k + '_ms']:5.2f}x"
            print(line, flush=True)
        out.append(res)
        del x, dy
        torch.cuda.empty_cache()
    tot = {k: sum(r[k + "_ms"] for r in out) for k in ("fwd", "dgrad", "wgrad") if k in a.passes.split(",")}
    print("total ours", {k: round(v, 3) for k, v in tot.items()})
    if not a.no_ref:
        rt = {k: sum(r["ref_" + k + "_ms"] for r in out) for k in ("fwd", "dgrad", "wgrad")}
        print("total MIOpen", {k: round(v, 3) for k, v in rt.items()})
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
