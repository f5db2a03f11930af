"""Time the weight-gradient kernels with parts of their mainloop removed (scripts/probe/build_wprobe.sh builds
the variants): probe0 = full kernel, 1 = no DMA, 2 = no LDS fragment reads, 3 = neither (MFMA + VALU +
barriers + epilogue).  Layers F2/F3/F4 (ring kernel) and F9/B1 (v2 256x256 kernel), batch 8, 768x1024.
Each line: ms per call (GEMM + slab reduction) and TF/s of the GEMM FLOPs; arms interleaved over 3 rounds."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from can_distributed_pytorch_amd.ops import conv as C  # noqa: E402

SHAPES = [("F2", 64, 64, 768, 1024, 1), ("F3", 64, 128, 384, 512, 1), ("F4", 128, 128, 384, 512, 1),
          ("F9", 512, 512, 96, 128, 1), ("B1", 1024, 512, 96, 128, 2)]


def main():
    fns = {}
    for m in range(4):
        lib = ctypes.CDLL(os.path.join(ROOT, "scripts", "probe", "bin", f"wgrad_probe{m}.so"))
        f = lib.can_conv_wgrad
        f.restype = ctypes.c_int
        f.argtypes = ([ctypes.c_void_p] * 6 + [ctypes.c_int] * 11 + [ctypes.c_float] * 2 + [ctypes.c_void_p] +
                      [ctypes.c_int] + [ctypes.c_void_p] * 2 + [ctypes.c_int])
        fns[m] = f
    n = 8
    ws = C.WgradWorkspace("cuda")
    st = torch.cuda.current_stream().cuda_stream
    for name, ci, co, h, w, dil in SHAPES:
        x = torch.randn(n, h, w, ci, device="cuda").to(torch.bfloat16)
        dy = torch.randn(n, h, w, co, device="cuda").to(torch.bfloat16)
        dw = torch.empty(co, ci, 3, 3, device="cuda")
        db = torch.empty(co, device="cuda")
        s, mslice, cfg, need = ws.plan(n * h * w, ci, co, 3, False, dil)
        buf = ws.reserve(need)
        wsb = buf.data_ptr() + 4 * s * 9 * ci * co
        fl = 2.0 * n * h * w * ci * co * 9
        res = {m: [] for m in fns}
        for rnd in range(3):
            for m, f in fns.items():
                def call():
                    rc = f(dy.data_ptr(), x.data_ptr(), buf.data_ptr(), wsb, dw.data_ptr(), db.data_ptr(), n, h, w, ci,
                           co, 3, dil, 0, s, mslice, cfg, 0.0, 1.0, None, 0, st, None, 0)
                    assert rc == 0, rc
                for _ in range(3):
                    call()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    call()
                e1.record()
                torch.cuda.synchronize()
                res[m].append(e0.elapsed_time(e1) / 10)
        parts = []
        for m in fns:
            ms = min(res[m])
            parts.append(f"probe{m} {ms:.3f} ms {fl / ms / 1e9:.0f} TF/s")
        print(f"{name} cfg {cfg} S {s}  " + " | ".join(parts), flush=True)


if __name__ == "__main__":
    main()
