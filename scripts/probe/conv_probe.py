"""Time the v2 conv kernel with parts of its mainloop removed (scripts/probe/build_probe.sh builds the
variants).  Output: ms per launch for each probe mode on the F9 / B1 / F6 shapes (batch 8, 768x1024)."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from can_distributed_pytorch_amd.ops import conv as C  # noqa: E402

TILE = int(os.environ.get("PROBE_TILE", "21"))   # 21: conv_glds2 256 x 256 (27: row ring, no probe hooks)
SHAPES = [("F9", 512, 512, 96, 128, 1), ("B1", 1024, 512, 96, 128, 2), ("F6", 256, 256, 192, 256, 1)]


def main():
    libs = {}
    for m in [int(v) for v in os.environ.get("PROBE_MODES", "0,1,2,3").split(",")]:
        lib = ctypes.CDLL(os.path.join(os.environ.get("PROBE_DIR", os.path.join(ROOT, "build", "probe")),
                                       os.environ.get("PROBE_PREFIX", "conv_probe") + f"{m}.so"))
        f = lib.can_conv_igemm
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_int] * 11 + [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                                                    ctypes.c_void_p]
        libs[m] = f
    n = 8
    for name, ci, co, h, w, dil in SHAPES * 3:
        x = torch.randn(n, h, w, ci, device="cuda").to(torch.bfloat16)
        wt = (torch.randn(co, ci, 3, 3, device="cuda") * 0.02)
        wp = C.pack_weight_fwd(wt)
        b = torch.zeros(co, device="cuda")
        y = torch.empty(n, h, w, co, dtype=torch.bfloat16, device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        res = []
        for m, f in libs.items():
            def call():
                rc = f(x.data_ptr(), wp.data_ptr(), b.data_ptr(), 0, y.data_ptr(), n, h, w, ci, co, 3, dil, 0, 0, TILE,
                       0, st, None, 0, None)
                assert rc == 0, rc
            for _ in range(3):
                call()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                call()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 20
            tf = 2.0 * n * h * w * ci * co * 9 / ms / 1e9
            res.append(f"probe{m} {ms:.3f} ms {tf:.0f} TF/s")
        print(name, " | ".join(res), flush=True)


if __name__ == "__main__":
    main()
