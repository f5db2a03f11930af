"""Isolated timings of the context module's kernels at the bench shape (fv = 8 x 96 x 128 x 512, i.e. batch 8 at
768 x 1024): the linearised one-GEMM form vs the direct per-scale form, forward and backward, plus the plain
GEMMs of the same shapes as a yardstick.  usage: python scripts/bench_ctx.py [n h w]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timeit(fn, reps=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1000.0     # us


def main():
    from can_distributed_pytorch_amd.models import CANNet
    from can_distributed_pytorch_amd.ops.executor import CANNetExecutor
    from can_distributed_pytorch_amd.ops import conv as C
    from can_distributed_pytorch_amd.ops import dispatch
    n, h, w = (int(v) for v in sys.argv[1:4]) if len(sys.argv) >= 4 else (8, 96, 128)
    c = 512
    torch.manual_seed(0)
    model = CANNet(backend="hip").cuda()
    ex = CANNetExecutor(model)
    ex.refresh_packs(force=True)
    fv = torch.relu(torch.randn(n, h, w, c, device="cuda")).to(torch.bfloat16)
    dcat = torch.randn(n, h, w, 2 * c, device="cuda").to(torch.bfloat16)
    params = list(model.parameters())
    grads = [torch.zeros_like(p) for p in params]
    ws = C.WgradWorkspace(fv.device)
    gf = 2 * n * h * w * c * c * 4 / 1e9
    res = {}
    for lin in (1, 0):
        with dispatch.override(ctx_linear=lin):
            tag = "linear" if lin == 1 else "direct"
            res[f"{tag} fwd"] = timeit(lambda: ex._context_fwd(fv, True))
            cat, sv = ex._context_fwd(fv, True)
            res[f"{tag} bwd (main+side, serial)"] = timeit(
                lambda: ex._context_bwd(sv, fv, dcat, grads, ws, 0.0, 1.0, lambda i: None))
    cat, sv = ex._context_fwd(fv, True)
    t = torch.randn(n, 50, c, device="cuda")
    u = torch.randn(n, 50, c, device="cuda")
    res["CTXF gemm"] = timeit(lambda: C.conv_ctx_fwd(fv, ex.ctx2cat_fwd, t, u))
    with dispatch.override(ctx_tile_f=128):
        res["CTXF gemm 128x128 tiles"] = timeit(lambda: C.conv_ctx_fwd(fv, ex.ctx2cat_fwd, t, u))
    res["plain 1x1 gemm fv x W2cat (EPI_NONE)"] = timeit(lambda: C.conv_igemm(fv, ex.ctx2cat_fwd, None, ksize=1,
                                                                                 epi=C.EPI_NONE))
    dg, rowacc = C.ctx_bwd_lin(dcat, sv["wts"], sv["u"])
    res["ctx_bwd_lin"] = timeit(lambda: C.ctx_bwd_lin(dcat, sv["wts"], sv["u"]))
    res["CTXB gemm"] = timeit(lambda: C.conv_ctx_bwd(dg, ex.ctx2cat_dgr, t, dcat, fv))
    with dispatch.override(ctx_tile_b=128):
        res["CTXB gemm 128x128 tiles"] = timeit(lambda: C.conv_ctx_bwd(dg, ex.ctx2cat_dgr, t, dcat, fv))
    res["plain 1x1 gemm dG x W2cat^T (EPI_NONE)"] = timeit(lambda: C.conv_igemm(dg, ex.ctx2cat_dgr, None, ksize=1,
                                                                                   epi=C.EPI_NONE))
    dw = torch.empty(4 * c, c, 1, 1, device="cuda")
    res["dW2cat wgrad"] = timeit(lambda: C.conv_wgrad(dg, fv, dw, None, ksize=1, ws=ws))
    for k, v in res.items():
        print(f"{k:45s} {v:9.1f} us" + (f"   {gf / v * 1e6 / 1e3:7.1f} TF/s" if "gemm" in k or "wgrad" in k else ""))


if __name__ == "__main__":
    main()
