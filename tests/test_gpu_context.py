"""The native context module (model/CANNet.py:42-87) in isolation: forward (fv -> cat(fv, fi)) and backward
(dcat -> d(F10 pre-activation), conv{S}_1 / conv{S}_2 weight gradients) of the executor against the fp32 autograd
reference of the same math, for the linearised one-GEMM form (conv_igemm.hip EPI_CTXF / EPI_CTXB, default when
the map is >= 64 columns wide) and the direct per-scale form (dispatch ctx_linear = 0)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

SCALES = (1, 2, 3, 6)


def _rel(a, b):
    return ((a.double() - b.double()).norm() / (b.double().norm() + 1e-30)).item()


def _ref_context(model, fv):
    """fv [N,C,h,w] fp32 -> cat [N,2C,h,w] (reference math, fp32 autograd)."""
    h, w = fv.shape[2:]
    num = den = None
    for s in SCALES:
        c1, c2 = getattr(model, f"conv{s}_1"), getattr(model, f"conv{s}_2")
        ave = c1(F.adaptive_avg_pool2d(fv, (s, s)))
        up = F.interpolate(ave, size=(h, w), mode="bilinear", align_corners=True)
        wgt = torch.sigmoid(c2(up - fv))
        num = wgt * up if num is None else num + wgt * up
        den = wgt if den is None else den + wgt
    return torch.cat((fv, num / (den + 1e-12)), 1)


def _run(dispatch_cfg, linear, n, h, w, seed, dtype=torch.bfloat16, beta=0.0, dscale=None):
    """beta: accumulate into pre-filled gradient buffers; dscale: the fp16 step's 1 / loss scale (dcat carries the
    scale 1 / dscale, the weight gradients must come out unscaled, d(fv) keeps the scale)."""
    from can_distributed_pytorch_amd.models import CANNet
    from can_distributed_pytorch_amd.ops.executor import CANNetExecutor
    from can_distributed_pytorch_amd.ops import conv as C
    dispatch_cfg(ctx_linear=1 if linear else 0)
    torch.manual_seed(seed)
    model = CANNet(backend="hip").cuda()
    with torch.no_grad():
        for s in SCALES:
            getattr(model, f"conv{s}_1").weight.normal_(0, 0.05)
            getattr(model, f"conv{s}_2").weight.normal_(0, 0.05)
    ex = CANNetExecutor(model, dtype=dtype)
    ex.refresh_packs(force=True)
    c = 512
    fv = (torch.randn(n, h, w, c, device="cuda") + 0.3).to(dtype)
    if linear:
        assert C.ctx_linear_ok(fv)
    cat, saved = ex._context_fwd(fv, save=True)
    assert bool(saved.get("linear", False)) == linear
    # reference on the same 16-bit fv
    fr = fv.float().permute(0, 3, 1, 2).contiguous().requires_grad_(True)
    cr = _ref_context(model, fr)
    e_fwd = _rel(cat.float().permute(0, 3, 1, 2), cr)
    # backward from a random dcat (16-bit, as the B1 data gradient delivers it)
    dcat = torch.randn(n, h, w, 2 * c, device="cuda").to(dtype)
    params = list(model.parameters())
    grads0 = [torch.randn_like(p) if beta else torch.zeros_like(p) for p in params]
    grads = [g.clone() for g in grads0]
    ws = C.WgradWorkspace(fv.device)
    lscale = 1.0
    dsc = None
    if dscale is not None:
        lscale = 1.0 / dscale
        dsc = torch.tensor([dscale], dtype=torch.float32, device="cuda")
    dcat_in = (dcat.float() * lscale).to(dtype)              # exact: a power-of-two scale
    dpre = ex._context_bwd(saved, fv, dcat_in, grads, ws, beta, 1.0, lambda idx: None, dsc)
    torch.cuda.synchronize()
    dpre = dpre.float() / lscale
    refs = torch.autograd.grad(cr, [fr] + [getattr(model, f"conv{s}_{k}").weight for s in SCALES for k in (1, 2)],
                               dcat.float().permute(0, 3, 1, 2))
    dfv_ref = refs[0] * (fr > 0)
    e_dfv = _rel(dpre.float().permute(0, 3, 1, 2), dfv_ref)
    e_w = {}
    i = 1
    for s in SCALES:
        for k in (1, 2):
            p = getattr(model, f"conv{s}_{k}").weight
            idx = next(j for j, q in enumerate(params) if q is p)
            e_w[f"conv{s}_{k}"] = _rel(grads[idx] - beta * grads0[idx], refs[i])
            i += 1
    return e_fwd, e_dfv, e_w


@pytest.mark.parametrize("tile", ["256", "128"])
@pytest.mark.parametrize("n,h,w", [(2, 17, 65), (1, 12, 128), (2, 9, 96)])
def test_context_linear_vs_fp32(dispatch_cfg, n, h, w, tile):
    dispatch_cfg(ctx_tile_f=int(tile), ctx_tile_b=int(tile))
    e_fwd, e_dfv, e_w = _run(dispatch_cfg, True, n, h, w, seed=n * 100 + h)
    assert e_fwd < 5e-3, e_fwd
    assert e_dfv < 2e-2, e_dfv
    assert all(v < 2e-2 for v in e_w.values()), e_w


@pytest.mark.parametrize("dtype,beta,dscale", [(torch.bfloat16, 1.0, None), (torch.float16, 0.0, 0.25),
                                               (torch.float16, 1.0, 0.5)])
def test_context_linear_accumulate_and_loss_scale(dispatch_cfg, dtype, beta, dscale):
    """The linearised backward's beta != 0 path (ctx_w2_scatter + ctx_gemm mode 2 accumulating into pre-filled
    gradients), the fp16 loss-scale path (dscale folded into every context weight gradient) and fp16 dG storage."""
    e_fwd, e_dfv, e_w = _run(dispatch_cfg, True, 2, 12, 96, seed=41, dtype=dtype, beta=beta, dscale=dscale)
    assert e_fwd < 5e-3, e_fwd
    assert e_dfv < 2e-2, e_dfv
    assert all(v < 2e-2 for v in e_w.values()), e_w


@pytest.mark.parametrize("n,h,w", [(2, 9, 12), (1, 12, 128)])
def test_context_direct_vs_fp32(dispatch_cfg, n, h, w):
    e_fwd, e_dfv, e_w = _run(dispatch_cfg, False, n, h, w, seed=7)
    assert e_fwd < 5e-3, e_fwd
    assert e_dfv < 2e-2, e_dfv
    assert all(v < 2e-2 for v in e_w.values()), e_w


def test_context_linear_matches_direct(dispatch_cfg):
    """Same inputs through both forms: the two bf16 implementations agree as closely as each agrees with fp32."""
    a = _run(dispatch_cfg, True, 1, 12, 128, seed=3)
    b = _run(dispatch_cfg, False, 1, 12, 128, seed=3)
    assert a[0] < 2 * b[0] + 1e-3 and a[1] < 2 * b[1] + 1e-3, (a, b)
