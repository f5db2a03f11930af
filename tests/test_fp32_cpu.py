"""CPU parts of the fp32 (split-bf16) path: the context module's adaptive pooling and bilinear upsampling as
GEMMs with pool / interpolation matrices == ATen (forward and gradients), incl. sizes S does not divide."""
import pytest
import torch
import torch.nn.functional as F

from can_distributed_pytorch_amd.ops.fp32 import _adaptive_pool_nhwc, _upsample_nhwc, split_weight


@pytest.mark.parametrize("h,w", [(12, 16), (13, 22), (96, 128), (7, 5)])
@pytest.mark.parametrize("S", [1, 2, 3, 6])
def test_pool_and_upsample_matrices_match_aten(h, w, S):
    torch.manual_seed(0)
    x = torch.randn(2, h, w, 8, dtype=torch.float64, requires_grad=True)
    a = _adaptive_pool_nhwc(x.float(), S).double()
    r = F.adaptive_avg_pool2d(x.permute(0, 3, 1, 2), (S, S)).permute(0, 2, 3, 1)
    assert torch.allclose(a, r, atol=1e-6)
    u = _upsample_nhwc(r.float(), h, w).double()
    ru = F.interpolate(r.permute(0, 3, 1, 2), size=(h, w), mode="bilinear", align_corners=True).permute(0, 2, 3, 1)
    assert torch.allclose(u, ru, atol=1e-6)
    # gradients through both (the fp32 step's backward of the context module)
    g = torch.randn(2, h, w, 8, dtype=torch.float64)
    xf = x.detach().float().requires_grad_()
    (gx,) = torch.autograd.grad(_upsample_nhwc(_adaptive_pool_nhwc(xf, S), h, w), xf, g.float())
    (rx,) = torch.autograd.grad(ru, x, g)
    assert torch.allclose(gx.double(), rx, atol=1e-5)


def test_split_weight_hi_lo():
    """hi = bf16(w), lo = bf16(w - hi): hi + lo carries ~16 significant bits of w."""
    torch.manual_seed(1)
    w = torch.randn(64, 64, 3, 3)
    hi, lo = split_weight(w)
    assert torch.equal(hi, hi.to(torch.bfloat16).float()) and torch.equal(lo, lo.to(torch.bfloat16).float())
    rel = ((hi + lo - w).abs() / w.abs().clamp_min(1e-30)).max().item()
    assert rel < 2 ** -15
