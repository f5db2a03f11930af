"""The GPU numerics checker (tests/numerics.py) must catch a kernel that drops ONE product term per output.

Emulated on the CPU: the "kernel output" is the fp32 reference rounded to bf16 (exactly what a correct kernel
returns up to summation order); the same output must FAIL against a reference in which one tap of one input
channel is removed (one of the K terms of every output), at the largest K of the model (the 1024-channel
dilated layer, K = 9216) and at a small one."""
import pytest
import torch
import torch.nn.functional as F

from numerics import check_out16, check_sum32


@pytest.mark.parametrize("ci,co,dil,dtype", [(1024, 64, 2, torch.bfloat16), (64, 64, 1, torch.bfloat16),
                                             (512, 64, 1, torch.float16)])
def test_checker_catches_one_dropped_term(ci, co, dil, dtype):
    torch.manual_seed(0)
    x = torch.randn(1, ci, 12, 16).to(dtype).float()
    w = (torch.randn(co, ci, 3, 3) * 0.05).to(dtype).float()
    ref = F.conv2d(x, w, padding=dil, dilation=dil)
    out = ref.to(dtype)                                      # a correct kernel: rounded output
    check_out16(out, ref)
    w_bad = w.clone()
    w_bad[:, 7, 1, 2] = 0.0                                  # one tap of one channel: one term per output
    bad = F.conv2d(x, w_bad, padding=dil, dilation=dil)
    with pytest.raises(AssertionError):
        check_out16(out, bad)
    w_dbl = w.clone()
    w_dbl[:, ci - 1, 0, 0] *= 2.0                            # one term doubled
    with pytest.raises(AssertionError):
        check_out16(out, F.conv2d(x, w_dbl, padding=dil, dilation=dil))


def test_sum32_catches_one_dropped_pixel_row():
    """Weight gradients: dropping one pixel's contribution out of 2048 fails the fp32 reduction check."""
    torch.manual_seed(1)
    dy = torch.randn(2048, 64)
    xx = torch.randn(2048, 64)
    ref = dy.t() @ xx
    check_sum32(ref.clone(), ref)
    bad = dy[1:].t() @ xx[1:]
    with pytest.raises(AssertionError):
        check_sum32(bad, ref)
