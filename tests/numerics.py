"""Tight numerics checkers for the HIP kernels (compared against an fp32 PyTorch reference computed on the SAME
16-bit-rounded operands, so the only legitimate differences are the output rounding and the summation order).

* ``check_out16`` — 16-bit outputs (forward / data-gradient convs): ELEMENTWISE
  |got - ref| <= rtol * |ref| + atol_rms * rms(ref), rtol = 8e-3 (2x the worst-case bf16 rounding, 2^-8) and a
  small absolute floor for outputs that cancel to ~0.  A single dropped or doubled product term perturbs an output
  by ~rms / sqrt(K) (>= 1 % of rms for K <= 9216) and fails it (``test_checker_catches_one_dropped_term``).
* ``check_sum32`` — fp32 long-K reductions (weight gradients over ~10^5-10^6 pixels): elementwise
  |got - ref| <= tol * (max|ref| + |ref|), tol = 1e-3 (fp32 order differences are ~1e-6 of the scale).
"""
import torch

RTOL16 = 8e-3
ATOL16_RMS = 2e-3


def check_out16(got: torch.Tensor, ref: torch.Tensor, rtol: float = RTOL16, atol_rms: float = ATOL16_RMS,
                what: str = ""):
    g, r = got.float(), ref.float()
    assert g.shape == r.shape, (what, g.shape, r.shape)
    rms = r.pow(2).mean().sqrt().item() + 1e-30
    err = (g - r).abs()
    bound = rtol * r.abs() + atol_rms * rms
    bad = err > bound
    if bool(bad.any()):
        i = int(torch.argmax((err - bound).flatten()))
        raise AssertionError(
            f"{what}: {int(bad.sum())} of {bad.numel()} elements outside rtol {rtol} + {atol_rms} rms "
            f"(rms {rms:.4g}); worst at flat {i}: got {g.flatten()[i].item():.6g} ref {r.flatten()[i].item():.6g}")


def check_sum32(got: torch.Tensor, ref: torch.Tensor, tol: float = 1e-3, what: str = ""):
    g, r = got.float(), ref.float()
    assert g.shape == r.shape, (what, g.shape, r.shape)
    scale = r.abs().max().item() + 1e-30
    err = (g - r).abs()
    bound = tol * (scale + r.abs())
    bad = err > bound
    if bool(bad.any()):
        i = int(torch.argmax((err - bound).flatten()))
        raise AssertionError(
            f"{what}: {int(bad.sum())} of {bad.numel()} elements outside {tol} x (max|ref| {scale:.4g} + |ref|); "
            f"worst at flat {i}: got {g.flatten()[i].item():.6g} ref {r.flatten()[i].item():.6g}")


def check(got: torch.Tensor, ref: torch.Tensor, what: str = ""):
    """16-bit result -> check_out16, fp32 result -> check_sum32."""
    if got.dtype in (torch.bfloat16, torch.float16):
        check_out16(got, ref, what=what)
    else:
        check_sum32(got, ref, what=what)
