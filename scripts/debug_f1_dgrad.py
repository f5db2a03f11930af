"""Determinism probe: conv1_2 dgrad stored path (conv_igemm EPI_MASK) vs conv1_1-recompute path (conv_f1),
each run 6 times on the same inputs (fp16 / bf16, 301x900 and 2x40x136)."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from can_distributed_pytorch_amd.ops import conv as C

for dtype in (torch.float16, torch.bfloat16) * 3:
    for (n, h, w) in ((1, 301, 900), (2, 40, 136)):
        torch.manual_seed(10)
        img = torch.randn(n, 3, h, w, device="cuda")
        x4 = C.to_nhwc4(img, dtype)
        w1 = (torch.randn(64, 3, 3, 3, device="cuda") * 0.2).to(dtype).float()
        b1 = torch.randn(64, device="cuda") * 0.1
        w2 = (torch.randn(64, 64, 3, 3, device="cuda") * 0.05).to(dtype).float()
        torch.randn(64, device="cuda")
        w1p = C.pack_weight_first(w1, dtype)
        x2 = C.conv_igemm(x4, w1p, b1, ksize=3, first=True)
        dy = torch.randn(n, h, w, 64, device="cuda").to(dtype)
        wd = C.pack_weight_dgrad(w2, dtype)
        refs = [C.conv_igemm(dy, wd, None, ksize=3, epi=C.EPI_MASK, mask=x2) for _ in range(6)]
        f1s = [C.conv_f1(dy, wd, None, x4, w1p, b1, epi=C.EPI_MASK) for _ in range(6)]
        x2s = [C.conv_igemm(x4, w1p, b1, ksize=3, first=True) for _ in range(3)]
        torch.cuda.synchronize()
        same = lambda l: all(torch.equal(l[0], t) for t in l[1:])
        d = (refs[0].float() - f1s[0].float()).abs()
        idx = torch.nonzero(d > 0)
        print(dtype, (n, h, w), "ref deterministic", same(refs), "f1 deterministic", same(f1s),
              "x2 deterministic", same(x2s), "ref==f1", torch.equal(refs[0], f1s[0]),
              "ndiff", int((d > 0).sum()), "max", float(d.max()), "first diffs", idx[:6].tolist(), flush=True)
