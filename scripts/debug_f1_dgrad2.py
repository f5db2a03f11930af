"""Where does the conv1_1-recompute dgrad (conv_f1, EPI_MASK) differ between runs?  Prints, per differing
element, the stored-path value, each run's value and the stored X2 (mask source)."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from can_distributed_pytorch_amd.ops import conv as C

dtype = torch.float16
n, h, w = 1, 301, 900
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
ref = C.conv_igemm(dy, wd, None, ksize=3, epi=C.EPI_MASK, mask=x2)
nomask = C.conv_igemm(dy, wd, None, ksize=3, epi=C.EPI_NONE)
runs = [C.conv_f1(dy, wd, None, x4, w1p, b1, epi=C.EPI_MASK) for _ in range(8)]
torch.cuda.synchronize()
bad = torch.zeros_like(ref, dtype=torch.bool)
for r in runs:
    bad |= r != ref
idx = torch.nonzero(bad)
print("differing elements", idx.shape[0], "pixels", torch.unique(idx[:, :3], dim=0).tolist()[:40], flush=True)
for e in idx[:12].tolist():
    t = tuple(e)
    print(t, "ref", float(ref[t]), "nomask", float(nomask[t]), "x2", float(x2[t]),
          "runs", [float(r[t]) for r in runs], flush=True)
