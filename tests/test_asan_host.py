"""Host AddressSanitizer build of the native runtime (sanitizers on host code).

``build_native.py --asan`` compiles the pybind bindings, the RCCL communicator /
bucketed reducer and the host half of every .hip unit with -fsanitize=address
(device code is not instrumented).  The checks run the instrumented module in
a child python under the ASan runtime (LD_PRELOAD), so any heap/stack error in
host code aborts the child and fails the test.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _asan_child(code: str, timeout: int = 240):
    from can_distributed_pytorch_amd import build_native as B
    if not os.path.exists(B.ext_path(asan=True)):
        B.build(jobs=min(8, os.cpu_count() or 1), asan=True)
    r = subprocess.run([sys.executable, "-c", code], env=B.asan_env(), cwd=ROOT, capture_output=True, text=True,
                       timeout=timeout)
    assert r.returncode == 0, f"rc={r.returncode}\n{r.stdout[-3000:]}\n{r.stderr[-6000:]}"
    assert "AddressSanitizer" not in r.stderr, r.stderr[-6000:]
    return r.stdout


def test_asan_host_planning_and_bindings():
    """Host-only entry points (argument conversion, wgrad planning for every CANNet layer shape) under ASan."""
    out = _asan_child("""
from can_distributed_pytorch_amd.ops import _ext
C = _ext.require()
assert C.__name__.endswith('_C_asan'), C.__name__
shapes = [(3, 64, True), (64, 64, False), (64, 128, False), (128, 128, False), (128, 256, False), (256, 256, False),
          (256, 512, False), (512, 512, False), (1024, 512, False), (512, 256, False), (256, 128, False),
          (128, 64, False)]
for m in (8 * 768 * 1024, 98304, 4096):
    for ci, co, first in shapes:
        s, ms, cfg = C.wgrad_plan(m, ci, co, 3, int(first), 1024)
        assert s >= 1 and cfg >= 0, (ci, co, s, cfg)
    assert C.wgrad_plan(m, 512, 512, 1, 0, 1024)[0] >= 1
print('ok', C.arch())
""")
    assert "ok" in out


@pytest.mark.gpu
def test_asan_host_native_step_with_rccl_reducer():
    """A native training step with the C++ RCCL bucketed reducer (1-rank communicator) under host ASan."""
    out = _asan_child("""
import torch
from can_distributed_pytorch_amd.engine.native import NativeStepper
from can_distributed_pytorch_amd.data.synthetic import make_synthetic_batch
from can_distributed_pytorch_amd.models import CANNet
torch.manual_seed(0)
st = NativeStepper('cuda', lr=1e-7, graph=False, model=CANNet(), reducer_transport='rccl', bucket_mb=2.0)
img, gt = make_synthetic_batch(1, 64, 64, seed=0, device='cuda')
for _ in range(2):
    st.step(img, gt)
torch.cuda.synchronize()
assert not st.nonfinite()
print('ok', st.last_loss())
""", timeout=300)
    assert "ok" in out
