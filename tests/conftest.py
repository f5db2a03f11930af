import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU and the built native extension")
    config.addinivalue_line("markers", "slow: long-running")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture
def dispatch_cfg():
    """Switch kernel-dispatch fields for one test (ops/dispatch.py); the previous config is restored after it.
    ``dispatch_cfg(rring=0)`` — the only way a test selects a non-default variant (no environment variables)."""
    import dataclasses
    from can_distributed_pytorch_amd.ops import dispatch
    prev = dispatch.current()

    def set_(**kw):
        dispatch.apply(dataclasses.replace(dispatch.current(), **kw))
    yield set_
    dispatch.apply(prev)
