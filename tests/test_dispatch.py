"""Dispatch configuration (ops/dispatch.py, csrc/dispatch.h) and the binary <-> source tie (ops/_ext.py): a stray
environment variable cannot change the default step, a bad override fails loudly, a stale _C is refused."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _py(code, env_extra=None):
    env = {k: v for k, v in os.environ.items() if not k.startswith("CANNET_") or k == "CANNET_ASAN"}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, "-c", f"import sys; sys.path.insert(0, {ROOT!r})\n" + code], env=env,
                          capture_output=True, text=True, timeout=300)


def test_defaults_and_parse():
    from can_distributed_pytorch_amd.ops import dispatch
    d = dispatch.DispatchConfig()
    assert dispatch.parse("") == d
    c = dispatch.parse("rring=0, ws64=0;ctx_tile_f=128")
    assert (c.rring, c.ws64, c.ctx_tile_f) == (0, 0, 128) and c.rring64 == d.rring64
    with pytest.raises(ValueError, match="unknown key"):
        dispatch.parse("rrring=1")
    with pytest.raises(ValueError, match="allowed"):
        dispatch.parse("rring=7")
    with pytest.raises(ValueError, match="key=value"):
        dispatch.parse("rring")


def test_stray_legacy_variables_do_not_change_the_step():
    """The round-3 per-switch variables (CANNET_RRING, CANNET_WS64, ...) are read by nothing any more."""
    stray = {k: "0" for k in ("CANNET_RRING", "CANNET_RRING64", "CANNET_WS64", "CANNET_W1G", "CANNET_CTX_LINEAR",
                              "CANNET_WGRAD_STREAM", "CANNET_BIAS_FUSED", "CANNET_REDUCE_GRIDSTRIDE")}
    code = ("from can_distributed_pytorch_amd.ops import dispatch, _ext\n"
            "assert dispatch.current() == dispatch.DispatchConfig(), dispatch.current()\n"
            "m = _ext.load()\n"
            "if m is not None:\n"
            "    _ext.require()\n"
            "    assert m.get_dispatch() == dispatch.DispatchConfig().native(), m.get_dispatch()\n"
            "print('ok')\n")
    r = _py(code, stray)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr


def test_override_reaches_the_extension_and_restores():
    from can_distributed_pytorch_amd.ops import _ext, dispatch
    m = _ext.load()
    if m is None:
        pytest.skip("native extension not built")
    _ext.require()
    base = m.get_dispatch()
    with dispatch.override(rring=0, reduce_tiled=0) as cfg:
        assert cfg.rring == 0 and m.get_dispatch()["rring"] == 0 and m.get_dispatch()["reduce_tiled"] == 0
        assert dispatch.current().rring == 0
    assert m.get_dispatch() == base and dispatch.current() == dispatch.DispatchConfig()


def test_env_override_is_validated_once():
    r = _py("from can_distributed_pytorch_amd.ops import dispatch\nprint(dispatch.current().rring)",
            {"CANNET_DISPATCH": "rring=1"})
    assert r.returncode == 0 and r.stdout.strip() == "1", r.stderr
    r = _py("from can_distributed_pytorch_amd.ops import dispatch\ndispatch.current()", {"CANNET_DISPATCH": "bogus=1"})
    assert r.returncode != 0 and "unknown key" in r.stderr


def test_no_getenv_on_the_launch_path():
    """No C++ source reads the environment; the Python launch path reads only CANNET_DISPATCH."""
    import glob
    for f in glob.glob(os.path.join(ROOT, "can_distributed_pytorch_amd", "csrc", "*")):
        src = open(f).read()
        assert "getenv(" not in src, f
    for f in ("ops/executor.py", "ops/conv.py", "engine/native.py"):
        src = open(os.path.join(ROOT, "can_distributed_pytorch_amd", f)).read()
        assert "os.environ" not in src, f


def test_binary_tied_to_sources(monkeypatch):
    from can_distributed_pytorch_amd import build_native
    from can_distributed_pytorch_amd.ops import _ext
    m = _ext.load()
    if m is None:
        pytest.skip("native extension not built")
    assert m.src_hash() == build_native.source_hash(), "the in-tree _C is stale: rebuild it"
    monkeypatch.setattr(build_native, "source_hash", lambda files=None: "0" * 64)
    with pytest.raises(RuntimeError, match="stale native extension"):
        _ext.check_source_hash(m)


def test_in_tree_binary_imports():
    """A built _C must import (an undefined symbol only shows up at import time, e.g. on the GPU box)."""
    from can_distributed_pytorch_amd import build_native
    from can_distributed_pytorch_amd.ops import _ext
    if not os.path.exists(build_native.ext_path()):
        pytest.skip("native extension not built")
    assert _ext.load() is not None, f"in-tree _C does not import: {_ext._err}"
