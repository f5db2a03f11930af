"""bench.py launcher contract (CPU): never report a node size other than --gpus."""
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=600)


@pytest.mark.skipif(torch.cuda.device_count() >= 2, reason="needs a machine with fewer than 2 GPUs")
def test_gpus_more_than_visible_fails_loudly():
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0"], {})
    assert r.returncode == 2, (r.returncode, r.stdout, r.stderr)
    assert "GPU(s) visible" in r.stderr and r.stdout.strip() == ""


def test_world_size_mismatch_fails_loudly():
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2, (r.returncode, r.stdout, r.stderr)
    assert "WORLD_SIZE=1" in r.stderr and r.stdout.strip() == ""


def test_mode_flag_defaults_to_training():
    """The driver's contract line is the training step; --mode infer is an opt-in serving measurement."""
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(os.path.dirname(__file__), "..", "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    assert bench.parse([]).mode == "train"
    assert bench.parse(["--mode", "infer"]).mode == "infer"
