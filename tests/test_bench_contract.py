"""bench.py launcher contract (CPU): never report a node size other than --gpus; the N-rank chain
(launch_ranks -> torch.distributed.run -> rank main -> max-reduced JSON) runs end to end on gloo."""
import json
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


def _json_line(stdout: str) -> dict:
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


@pytest.mark.timeout(600)
def test_cpu_two_rank_chain_end_to_end():
    """The driver's N-GPU launch path, rehearsed on gloo: bare ``bench.py --gpus 2`` spawns torchrun, each rank runs
    the flat-arena data-parallel step with the bucketed reducer, rank 0 prints ONE max-over-ranks JSON line."""
    r = _run(["--device", "cpu", "--gpus", "2", "--steps", "2", "--warmup", "1", "--comm-steps", "1"],
             {"OMP_NUM_THREADS": "2"})
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    out = _json_line(r.stdout)
    assert out["n_gpus"] == 2 and out["steps"] == 2 and out["warmup"] == 1
    cfg = out["config"]
    assert cfg["global_batch"] == 2 * cfg["per_gpu_batch"] and cfg["parallelism"] == "dp2"
    assert cfg["device"] == "cpu" and cfg["impl"] == "arena"
    assert out["replicas_consistent"] is True
    assert out["value"] > 0 and out["final_loss"] == out["final_loss"]
    tl = out["allreduce_timeline"]
    assert [b["bucket"] for b in tl["buckets"]] == list(range(len(out["buckets_mib"])))
    assert tl["exposed_ms_max_over_ranks"] >= tl["exposed_ms"] >= 0.0
    assert "64x64" in out["data"]


def test_launcher_never_imports_torch():
    """launch_ranks runs before any rank exists: it must not touch HIP (a process that initialised the GPU must
    not start the rank processes).  It does not even import torch: GPUs are counted from the KFD topology."""
    code = (
        "import sys, subprocess\n"
        f"sys.path.insert(0, {ROOT!r})\n"
        "import bench\n"
        "calls = []\n"
        "class R: returncode = 0\n"
        "subprocess.run = lambda cmd, env=None: (calls.append(cmd), R())[1]\n"
        "rc = bench.main(['--device', 'cpu', '--gpus', '3', '--steps', '1'])\n"
        "assert rc == 0 and len(calls) == 1, (rc, calls)\n"
        "cmd = calls[0]\n"
        "assert '--nproc-per-node=3' in cmd and '127.0.0.1' in cmd, cmd\n"
        "rc2 = bench.main(['--gpus', '64', '--steps', '1'])\n"
        "assert rc2 == 2, rc2\n"
        "assert 'torch' not in sys.modules, 'launcher imported torch'\n"
        "print('ok')\n")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "ok" in r.stdout, (r.stdout, r.stderr)


def test_visible_gpu_count_honours_masks(monkeypatch):
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod2", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    n = bench.visible_gpu_count()
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    base = bench.visible_gpu_count()
    assert n <= base
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    assert bench.visible_gpu_count() == 0
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0")
    assert bench.visible_gpu_count() == min(1, base)


@pytest.mark.gpu
def test_visible_gpu_count_matches_hip():
    """On a GPU box the HIP-free count equals HIP's own (computed first, in a fresh process)."""
    code = (f"import sys; sys.path.insert(0, {ROOT!r}); import bench; n = bench.visible_gpu_count(); "
            "import torch; assert not torch.cuda.is_initialized(); print(n, torch.cuda.device_count())")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    ours, hip = map(int, r.stdout.split()[-2:])
    assert ours == hip >= 1
