"""End to end on the GPU: train.py (native step, GPU input pipeline, real-format ShanghaiTech-layout
files) and test.py on the checkpoint it writes."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _make_dataset(root, n_train=4, n_test=2, seed=0):
    from PIL import Image
    from can_distributed_pytorch_amd.data.density import gaussian_filter_density
    rng = np.random.default_rng(seed)
    for part, n in (("train_data", n_train), ("test_data", n_test)):
        os.makedirs(os.path.join(root, part, "images"), exist_ok=True)
        os.makedirs(os.path.join(root, part, "ground_truth"), exist_ok=True)
        for i in range(n):
            h, w = 96 + 8 * (i % 2), 130 + 3 * i          # varied sizes, not multiples of 8
            img = (rng.random((h, w, 3)) * 255).astype(np.uint8)
            Image.fromarray(img).save(os.path.join(root, part, "images", f"IMG_{i}.jpg"))
            pts = np.stack([rng.random(30) * w, rng.random(30) * h], 1)
            np.save(os.path.join(root, part, "ground_truth", f"IMG_{i}.npy"), gaussian_filter_density((h, w), pts))


def test_train_and_test_py_native(tmp_path):
    data = tmp_path / "data"
    _make_dataset(str(data))
    ck = tmp_path / "ck"
    cmd = [sys.executable, os.path.join(ROOT, "train.py"), "--data_root", str(data), "--epochs", "2",
           "--batch-size", "1", "--num-workers", "0", "--wandb", "false", "--show", "true", "--lr", "1e-6",
           "--checkpoint-dir", str(ck), "--log-jsonl", str(ck / "metrics.jsonl")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    recs = [json.loads(x) for x in open(ck / "metrics.jsonl")]
    ep = [x for x in recs if x["kind"] == "epoch"]
    assert len(ep) == 2 and all(np.isfinite(x["loss"]) and np.isfinite(x["mae"]) for x in ep)
    best = sorted(p for p in os.listdir(ck) if p.startswith("epoch_"))
    assert best and os.path.exists(ck / "temp" / "temp_et_0.png")
    r2 = subprocess.run([sys.executable, os.path.join(ROOT, "test.py"), "--data_root", str(data), "--checkpoint",
                         str(ck / best[-1]), "--show", "0"], capture_output=True, text=True, timeout=300,
                        cwd=str(tmp_path))
    assert r2.returncode == 0 and "mae:" in r2.stdout, r2.stderr[-3000:]


def test_train_py_hip_fp32_save_and_resume(tmp_path):
    """--impl hip --dtype fp32 runs the split-bf16 Fp32Stepper (a TorchStepper): the epoch loop, the lr
    schedule, last_state.pth (torch optimizer momentum) and --resume must all take the torch-optimizer branch."""
    data = tmp_path / "data"
    _make_dataset(str(data))
    ck = tmp_path / "ck"
    base = [sys.executable, os.path.join(ROOT, "train.py"), "--data_root", str(data), "--batch-size", "1",
            "--num-workers", "0", "--wandb", "false", "--show", "false", "--lr", "1e-6", "--impl", "hip",
            "--dtype", "fp32", "--lr-schedule", "cosine", "--checkpoint-dir", str(ck),
            "--log-jsonl", str(ck / "metrics.jsonl")]
    r = subprocess.run(base + ["--epochs", "1"], capture_output=True, text=True, timeout=600, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert os.path.exists(ck / "last_state.pth")
    r = subprocess.run(base + ["--epochs", "2", "--resume", str(ck / "last_state.pth")], capture_output=True,
                       text=True, timeout=600, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    ep = [json.loads(x) for x in open(ck / "metrics.jsonl")]
    ep = [x for x in ep if x["kind"] == "epoch"]
    assert [x["epoch"] for x in ep] == [0, 1] and all(np.isfinite(x["loss"]) for x in ep)
