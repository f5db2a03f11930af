#!/usr/bin/env python
"""Headline benchmark: CANNet training throughput (imgs/sec, whole node).

Config (BASELINE.json): CANNet, ShanghaiTech-shape synthetic 768x1024 (HxW)
crowd images, per-GPU batch 8 (weak scaling: global batch = 8*N), bf16
compute with fp32 master weights, MSE(sum) loss, SGD momentum 0.95,
lr 1e-7*world (train.py:25,63 of the reference), data-parallel over RCCL.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``.
  * launched by torch.distributed.run (WORLD_SIZE set): one rank per GPU;
    WORLD_SIZE must equal --gpus (else exit 2 — never a silent 1-GPU number);
  * launched bare with --gpus N > 1: this process spawns the N ranks itself
    (``python -m torch.distributed.run --nproc-per-node N``) BEFORE touching
    the GPU and exits with their status; fewer than N visible GPUs -> exit 2.
W untimed steps, then exactly K timed steps bracketed by barrier +
synchronize; the max over ranks is reported; rank 0 prints ONE JSON line.

Every timed step is a full training step: H2D-free synthetic batch already
resident (data="synthetic"), forward, loss, backward, gradient all-reduce,
optimizer step.  After the timed region (not timed): a few steps with
hipEvents around the all-reduce join (``exposed_allreduce_ms``), the
cross-rank replica fingerprint check (``replicas_consistent``) and the peak
HBM of the run.  ``--impl torch`` measures the stock PyTorch-ROCm reference
stack (MIOpen convs + torch DDP) on the same config for comparison.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

BASELINE_IMGS_PER_SEC = 119.692  # stock PyTorch-ROCm bf16 stack on 1x MI355X (reference publishes none)
METRIC = "imgs/sec (whole node) + ShanghaiTech-A MAE, CANNet at 1/2/4/8 MI355X"


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--batch", type=int, default=8, help="per-GPU batch")
    p.add_argument("--height", type=int, default=768)
    p.add_argument("--width", type=int, default=1024)
    p.add_argument("--impl", choices=["hip", "torch"], default=os.environ.get("CANNET_BENCH_IMPL", "hip"))
    p.add_argument("--dtype", choices=["bf16", "fp32", "fp16"], default="bf16")
    p.add_argument("--bucket-mb", type=float, default=25.0, help="gradient all-reduce bucket cap (MiB)")
    p.add_argument("--reducer", choices=["rccl", "torch"], default=os.environ.get("CANNET_REDUCER", "rccl"),
                   help="rccl: own C++ RCCL communicator + bucketed reducer; torch: torch.distributed (NCCL=RCCL)")
    p.add_argument("--graph", type=int, default=0,
                   help="hipGraph-capture the step (hip impl).  Off by default: see profiles/README.md (graph)")
    p.add_argument("--comm-steps", type=int, default=3, help="extra untimed steps with all-reduce timing events")
    p.add_argument("--mode", choices=["train", "infer"], default="train",
                   help="train: the headline training step; infer: forward-only density estimation (serving)")
    return p.parse_args(argv)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(a) -> int:
    """--gpus N without a launcher: spawn N ranks with torch.distributed.run (no GPU call in this process)."""
    import torch
    n_vis = torch.cuda.device_count()          # does not initialise the GPU
    if n_vis < a.gpus:
        print(f"bench.py: --gpus {a.gpus} requested but only {n_vis} GPU(s) visible; refusing to report a "
              f"different node size", file=sys.stderr)
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def infer(a, trainer, pool, sync_all, world, rank, local, dev) -> int:
    """Forward-only throughput (test.py's density estimation): eval mode, no autograd, the same kernels as the
    training forward (native: executor.forward_eval + the 1x1 head)."""
    import torch
    import torch.distributed as dist
    model = trainer.model
    model.eval()
    cast = {"bf16": torch.bfloat16, "fp16": torch.float16}.get(a.dtype) if a.impl == "torch" else None
    imgs = [p[0] for p in pool]

    def fwd(x):
        with torch.no_grad():
            if cast is not None:
                with torch.autocast("cuda", dtype=cast):
                    return model(x.contiguous(memory_format=torch.channels_last))
            return model(x)
    for i in range(a.warmup):
        fwd(imgs[i % len(imgs)])
    sync_all()
    t0 = time.perf_counter()
    for i in range(a.steps):
        et = fwd(imgs[i % len(imgs)])
    sync_all()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    if rank == 0:
        print(json.dumps({
            "metric": "CANNet inference imgs/sec (forward only, density map)", "value": round(a.batch * world * a.steps / dt, 3),
            "unit": "imgs/sec", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(1000.0 * dt / a.steps, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": a.dtype, "data": "synthetic",
            "config": {"model": "CANNet", "global_batch": a.batch * world, "per_gpu_batch": a.batch,
                       "image_hw": [a.height, a.width], "impl": a.impl, "mode": "infer"},
            "count_first_image": float(et[0].sum())}), flush=True)
    if world > 1:
        dist.barrier(device_ids=[local])
        dist.destroy_process_group()
    return 0


def main(argv=None) -> int:
    a = parse(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and a.gpus > 1:
        return launch_ranks(a)
    world = int(env_world or "1")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}: refusing to mislabel the run", file=sys.stderr)
        return 2

    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from can_distributed_pytorch_amd.engine.trainer import build_trainer
    from can_distributed_pytorch_amd.data.synthetic import make_synthetic_batch, expected_flops_per_image

    torch.manual_seed(0)
    transport = None if a.reducer == "rccl" else "torch"
    trainer = build_trainer(impl=a.impl, dtype=a.dtype, device=dev, world=world, lr=1e-7, batch=a.batch,
                            height=a.height, width=a.width, graph=bool(a.graph), bucket_mb=a.bucket_mb,
                            reducer_transport=transport)
    # a small pool of distinct synthetic batches, resident on the GPU
    pool = [make_synthetic_batch(a.batch, a.height, a.width, seed=1000 * rank + i, device=dev) for i in range(2)]

    def sync_all():
        if world > 1:
            dist.barrier(device_ids=[local])
        torch.cuda.synchronize()

    if a.mode == "infer":
        return infer(a, trainer, pool, sync_all, world, rank, local, dev)

    for i in range(a.warmup):
        trainer.step(*pool[i % len(pool)])
    sync_all()
    t0 = time.perf_counter()
    for i in range(a.steps):
        trainer.step(*pool[i % len(pool)])
    sync_all()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    loss = trainer.last_loss()

    # ---- untimed diagnostics
    extra = {}
    red = getattr(trainer, "reducer", None)
    native = a.impl == "hip" and a.dtype != "fp32"       # hip + fp32 = split-bf16 convs under the torch step
    if native:
        extra["reducer"] = None if red is None else red.transport
        extra["rccl_world"] = (red.comm.world if (red is not None and red.comm is not None) else
                               (1 if red is None else None))
        extra["buckets_mib"] = None if red is None else [round(b.numel * 4 / 2 ** 20, 3) for b in red.buckets]
        if a.comm_steps > 0 and not a.graph:
            trainer.comm_timing = True
            for i in range(a.comm_steps):
                trainer.step(*pool[i % len(pool)])
            trainer.comm_timing = False
            ms_comm = trainer.exposed_comm_ms()
            extra["exposed_allreduce_ms"] = None if ms_comm is None else round(ms_comm, 4)
        sync_all()
        from can_distributed_pytorch_amd.parallel.consistency import check_replicas_consistent
        try:
            extra["replicas_consistent"] = bool(check_replicas_consistent(trainer.arena.data))
        except RuntimeError as e:
            extra["replicas_consistent"] = False
            print(f"bench.py: {e}", file=sys.stderr)
    peak = torch.tensor([torch.cuda.max_memory_allocated(dev), torch.cuda.max_memory_reserved(dev)],
                        device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(peak, op=dist.ReduceOp.MAX)
    extra["peak_hbm_gb"] = {"allocated": round(float(peak[0]) / 1e9, 3), "reserved": round(float(peak[1]) / 1e9, 3)}

    ms = 1000.0 * dt / a.steps
    imgs = a.batch * world * a.steps / dt
    tflops = 3.0 * expected_flops_per_image(a.height, a.width) * imgs / 1e12
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(imgs, 3),
            "unit": "imgs/sec",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            # stock stack measured on 1 GPU; for N GPUs it is credited with perfect (N x) scaling
            "vs_baseline": (round(imgs / (BASELINE_IMGS_PER_SEC * world), 4) if BASELINE_IMGS_PER_SEC else None),
            "dtype": a.dtype,
            "data": "synthetic (random-init weights, synthetic 768x1024 crowd images + count-preserving 1/8 density maps)",
            "config": {"model": "CANNet", "global_batch": a.batch * world, "per_gpu_batch": a.batch,
                       "image_hw": [a.height, a.width], "seq_len": None,
                       "parallelism": f"dp{world}", "impl": a.impl,
                       "graph": bool(a.graph) and native, "bucket_mb": a.bucket_mb,
                       "optimizer": "SGD(m=0.95) fp32 master", "loss": "MSE(sum)"},
            "train_tflops_per_s": round(tflops, 2),
            "final_loss": loss,
        }
        out.update(extra)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier(device_ids=[local])
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
