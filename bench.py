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

``--device cpu`` rehearses the same chain without a GPU (gloo, this framework's
flat-arena data-parallel engine on the plain-ATen model, tiny default shape):
``bench.py --device cpu --gpus 2`` goes launch_ranks -> torchrun -> rank main
-> max-reduced JSON exactly as the driver's N-GPU run does (tests/test_bench_contract.py).

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
    p.add_argument("--batch", type=int, default=None, help="per-GPU batch (default 8; cpu: 2)")
    p.add_argument("--height", type=int, default=None, help="default 768 (cpu: 64)")
    p.add_argument("--width", type=int, default=None, help="default 1024 (cpu: 64)")
    p.add_argument("--device", choices=["cuda", "cpu"], default="cuda",
                   help="cpu: gloo rehearsal of the multi-rank chain (--impl arena by default)")
    p.add_argument("--impl", choices=["hip", "torch", "arena"], default=None,
                   help="hip: native kernels + RCCL reducer (cuda default); torch: stock PyTorch + DDP; "
                        "arena: plain-ATen model + this framework's flat-arena bucketed reducer (cpu default)")
    p.add_argument("--dtype", choices=["bf16", "fp32", "fp16"], default="bf16")
    p.add_argument("--bucket-mb", type=float, default=25.0, help="gradient all-reduce bucket cap (MiB)")
    p.add_argument("--reducer", choices=["rccl", "torch"], default=os.environ.get("CANNET_REDUCER", "rccl"),
                   help="rccl: own C++ RCCL communicator + bucketed reducer; torch: torch.distributed (NCCL=RCCL)")
    p.add_argument("--graph", type=int, default=0,
                   help="hipGraph-capture the step (hip impl).  Off by default: see profiles/README.md (graph)")
    p.add_argument("--comm-steps", type=int, default=3, help="extra untimed steps with all-reduce timing events")
    p.add_argument("--mode", choices=["train", "infer"], default="train",
                   help="train: the headline training step; infer: forward-only density estimation (serving)")
    a = p.parse_args(argv)
    cpu = a.device == "cpu"
    if a.impl is None:
        a.impl = "arena" if cpu else os.environ.get("CANNET_BENCH_IMPL", "hip")
    if cpu and a.impl == "hip":
        p.error("--impl hip needs --device cuda")
    if cpu and a.dtype != "fp32":
        a.dtype = "fp32"                       # the CPU rehearsal computes in fp32
    a.batch = a.batch or (2 if cpu else 8)
    a.height = a.height or (64 if cpu else 768)
    a.width = a.width or (64 if cpu else 1024)
    return a


def visible_gpu_count() -> int:
    """GPUs this process may use, counted WITHOUT initialising HIP (torch.cuda.device_count() can fall back to
    hipGetDeviceCount, and a process that has touched the GPU must not start the rank processes).

    KFD topology nodes with SIMDs are the GPUs; one counts only if its render node /dev/dri/renderD<minor> is
    accessible (a container sees only the devices it was given), then ROCR_/HIP_/CUDA_VISIBLE_DEVICES narrow it."""
    base = "/sys/class/kfd/kfd/topology/nodes"
    n = 0
    try:
        nodes = os.listdir(base)
    except OSError:
        nodes = []
    for node in nodes:
        try:
            props = dict(line.split()[:2] for line in open(os.path.join(base, node, "properties")) if line.strip())
        except (OSError, ValueError):
            continue
        if int(props.get("simd_count", "0")) <= 0:
            continue                           # a CPU node
        minor = props.get("drm_render_minor")
        if minor is not None and not os.access(f"/dev/dri/renderD{minor}", os.R_OK | os.W_OK):
            continue
        n += 1
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip()]))
    return n


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(a) -> int:
    """--gpus N without a launcher: spawn N ranks with torch.distributed.run.  Nothing here touches the GPU (no torch
    import even): the GPUs are counted from the KFD topology (visible_gpu_count)."""
    if a.device == "cuda":
        n_vis = visible_gpu_count()
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
        dist.barrier(**({} if cpu else {"device_ids": [local]}))
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

    if a.graph:
        # hipGraph replay with ONE graph queue: the runtime default spreads the captured two-stream step over several
        # queues and resolved fewer concurrent kernels (497.5 vs 513.7 img/s, profiles/r4/graph_queues.txt).  Read
        # by the HIP runtime at its initialisation, so set before the first GPU call.
        os.environ.setdefault("DEBUG_HIP_FORCE_GRAPH_QUEUES", "1")
    import torch
    import torch.distributed as dist
    cpu = a.device == "cpu"
    if cpu:
        dev = torch.device("cpu")
        if world > 1:
            dist.init_process_group("gloo")
    else:
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
            dist.barrier(**({} if cpu else {"device_ids": [local]}))
        if not cpu:
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
    if native or a.impl == "arena":
        extra["reducer"] = None if red is None else red.transport
        if native:
            extra["rccl_world"] = (red.comm.world if (red is not None and red.comm is not None) else
                                   (1 if red is None else None))
        extra["buckets_mib"] = None if red is None else [round(b.numel * 4 / 2 ** 20, 3) for b in red.buckets]
        if a.comm_steps > 0 and not a.graph:
            trainer.comm_timing = True
            for i in range(a.comm_steps):
                trainer.step(*pool[i % len(pool)])
            trainer.comm_timing = False
            if native:
                ms_comm = trainer.exposed_comm_ms()
                extra["exposed_allreduce_ms"] = None if ms_comm is None else round(ms_comm, 4)
            # per-bucket all-reduce timeline of the last diagnostic step (ms after the backward started), max over
            # ranks of the exposed tail: shows whether the all-reduce kernels got CUs while the backward ran
            rep = trainer.comm_report()
            if rep is not None:
                ex_t = torch.tensor([rep["exposed_ms"]], dtype=torch.float64, device=dev)
                if world > 1:
                    dist.all_reduce(ex_t, op=dist.ReduceOp.MAX)
                rep["exposed_ms_max_over_ranks"] = round(float(ex_t), 4)
            extra["allreduce_timeline"] = rep
        sync_all()
        from can_distributed_pytorch_amd.parallel.consistency import check_replicas_consistent
        try:
            extra["replicas_consistent"] = bool(check_replicas_consistent(trainer.arena.data))
        except RuntimeError as e:
            extra["replicas_consistent"] = False
            print(f"bench.py: {e}", file=sys.stderr)
    if not cpu:
        peak = torch.tensor([torch.cuda.max_memory_allocated(dev), torch.cuda.max_memory_reserved(dev)],
                            device=dev, dtype=torch.float64)
        if world > 1:
            dist.all_reduce(peak, op=dist.ReduceOp.MAX)
        extra["peak_hbm_gb"] = {"allocated": round(float(peak[0]) / 1e9, 3),
                                "reserved": round(float(peak[1]) / 1e9, 3)}

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
            "data": f"synthetic (random-init weights, synthetic {a.height}x{a.width} crowd images + "
                    f"count-preserving 1/8 density maps)",
            "config": {"model": "CANNet", "global_batch": a.batch * world, "per_gpu_batch": a.batch,
                       "image_hw": [a.height, a.width], "seq_len": None,
                       "parallelism": f"dp{world}", "impl": a.impl, "device": a.device,
                       "graph": bool(a.graph) and native, "bucket_mb": a.bucket_mb,
                       "optimizer": "SGD(m=0.95) fp32 master", "loss": "MSE(sum)"},
            "train_tflops_per_s": round(tflops, 2),
            "final_loss": loss,
        }
        out.update(extra)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier(**({} if cpu else {"device_ids": [local]}))
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
