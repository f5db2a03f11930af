#!/usr/bin/env python
"""Distributed CANNet training (reference: train.py of zgzhengSEU/CAN-distributed-pytorch).

Launch exactly like the reference (one process per GPU, env rendezvous):
    python -m torch.distributed.run --nproc_per_node=8 --master-addr 127.0.0.1 train.py --data_root data/SHA/
    python train.py --synthetic 768x1024 --epochs 2          # single GPU, synthetic data
All reference flags are accepted with the same names and defaults (train.py:174-197);
booleans parse properly (--wandb false works; reference Q2), --data_root is honoured
(ShanghaiTech layout {train,test}_data/{images,ground_truth}; reference Q3).

Per epoch: train (native fused step: HIP kernels + RCCL bucketed reducer +
fused SGD), distributed MAE evaluation (sum over ranks / padded test-set size,
reference train.py:157), best-MAE checkpoint ``checkpoints/epoch_{e}.pth``
(plain CANNet state_dict, loadable by test.py and by the reference's test.py),
a resumable ``checkpoints/last_state.pth``, JSONL metrics.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from can_distributed_pytorch_amd.models import CANNet  # noqa: E402
from can_distributed_pytorch_amd.parallel.distributed import init_distributed_mode, barrier, cleanup  # noqa: E402
from can_distributed_pytorch_amd.utils.checkpoint import (save_checkpoint, load_checkpoint,  # noqa: E402
                                                          save_train_state, load_train_state)
from can_distributed_pytorch_amd.utils.metrics import JsonlLogger, wandb_init, wandb_log  # noqa: E402


def str2bool(v):
    if isinstance(v, bool):
        return v
    if str(v).lower() in ("1", "true", "yes", "y", "t"):
        return True
    if str(v).lower() in ("0", "false", "no", "n", "f"):
        return False
    raise argparse.ArgumentTypeError(f"boolean expected, got {v!r}")


def build_parser():
    p = argparse.ArgumentParser(description="CANNet training on MI355X")
    # ---- reference flags (same names / defaults)
    p.add_argument("--epochs", type=int, default=500)
    p.add_argument("--batch-size", type=int, default=1)
    p.add_argument("--lr", type=float, default=1e-7)
    p.add_argument("--lrf", type=float, default=0.1, help="final lr factor for --lr-schedule cosine (unused otherwise, as in the reference)")
    p.add_argument("--syncBN", type=str2bool, default=True,
                   help="convert BatchNorm to SyncBatchNorm when world > 1 (the reference model has no BN: a no-op "
                        "unless --batch-norm)")
    p.add_argument("--wandb", type=str2bool, default=True, help="log to wandb if it is installed")
    p.add_argument("--show", type=str2bool, default=True, help="save GT/prediction overlay PNGs each epoch")
    p.add_argument("--data_root", type=str, default="./data/Shanghai_part_A/")
    p.add_argument("--init_checkpoint", type=str, default="./checkpoints/epoch_26.pth")
    p.add_argument("--device", default="cuda")
    p.add_argument("--world-size", default=4, type=int)
    p.add_argument("--dist-url", default="env://")
    # ---- new flags
    p.add_argument("--impl", choices=["hip", "torch"], default="hip", help="hip: native kernels; torch: stock PyTorch (reference stack)")
    p.add_argument("--dtype", choices=["bf16", "fp32", "fp16"], default="bf16")
    p.add_argument("--synthetic", type=str, default="", help="HxW: train/eval on synthetic crowds of this size")
    p.add_argument("--synthetic-n", type=int, default=64, help="synthetic train-set size (test set = n/4)")
    p.add_argument("--graph", type=str2bool, default=False,
                   help="hipGraph-capture the step (fixed-size inputs only; off by default: the eager step overlaps "
                        "weight gradients on a side stream, which the ROCm graph serialises)")
    p.add_argument("--bucket-mb", type=float, default=25.0)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--num-workers", type=int, default=8, help="JPEG-decoding DataLoader workers per rank")
    p.add_argument("--lr-schedule", choices=["none", "cosine"], default="none")
    p.add_argument("--checkpoint-dir", default="checkpoints")
    p.add_argument("--resume", type=str, default="", help="resume from a last_state.pth written by this script")
    p.add_argument("--log-jsonl", type=str, default="checkpoints/metrics.jsonl")
    p.add_argument("--vgg16", type=str, default="", help="local torchvision VGG-16 state_dict for the frontend (reference downloads it)")
    p.add_argument("--eval-every", type=int, default=1)
    p.add_argument("--check-sync-every", type=int, default=1, help="epochs between cross-rank weight fingerprint checks (0: off)")
    p.add_argument("--batch-norm", type=str2bool, default=False,
                   help="make_layers(batch_norm=True) variant (reference C04 branch; stock autograd path only)")
    p.add_argument("--gpu-preprocess", type=str2bool, default=True,
                   help="decode on CPU workers, resize/flip/normalise on the GPU (hip impl, real data)")
    return p


def make_loaders(args, world, rank, raw=False, device=None, dtype=None):
    """Train / test loaders.  raw=True: decoded uint8 samples packed per batch in the workers (PackedCollate),
    one H2D copy + one preprocessing launch per batch on the GPU.  Synthetic data on a GPU run is rendered on
    the GPU (SyntheticGPULoader), sharded by the same DistributedSampler."""
    from torch.utils.data import DataLoader, DistributedSampler, BatchSampler
    from can_distributed_pytorch_amd.data import CrowdDataset, SyntheticCrowdDataset
    from can_distributed_pytorch_amd.data.dataset import EpochTaggedSampler
    from can_distributed_pytorch_amd.ops.preprocess import PackedCollate
    collate = PackedCollate() if raw else None
    if args.synthetic:
        h, w = (int(v) for v in args.synthetic.lower().split("x"))
        train_ds = SyntheticCrowdDataset(args.synthetic_n, h, w, seed=args.seed)
        test_ds = SyntheticCrowdDataset(max(1, args.synthetic_n // 4), h, w, seed=args.seed + 1)
    else:
        r = args.data_root
        train_ds = CrowdDataset(os.path.join(r, "train_data", "images"), os.path.join(r, "train_data", "ground_truth"),
                                gt_downsample=8, phase="train", seed=args.seed, raw=raw)
        test_ds = CrowdDataset(os.path.join(r, "test_data", "images"), os.path.join(r, "test_data", "ground_truth"),
                               gt_downsample=8, phase="test", raw=raw)
    train_sampler = DistributedSampler(train_ds, num_replicas=world, rank=rank, shuffle=True, seed=args.seed)
    test_sampler = DistributedSampler(test_ds, num_replicas=world, rank=rank, shuffle=True, seed=args.seed)
    # indices carry the epoch into (persistent) workers: the flip is a function of (seed, epoch, index)
    bs = BatchSampler(EpochTaggedSampler(train_sampler), args.batch_size, drop_last=False)
    if args.synthetic and device is not None and device.type == "cuda" and args.impl == "hip" and \
            args.dtype != "fp32" and h % 16 == 0 and w % 16 == 0:
        from can_distributed_pytorch_amd.data.synthetic import SyntheticGPULoader
        train_loader = SyntheticGPULoader(bs, h, w, args.seed, device, dtype=dtype)
        test_loader = SyntheticGPULoader(BatchSampler(test_sampler, args.batch_size, drop_last=False), h, w,
                                         args.seed + 1, device, dtype=dtype)
        return train_loader, test_loader, train_sampler, test_sampler
    pin = torch.cuda.is_available()
    train_loader = DataLoader(train_ds, batch_sampler=bs, num_workers=args.num_workers, pin_memory=pin,
                              persistent_workers=args.num_workers > 0, collate_fn=collate,
                              prefetch_factor=4 if args.num_workers > 0 else None)
    test_loader = DataLoader(test_ds, sampler=test_sampler, batch_size=args.batch_size, num_workers=args.num_workers,
                             pin_memory=pin, shuffle=False, collate_fn=collate)
    return train_loader, test_loader, train_sampler, test_sampler


def main(args):
    if args.graph:
        # one hipGraph queue for the replayed step (bench.py, profiles/r4/graph_queues.txt); read at HIP init
        os.environ.setdefault("DEBUG_HIP_FORCE_GRAPH_QUEUES", "1")
    init_distributed_mode(args)
    rank, world = args.rank, args.world_size
    use_gpu = str(args.device).startswith("cuda") and torch.cuda.is_available()
    device = torch.device("cuda", args.gpu) if use_gpu else torch.device("cpu")
    if args.impl == "hip" and not use_gpu:
        print("[no GPU: falling back to --impl torch on CPU]")
        args.impl = "torch"
    if args.batch_norm and args.impl == "hip":
        print("[--batch-norm: the fused native step has no BN layers; using --impl torch]")
        args.impl = "torch"
    base_lr = args.lr
    torch.manual_seed(args.seed)
    os.makedirs(args.checkpoint_dir, exist_ok=True)
    log = JsonlLogger(args.log_jsonl, enabled=(rank == 0))
    use_wandb = rank == 0 and wandb_init(args.wandb, project="CANNet-MI355X", name="CANNet", config=vars(args))
    if rank == 0:
        print(f"[train start {time.strftime('%Y.%m.%d %H:%M:%S')}] world {world} impl {args.impl} {args}")

    # the NHWC4 16-bit input layout the GPU preprocessing writes is the native bf16/fp16 step's
    raw = bool(args.gpu_preprocess and args.impl == "hip" and args.dtype != "fp32" and not args.synthetic)
    act = torch.float16 if args.dtype == "fp16" else torch.bfloat16
    train_loader, test_loader, train_sampler, test_sampler = make_loaders(args, world, rank, raw=raw, device=device,
                                                                          dtype=act)
    prep = None
    if raw:
        from can_distributed_pytorch_amd.ops.preprocess import preprocess_packed
        prep = lambda b: preprocess_packed(b, device, dtype=act)  # noqa: E731

    model = CANNet(vgg16_path=args.vgg16 or None, backend="hip" if args.impl == "hip" else "torch",
                   batch_norm=args.batch_norm)
    if args.syncBN and world > 1 and args.batch_norm:
        model = torch.nn.SyncBatchNorm.convert_sync_batchnorm(model)      # train.py:116-118
    if os.path.exists(args.init_checkpoint):
        res = load_checkpoint(model, args.init_checkpoint, strict=False)
        if rank == 0:
            print(f"[load {args.init_checkpoint}: missing {len(res.missing_keys)} unexpected {len(res.unexpected_keys)}]")
    # init-weight consistency (train.py:98-114 + DDP broadcast): one collective in the stepper
    from can_distributed_pytorch_amd.engine.trainer import build_trainer
    fixed = bool(args.synthetic)
    graph = bool(args.graph) and fixed
    # the fused native stepper (flat arena, RCCL reducer, device lr) runs --impl hip in bf16 / fp16; every other
    # combination (--impl torch, and --impl hip --dtype fp32 = Fp32Stepper) is a TorchStepper with a torch optimizer
    native = args.impl == "hip" and args.dtype != "fp32"
    if native:
        stepper = build_trainer(impl="hip", dtype=args.dtype, device=device, world=world, lr=base_lr, graph=graph,
                                model=model, bucket_mb=args.bucket_mb)
        net = stepper.model
        momentum = stepper.mom
    else:
        # --impl torch: stock ATen / MIOpen; --impl hip --dtype fp32: split-bf16 convolutions on the native
        # MFMA kernels (engine/trainer.Fp32Stepper), the rest of the step as the torch one
        stepper = build_trainer(impl=args.impl, dtype=args.dtype if use_gpu else "fp32", device=device, world=world,
                                lr=base_lr, model=model, bucket_mb=args.bucket_mb)
        if world > 1:
            for p in stepper.model.parameters():
                dist.broadcast(p.data, src=0)
        net = stepper.net
        momentum = None

    start_epoch, min_mae, min_epoch = 0, float("inf"), 0
    if args.resume and os.path.exists(args.resume):
        rs = load_train_state(args.resume, stepper.model, momentum,
                              optimizer=None if native else stepper.opt)
        start_epoch, min_mae, min_epoch = rs["epoch"] + 1, rs["min_mae"], rs["min_epoch"]
        if native:
            stepper.load_resume_state(rs["stepper"])

    from can_distributed_pytorch_amd.engine.train_eval import train_one_epoch_native, evaluate, train_one_epoch
    import math
    for epoch in range(start_epoch, args.epochs):
        train_sampler.set_epoch(epoch)
        if args.lr_schedule == "cosine":
            f = ((1 + math.cos(epoch * math.pi / args.epochs)) / 2) * (1 - args.lrf) + args.lrf
            if native:
                stepper.lr = base_lr * world * f
            else:
                for g in stepper.opt.param_groups:
                    g["lr"] = base_lr * world * f
        t0 = time.perf_counter()
        if native:
            mean_loss = train_one_epoch_native(stepper, train_loader, device, epoch, log=log, prep=prep)
        else:
            mean_loss = train_one_epoch(net, stepper.opt, train_loader, device, epoch)
        t_train = time.perf_counter() - t0
        if (epoch + 1) % args.eval_every == 0 or epoch == args.epochs - 1:
            mae_sum = evaluate(net, test_loader, device, epoch, show_images=args.show and rank == 0,
                               use_wandb=use_wandb, out_dir=os.path.join(args.checkpoint_dir, "temp"), prep=prep)
        else:
            mae_sum = float("nan")
        if args.check_sync_every and (epoch + 1) % args.check_sync_every == 0 and world > 1:
            from can_distributed_pytorch_amd.parallel.consistency import check_replicas_consistent, check_comm_health
            if native:
                check_comm_health(stepper.reducer)
                check_replicas_consistent(stepper.arena.data)
            else:
                check_replicas_consistent(torch.cat([p.detach().reshape(-1) for p in stepper.model.parameters()]))
        if rank == 0:
            mean_mae = mae_sum / test_sampler.total_size      # padded size, reference parity (Q6)
            if mean_mae < min_mae:
                min_mae, min_epoch = mean_mae, epoch
                save_checkpoint(stepper.model, os.path.join(args.checkpoint_dir, f"epoch_{epoch}.pth"))
            save_train_state(os.path.join(args.checkpoint_dir, "last_state.pth"), stepper.model, momentum, epoch,
                             min_mae, optimizer=None if native else stepper.opt, min_epoch=min_epoch,
                             stepper_state=stepper.resume_state() if native else None)
            lr_now = stepper.lr if native else stepper.opt.param_groups[0]["lr"]
            ips = len(train_loader) * args.batch_size * world / max(t_train, 1e-9)
            print(f"[epoch {epoch}] loss: {mean_loss:.4f} mae: {mean_mae:.3f}, min_mae: {min_mae:.3f}, "
                  f"min_epoch: {min_epoch}, train img/s {ips:.1f}")
            st = getattr(stepper, "last_epoch_stats", None) or {}
            log.log(kind="epoch", epoch=epoch, loss=mean_loss, mae=mean_mae, min_mae=min_mae, lr=lr_now,
                    train_imgs_per_s=ips, train_s=t_train, train_mpix_per_s=st.get("mpix_per_s"),
                    train_loop_imgs_per_s=st.get("imgs_per_s"), batch_size=args.batch_size, world=world)
            if use_wandb:
                wandb_log(loss=mean_loss, mae=mean_mae, lr=lr_now)
        barrier()
    cleanup()


if __name__ == "__main__":
    main(build_parser().parse_args())
