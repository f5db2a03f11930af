"""Epoch loops: training and distributed evaluation.

Parity: utils/train_eval_utils.py of the reference —
  * ``train_one_epoch(model, optimizer, train_loader, device, epoch)`` (:13-58):
    MSELoss(sum), loss reduced (averaged) over ranks, running-mean loss,
    non-finite guard -> exit(1), optimizer.step; returns the mean loss;
  * ``evaluate(model, test_loader, device, epoch, show_images, use_wandb)``
    (:61-138): mae += |sum(et) - sum(gt)| per batch, optional overlay PNGs of
    one random batch, SUM-reduced over ranks; returns the MAE sum.

Native fast path: ``train_one_epoch_native(stepper, ...)`` drives the fused
NativeStepper (HIP executor + RCCL reducer + fused SGD): no host sync per
step — the loss is read back only every ``log_every`` steps and the
non-finite flag (device-side, all-reduced with the loss, and latched by the
SGD kernel so a NaN on a step that is not read is never lost) is checked at
the same cadence and at the end of the epoch.
"""
from __future__ import annotations

import random
import sys
import time
from typing import Optional

import torch

from ..parallel.distributed import is_main_process, reduce_value, get_world_size


def _progress(it, enabled):
    if not enabled:
        return it
    try:
        from tqdm import tqdm
        return tqdm(it, file=sys.stdout)
    except Exception:  # pragma: no cover
        return it


def train_one_epoch(model, optimizer, train_loader, device, epoch, log=None):
    """Generic autograd path (any model/optimizer, DDP or our hook reducer)."""
    model.train()
    criterion = torch.nn.MSELoss(reduction="sum")
    mean_loss = torch.zeros(1, device=device)
    loader = _progress(train_loader, is_main_process())
    for step, (img, gt) in enumerate(loader):
        optimizer.zero_grad()
        img, gt = img.to(device, non_blocking=True), gt.to(device, non_blocking=True)
        et = model(img)
        loss = criterion(et, gt)
        loss.backward()
        loss = reduce_value(loss.detach(), average=True)
        mean_loss = (mean_loss * step + loss) / (step + 1)
        if is_main_process() and hasattr(loader, "desc"):
            loader.desc = f"[epoch {epoch}] mean loss {round(mean_loss.item(), 3)}"
        if not torch.isfinite(loss):
            print("WARNING: non-finite loss, ending training ", loss)
            sys.exit(1)
        optimizer.step()
    if torch.device(device).type == "cuda":
        torch.cuda.synchronize(device)
    return mean_loss.item()


def train_one_epoch_native(stepper, train_loader, device, epoch, log=None, log_every: int = 20, prep=None):
    """Fused native step per batch (see engine/native.py).  ``prep`` maps a raw
    loader batch to (img, gt) on the device (GPU preprocessing)."""
    stepper.model.train()
    stepper.reset_nonfinite()          # the device flag is sticky: any non-finite step of this epoch latches it
    loader = _progress(train_loader, is_main_process())
    total = torch.zeros(1, device=device)
    n = 0
    t0 = time.perf_counter()
    imgs = 0
    pix = 0
    for step, batch in enumerate(loader):
        img, gt = prep(batch) if prep is not None else batch
        loss = stepper.step(img, gt)          # SUM of the per-rank losses (averaged below)
        total += loss.reshape(1) / max(1, get_world_size())
        n += 1
        imgs += img.shape[0] * get_world_size()
        # NHWC4 (GPU-preprocessed) or NCHW input: per-pixel throughput for variable-size images
        hw = img.shape[1] * img.shape[2] if (img.dim() == 4 and img.shape[-1] == 4) else img.shape[-2] * img.shape[-1]
        pix += img.shape[0] * hw * get_world_size()
        if (step + 1) % log_every == 0:
            if stepper.nonfinite():
                print("WARNING: non-finite loss, ending training")
                sys.exit(1)
            if is_main_process():
                ml = (total / n).item()
                if hasattr(loader, "desc"):
                    loader.desc = f"[epoch {epoch}] mean loss {round(ml, 3)}"
                if log is not None:
                    dt = time.perf_counter() - t0
                    log.log(kind="train", epoch=epoch, step=step + 1, mean_loss=ml, imgs_per_s=imgs / max(dt, 1e-9))
    if torch.device(device).type == "cuda":
        torch.cuda.synchronize(device)
    dt = time.perf_counter() - t0
    stepper.last_epoch_stats = {"imgs": imgs, "mpix": pix / 1e6, "seconds": dt,
                                "imgs_per_s": imgs / max(dt, 1e-9), "mpix_per_s": pix / 1e6 / max(dt, 1e-9)}
    if stepper.nonfinite():
        print("WARNING: non-finite loss, ending training")
        sys.exit(1)
    return (total / max(n, 1)).item()


@torch.no_grad()
def evaluate(model, test_loader, device, epoch, show_images=False, use_wandb=False, out_dir="checkpoints/temp",
             prep=None):
    model.eval()
    mae = torch.zeros(1, device=device)
    loader = _progress(test_loader, is_main_process())
    index = random.randint(0, max(0, len(test_loader) - 1))
    for step, batch in enumerate(loader):
        img, gt = prep(batch) if prep is not None else batch
        img, gt = img.to(device, non_blocking=True), gt.to(device, non_blocking=True)
        et = model(img)
        mae += torch.abs(et.sum() - gt.sum())
        if is_main_process():
            if hasattr(loader, "desc"):
                loader.desc = f"[epoch {epoch}]"
            if show_images and step == index:
                from ..utils.vis import save_overlays
                im0 = img[0]
                if im0.dim() == 3 and im0.shape[-1] == 4:          # NHWC4 bf16 -> CHW float
                    im0 = im0[..., :3].float().permute(2, 0, 1)
                paths = save_overlays(im0, gt[0], et[0], epoch, out_dir)
                if use_wandb:
                    from ..utils.metrics import wandb_log_images
                    wandb_log_images(paths, epoch)
    if torch.device(device).type == "cuda":
        torch.cuda.synchronize(device)
    mae_sum = reduce_value(mae, average=False)
    return mae_sum.item()


@torch.no_grad()
def evaluate_per_image(model, loader, device):
    """Single-process per-image MAE / RMSE (test.py:cal_mae semantics)."""
    model.eval()
    ae, se, n = 0.0, 0.0, 0
    for img, gt in loader:
        img, gt = img.to(device), gt.to(device)
        et = model(img)
        d = (et.flatten(1).sum(1) - gt.flatten(1).sum(1)).double()
        ae += d.abs().sum().item()
        se += (d * d).sum().item()
        n += img.shape[0]
    return ae / max(n, 1), (se / max(n, 1)) ** 0.5
