"""Training-step engines shared by train.py and bench.py.

Two implementations of ONE training step (zero_grad -> forward -> MSE(sum)
-> backward + gradient all-reduce -> SGD(momentum 0.95)), the reference's
step (utils/train_eval_utils.py:28-52):

* ``TorchStepper`` — the stock PyTorch-ROCm reference stack: nn.Conv2d
  (MIOpen), ATen elementwise, torch DDP (RCCL), torch.optim.SGD.  Used as the
  "reference stack on MI355X" baseline and as the CPU/gloo path.
* ``NativeStepper`` — this framework: the native executor (HIP MFMA kernels,
  NHWC bf16, fused context module), the C++/RCCL bucketed reducer overlapped
  with backward on a side stream, fused multi-tensor SGD over the flat fp32
  master arena that also refreshes the bf16 packed weights, and (optionally)
  the whole step captured once into a hipGraph and replayed.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from ..models.cannet import CANNet


class TorchStepper:
    exec_backend = "torch"

    def __init__(self, device, dtype="fp32", world=1, lr=1e-7, momentum=0.95, channels_last=None, model=None,
                 bucket_mb: float = 25.0):
        self.device = torch.device(device)
        self.model = (model or CANNet(backend=self.exec_backend)).to(self.device)
        self.model.exec_backend = self.exec_backend
        self.dtype = dtype
        self.channels_last = (dtype != "fp32") if channels_last is None else channels_last
        if self.channels_last:
            self.model = self.model.to(memory_format=torch.channels_last)
        self.net = self.model
        if world > 1:
            dev_ids = [self.device.index] if self.device.type == "cuda" else None
            self.net = torch.nn.parallel.DistributedDataParallel(self.model, device_ids=dev_ids,
                                                                 bucket_cap_mb=bucket_mb)
        self.opt = torch.optim.SGD([p for p in self.model.parameters() if p.requires_grad],
                                   lr=lr * world, momentum=momentum, weight_decay=0)
        self.crit = torch.nn.MSELoss(reduction="sum")
        self._loss = None
        self.autocast = {"bf16": torch.bfloat16, "fp16": torch.float16}.get(dtype)
        self.scaler = torch.amp.GradScaler("cuda") if dtype == "fp16" else None

    def step(self, img, gt):
        self.opt.zero_grad(set_to_none=True)
        if self.channels_last:
            img = img.contiguous(memory_format=torch.channels_last)
        if self.autocast is not None:
            with torch.autocast(self.device.type, dtype=self.autocast):
                et = self.net(img)
            loss = self.crit(et.float(), gt)
        else:
            et = self.net(img)
            loss = self.crit(et, gt)
        if self.scaler is not None:
            self.scaler.scale(loss).backward()
            self.scaler.step(self.opt)
            self.scaler.update()
        else:
            loss.backward()
            self.opt.step()
        self._loss = loss.detach()
        return self._loss

    def last_loss(self) -> Optional[float]:
        return None if self._loss is None else float(self._loss)


class Fp32Stepper(TorchStepper):
    """Approximately-fp32 training numerics (the reference trains fp32, train.py:126) on the native kernels: every
    convolution — forward, data and weight gradient — runs as split-bf16 GEMMs on the MFMA conv kernels with fp32
    accumulation (ops/fp32.py: ~2^-16 relative error per product, not bitwise fp32); ReLU / pooling / the context module's elementwise math, the loss, DDP and SGD
    are the fp32 ATen / torch.distributed ones of TorchStepper."""
    exec_backend = "hip_fp32"

    def __init__(self, device, dtype="fp32", **kw):
        if dtype != "fp32":
            raise ValueError("Fp32Stepper is the fp32 step")
        super().__init__(device, dtype="fp32", channels_last=False, **kw)


class ArenaStepper:
    """This framework's data-parallel engine on the plain-ATen CANNet: the CPU / gloo rehearsal of the native step's
    distributed path (engine/native.py), used by ``bench.py --device cpu`` and the multi-process CPU tests.

    Same structure as the native step: fp32 parameters and gradients in one flat arena laid out in gradient-ready
    order (utils/flat.py), the bucketed reducer (parallel/reducer.py) driven by post-accumulate-grad hooks so
    buckets are all-reduced while autograd still runs, the loss and its non-finite flag in one 2-element collective,
    1/world folded into the SGD update (momentum 0.95, train.py:63,126 of the reference), the update skipped on a
    non-finite loss on every rank alike, and the init-time parameter sync as one broadcast of the arena."""
    exec_backend = "torch"

    def __init__(self, device="cpu", world=1, lr=1e-7, momentum=0.95, model=None, bucket_mb: float = 25.0):
        from ..models.cannet import grad_ready_order
        from ..parallel.reducer import BucketedReducer
        from ..utils.flat import FlatArena
        self.device = torch.device(device)
        self.model = (model or CANNet(backend=self.exec_backend)).to(self.device)
        self.model.exec_backend = self.exec_backend
        self.world = world
        self.lr = lr * world                       # train.py:25 linear scaling
        self.momentum = momentum
        self.params = list(self.model.parameters())
        order = grad_ready_order(self.model)
        self.arena = FlatArena(self.params, self.device, order=order)
        self.mom = torch.zeros_like(self.arena.data)
        self.reducer = BucketedReducer(self.arena, order, bucket_mb=bucket_mb, transport="torch")
        self.reducer.attach_hooks()
        self.flags = torch.zeros(2, dtype=torch.float32, device=self.device)
        self.crit = torch.nn.MSELoss(reduction="sum")
        self.comm_timing = False
        self._timings = []
        self._loss = None
        if world > 1:
            self.reducer.broadcast_arena(0)

    def step(self, img, gt):
        red = self.reducer
        red.set_timing(self.comm_timing)
        self.arena.grad.zero_()
        self.arena.attach_grads()                  # autograd accumulates into the arena views in place
        red.begin()
        et = self.model(img.to(self.device))
        loss = self.crit(et, gt.to(self.device))
        loss.backward()
        red.finish()
        if self.comm_timing:
            self._timings.append(red.timings())
        with torch.no_grad():
            self.flags[0] = 0.0 if bool(torch.isfinite(loss)) else 1.0
            self.flags[1] = loss.detach()
            red.allreduce_scalars(self.flags)
            if self.flags[0] == 0:
                # buf = m * buf + g / W ; p -= lr * buf   (torch.optim.SGD semantics, zero-initialised buffer)
                self.mom.mul_(self.momentum).add_(self.arena.grad, alpha=1.0 / self.world)
                self.arena.data.add_(self.mom, alpha=-self.lr)
        self._loss = self.flags[1:2] / self.world
        return self._loss

    def comm_report(self, reset: bool = True) -> Optional[dict]:
        """The last timed step's per-bucket all-reduce report (BucketedReducer.timings)."""
        t = [x for x in self._timings if x is not None]
        if reset:
            self._timings = []
        return t[-1] if t else None

    def last_loss(self) -> Optional[float]:
        return None if self._loss is None else float(self._loss.reshape(-1)[0])


def build_trainer(impl="hip", dtype="bf16", device="cuda", world=1, lr=1e-7, batch=8,
                  height=768, width=1024, graph=True, model=None, bucket_mb: float = 25.0,
                  reducer_transport: Optional[str] = None):
    if impl == "arena":
        return ArenaStepper(device, world=world, lr=lr, model=model, bucket_mb=bucket_mb)
    if impl == "torch":
        return TorchStepper(device, dtype=dtype, world=world, lr=lr, model=model, bucket_mb=bucket_mb)
    if dtype == "fp32":
        return Fp32Stepper(device, world=world, lr=lr, model=model, bucket_mb=bucket_mb)
    from .native import NativeStepper
    return NativeStepper(device, dtype=dtype, world=world, lr=lr, batch=batch, height=height,
                         width=width, graph=graph, model=model, bucket_mb=bucket_mb,
                         reducer_transport=reducer_transport)
