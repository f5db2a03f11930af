"""The native training step (this framework's hot path).

One step = the reference's step (utils/train_eval_utils.py:28-52):
zero_grad -> forward -> MSE(sum) -> backward (+ DDP all-reduce) -> SGD,
re-designed for MI355X:

* forward/backward: the static executor over gfx950 MFMA kernels
  (ops/executor.py), NHWC bf16 activations, fused head + loss + head-backward;
* gradients are written straight into a flat fp32 arena (utils/flat.py); each
  finished layer is handed to the bucketed reducer (parallel/reducer.py),
  which all-reduces full buckets over RCCL on a side stream while the
  remaining layers of the backward still run;
* loss all-reduce + non-finite flag travel in one 8-byte collective;
  averaging by 1/world is folded into the fused SGD kernel, which also skips
  the update on a non-finite loss (the reference's sys.exit guard,
  utils/train_eval_utils.py:48-50, made device-side and graph-safe);
* the bf16 weight packs are refreshed by pack kernels right after SGD;
* with ``graph=True`` the whole step (for a fixed input shape) is captured
  once into a hipGraph (torch.cuda.CUDAGraph) and replayed: one launch per
  step instead of ~150 kernel launches.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from ..models.cannet import CANNet
from ..ops import _ext
from ..ops.executor import CANNetExecutor
from ..utils.flat import FlatArena


class NativeStepper:
    def __init__(self, device, dtype="bf16", world=1, lr=1e-7, momentum=0.95, batch=8, height=768, width=1024,
                 graph=True, model: Optional[CANNet] = None, reducer=None, bucket_mb: float = 25.0,
                 reducer_transport: Optional[str] = None):
        if dtype != "bf16":
            raise ValueError("the native step computes in bf16 (fp32 master weights); use --impl torch for fp32")
        self.C = _ext.require()
        self.device = torch.device(device)
        self.model = (model or CANNet(backend="hip")).to(self.device)
        self.model.exec_backend = "hip"
        self.world = world
        self.lr = lr * world                       # train.py:25 linear scaling
        self.momentum = momentum
        self.params = list(self.model.parameters())
        self.ex = CANNetExecutor(self.model)
        self.model._executor = self.ex
        # fp32 master/grad arenas laid out in gradient-ready order (contiguous buckets)
        self.arena = FlatArena(self.params, self.device, order=self.ex.grad_ready_order())
        self.mom = torch.zeros_like(self.arena.data)  # momentum buffer (zero init == torch's first-step clone)
        self.grads = self.arena.grad_views()
        self.flags = torch.zeros(4, dtype=torch.float32, device=self.device)   # [nonfinite, loss, ...]
        self.reducer = reducer
        if self.reducer is None and (world > 1 or reducer_transport is not None):
            from ..parallel.reducer import BucketedReducer
            self.reducer = BucketedReducer(self.arena, self.ex.grad_ready_order(), bucket_mb=bucket_mb,
                                           transport=reducer_transport or "auto")
        if world > 1:
            self._broadcast_params()
        self.use_graph = graph
        self.graph = None
        self.static_img = None
        self.static_gt = None
        self._loss = None
        self.steps = 0

    # ------------------------------------------------------------ helpers
    def _broadcast_params(self):
        """Init-time consistency (train.py:98-114 + DDP ctor broadcast) in ONE collective."""
        if self.reducer is not None:
            self.reducer.broadcast_arena(0)
        else:
            dist.broadcast(self.arena.data, src=0)
        self.ex.refresh_packs(force=True)

    def _step_body(self, img, gt, update: bool = True):
        ex = self.ex
        st = _ext.stream_ptr(self.device)
        b6, sv = ex.forward_features(img, save=True)
        ex.workspace(*ex.input_hw(img))
        loss, et, d_b6 = ex.head_train(b6, gt, self.grads)
        red = self.reducer
        if red is not None:
            red.begin()
            red.mark_ready([ex.head_w_index, ex.head_b_index])
        ex.backward_features(sv, d_b6, self.grads, on_grad_ready=(red.mark_ready if red is not None else None))
        del sv
        # scalars: [nonfinite flag, loss]
        self.flags[0:1].copy_((~torch.isfinite(loss)).float())
        self.flags[1:2].copy_(loss)
        if red is not None:
            red.finish()
            red.allreduce_scalars(self.flags[0:2])
        if not update:
            return self.flags[1:2]
        gscale = 1.0 / self.world
        self.C.sgd_momentum(self.arena.data.data_ptr(), self.mom.data_ptr(), self.arena.grad.data_ptr(),
                            self.arena.numel, float(self.lr), float(self.momentum), float(gscale), 0,
                            self.flags.data_ptr(), st)
        ex.refresh_packs(force=True)
        ex.mark_weights_updated()
        return self.flags[1:2]

    # ------------------------------------------------------------ public
    def step(self, img, gt):
        img = img.to(self.device, non_blocking=True)
        gt = gt.to(self.device, non_blocking=True)
        if not self.use_graph:
            out = self._step_body(img, gt)
            self._loss = out
            self.steps += 1
            return out
        if self.graph is None or self.static_img.shape != img.shape or self.static_gt.shape != gt.shape:
            self._capture(img, gt)
        self.static_img.copy_(img, non_blocking=True)
        self.static_gt.copy_(gt, non_blocking=True)
        self.graph.replay()
        self._loss = self._static_loss
        self.steps += 1
        return self._static_loss

    def _capture(self, img, gt):
        self.static_img = img.clone()
        self.static_gt = gt.clone()
        # warm up on a side stream (allocations, workspace sizing, kernel attrs)
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            self._step_body(self.static_img, self.static_gt, update=False)
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self._static_loss = self._step_body(self.static_img, self.static_gt)
        torch.cuda.synchronize(self.device)

    def last_loss(self) -> Optional[float]:
        return None if self._loss is None else float(self._loss.reshape(-1)[0])

    def nonfinite(self) -> bool:
        return bool(self.flags[0].item() != 0)
