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
* the loss and its non-finite flag are written by the fused head's reduction
  kernel straight into a device flag vector, and travel in one 8-byte
  collective; averaging by 1/world is folded into the fused SGD kernel, which
  also skips the update on a non-finite loss and latches a sticky flag the
  host polls at its logging cadence (the reference's sys.exit guard,
  utils/train_eval_utils.py:48-50, made device-side and graph-safe);
* the learning rate lives in a device scalar read by the SGD kernel, so a
  captured step follows an lr schedule;
* roctx ranges (utils/profiling.trace_range, CANNET_ROCTX=1) mark the
  forward / backward / all-reduce / optimizer phases; ``comm_timing`` records
  hipEvents around the post-backward all-reduce join (exposed comm time);
* the bf16 weight packs are refreshed by pack kernels right after SGD;
* with ``graph=True`` the whole step (for a fixed input shape) is captured
  once into a hipGraph (torch.cuda.CUDAGraph) and replayed: one launch per
  step instead of ~150 kernel launches;
* ``dtype="fp16"`` runs the same kernels on fp16 activations / weight packs
  (v_mfma_f32_16x16x32_f16) with dynamic loss scaling kept on the device
  (graph-safe): the scale multiplies d(b6) inside the fused head, 1/scale is
  folded into every weight-gradient reduction, a gradient-overflow check
  after the all-reduce makes the fused SGD skip the step, and a one-thread
  kernel backs the scale off / grows it (GradScaler semantics: x0.5 on
  overflow, x2 after ``scale_interval`` clean steps).
"""
from __future__ import annotations

import contextlib
from typing import Optional

import torch
import torch.distributed as dist

from ..models.cannet import CANNet
from ..ops import _ext
from ..ops.executor import CANNetExecutor
from ..utils.flat import FlatArena
from ..utils.profiling import trace_range

ACT_DTYPES = {"bf16": torch.bfloat16, "fp16": torch.float16}


class NativeStepper:
    def __init__(self, device, dtype="bf16", world=1, lr=1e-7, momentum=0.95, batch=8, height=768, width=1024,
                 graph=True, model: Optional[CANNet] = None, reducer=None, bucket_mb: float = 25.0,
                 reducer_transport: Optional[str] = None, init_scale: float = 65536.0, scale_interval: int = 2000):
        if dtype not in ACT_DTYPES:
            raise ValueError(f"the native step computes in bf16 or fp16 (fp32 master weights), got {dtype!r}; "
                             "use --impl torch for fp32")
        self.C = _ext.require()
        self.dtype = dtype
        self.device = torch.device(device)
        self.model = (model or CANNet(backend="hip")).to(self.device)
        self.model.exec_backend = "hip"
        self.world = world
        self.momentum = momentum
        self.params = list(self.model.parameters())
        self.ex = CANNetExecutor(self.model, dtype=ACT_DTYPES[dtype])
        self.model._executor = self.ex
        # fp32 master/grad arenas laid out in gradient-ready order (contiguous buckets)
        self.arena = FlatArena(self.params, self.device, order=self.ex.grad_ready_order())
        self.mom = torch.zeros_like(self.arena.data)  # momentum buffer (zero init == torch's first-step clone)
        self.grads = self.arena.grad_views()
        # [non-finite loss (any rank after the all-reduce), loss, non-finite gradient (fp16), sticky non-finite]
        self.flags = torch.zeros(4, dtype=torch.float32, device=self.device)
        self._lr_dev = torch.zeros(1, dtype=torch.float32, device=self.device)
        self.lr = lr * world                       # train.py:25 linear scaling
        # fp16: device-side dynamic loss scale {S, 1/S, clean steps, 0}
        self.scaler = None
        self.scale_interval = scale_interval
        if dtype == "fp16":
            self.scaler = torch.tensor([init_scale, 1.0 / init_scale, 0.0, 0.0], dtype=torch.float32,
                                       device=self.device)
        self.bucket_mb = bucket_mb
        self.comm_timing = False
        self._comm_events = []
        self._bucket_reports = []
        self.reducer = reducer
        if self.reducer is None and (world > 1 or reducer_transport is not None):
            from ..parallel.reducer import BucketedReducer
            self.reducer = BucketedReducer(self.arena, self.ex.grad_ready_order(), bucket_mb=bucket_mb,
                                           transport=reducer_transport or "auto")
        self.reducer_transport = None if self.reducer is None else self.reducer.transport
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

    @property
    def lr(self) -> float:
        return self._lr

    @lr.setter
    def lr(self, v: float):
        """Host value + the device scalar the SGD kernel reads (a captured step sees updates)."""
        self._lr = float(v)
        self._lr_dev.fill_(self._lr)

    def _step_body(self, img, gt, update: bool = True):
        ex = self.ex
        st = _ext.stream_ptr(self.device)
        with trace_range("cannet/forward"):
            b6, sv = ex.forward_features(img, save=True)
            ex.workspace(*ex.input_hw(img))
            sc = self.scaler
            # fused head: loss -> flags[1], its non-finite flag -> flags[0] (same kernel, no extra launch)
            loss, et, d_b6 = ex.head_train(b6, gt, self.grads, lscale=sc[0:1] if sc is not None else None,
                                           flags=self.flags)
        red = self.reducer
        timing = self.comm_timing and self.device.type == "cuda"
        if red is not None:
            red.set_timing(timing)
            red.begin()
            red.mark_ready([ex.head_w_index, ex.head_b_index])
        with trace_range("cannet/backward"):
            ex.backward_features(sv, d_b6, self.grads, on_grad_ready=(red.mark_ready if red is not None else None),
                                 dscale=sc[1:2] if sc is not None else None)
        del sv
        if timing:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
        if red is not None:
            with trace_range("cannet/allreduce"):
                red.finish()
                red.allreduce_scalars(self.flags[0:2])
        if timing:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            self._comm_events.append((e0, e1))
            if red is not None:
                self._bucket_reports.append(red.timings())
        if sc is not None:
            # after the all-reduce every rank holds the same gradients -> the same verdict
            self.flags[2:3].zero_()
            self.C.grad_nonfinite(self.arena.grad.data_ptr(), self.arena.numel, self.flags.data_ptr() + 8, st)
        if not update:
            return self.flags[1:2]
        with trace_range("cannet/sgd"):
            gscale = 1.0 / self.world
            self.C.sgd_momentum(self.arena.data.data_ptr(), self.mom.data_ptr(), self.arena.grad.data_ptr(),
                                self.arena.numel, float(self._lr), float(self.momentum), float(gscale), 0,
                                self.flags.data_ptr(), self._lr_dev.data_ptr(), st)
            if sc is not None:
                self.C.scale_update(self.flags.data_ptr() + 8, sc.data_ptr(), int(self.scale_interval), 2.0, 0.5,
                                    float(2 ** 24), st)
            ex.refresh_packs(force=True)
            ex.mark_weights_updated()
        return self.flags[1:2]

    def exposed_comm_ms(self, reset: bool = True) -> Optional[float]:
        """Mean device time between 'every gradient written' and 'all-reduce joined back' over the steps run
        with ``comm_timing`` (the part of the gradient all-reduce NOT hidden behind the backward)."""
        if not self._comm_events:
            return None
        torch.cuda.synchronize(self.device)
        v = sum(a.elapsed_time(b) for a, b in self._comm_events) / len(self._comm_events)
        if reset:
            self._comm_events = []
        return v

    def comm_report(self, reset: bool = True) -> Optional[dict]:
        """Per-bucket all-reduce timing of the last step run with ``comm_timing`` (BucketedReducer.timings: when
        each bucket's gradients were ready, when its all-reduce started / ended, relative to the start of the
        backward, and how long the all-reduce ran past the backward)."""
        t = [x for x in self._bucket_reports if x is not None]
        if reset:
            self._bucket_reports = []
        return t[-1] if t else None

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

    def resume_state(self) -> dict:
        """Device state a resumed run needs besides weights and momentum (checkpoint.save_train_state)."""
        st = {"lr": self._lr, "steps": self.steps}
        if self.scaler is not None:
            st["scaler"] = self.scaler
        return st

    def load_resume_state(self, st: Optional[dict]):
        if not st:
            return
        self.lr = float(st.get("lr", self._lr))
        self.steps = int(st.get("steps", self.steps))
        if self.scaler is not None and st.get("scaler") is not None:
            self.scaler.copy_(st["scaler"].to(self.scaler.device))
        self.ex.refresh_packs(force=True)

    def last_loss(self) -> Optional[float]:
        return None if self._loss is None else float(self._loss.reshape(-1)[0])

    def nonfinite(self) -> bool:
        """A non-finite loss in ANY step since the last ``reset_nonfinite()`` (the reference's exit condition,
        utils/train_eval_utils.py:48-50; sticky on the device, so polling every k steps misses none).  An fp16
        gradient overflow is not one: that step is skipped and the loss scale backed off."""
        return bool(self.flags[3].item() != 0)

    def reset_nonfinite(self):
        self.flags[3:4].zero_()

    def loss_scale(self) -> float:
        return 1.0 if self.scaler is None else float(self.scaler[0].item())

    def skipped_last(self) -> bool:
        """True when the last step's update was skipped (non-finite loss or gradient)."""
        f = self.flags.tolist()
        return f[0] != 0 or f[2] != 0
