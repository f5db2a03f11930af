"""Native CANNet executor: a static, hand-scheduled forward/backward over the
gfx950 kernels (no tracing compiler, no autograd graph of ATen ops).

Reference math: model/CANNet.py:39-91 (forward), the backward is what
autograd derives for it in the reference (SURVEY §2.5 kernel inventory).

Data layout: NHWC 16-bit activations (bf16 by default, fp16 optional: one
element type for every activation / weight pack of the executor), fp32
master weights in the model's own nn.Parameters, 16-bit packed weight copies
(forward + flipped dgrad layouts) refreshed by one pack launch whenever the
fp32 weights change.

Forward (training) saves exactly what the backward needs: every conv input
(NHWC bf16), the max-pool codes of the three pools (4-bit first-max one-hots:
the full-resolution pre-pool activations are never stored), the context
cell tables and the sigmoid maps w_S (linearised context module: c_S is
never formed).
Backward (per layer, reverse order) = weight-gradient (split-pixel MFMA +
deterministic slab reduction) + data-gradient (same MFMA kernel as forward,
flipped weights, ReLU mask / maxpool-backward fused), and after each layer's
gradients are written a ``on_grad_ready(param_indices)`` callback fires so
a bucketed reducer can start all-reducing while the remaining layers run.

Two ways in:
  * ``executor(x)``            — autograd-compatible (CANNet.forward on GPU):
                                 an autograd.Function whose backward returns
                                 ordinary gradients.
  * ``forward_train / backward_from_head`` — used by the native training step
                                 (engine/native.py): gradients go straight into
                                 caller-provided fp32 buffers (the flat gradient
                                 arena), the head/MSE loss is fused.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Sequence

import torch
import torch.nn as nn

from . import _ext
from . import conv as C
from . import dispatch
from ..models.cannet import CONTEXT_SCALES

BF16 = torch.bfloat16
CELL_OFF = {1: 0, 2: 1, 3: 5, 6: 14}


@dataclass
class ConvSpec:
    idx: int                 # position in the executor's conv list
    module: nn.Conv2d
    cin: int
    cout: int
    ksize: int
    dil: int
    first: bool = False
    pool_after: bool = False  # a 2x2 maxpool follows this conv's ReLU
    w_index: int = -1         # index of weight in model.parameters()
    b_index: int = -1


class CANNetExecutor:
    def __init__(self, model: nn.Module, dtype: torch.dtype = BF16):
        self.C = _ext.require()
        self.model = model
        self.act = dtype                   # activation / weight-pack element type
        self.dt = C.dt_code(dtype)
        params = list(model.parameters())
        pid = {id(p): i for i, p in enumerate(params)}
        self.n_params = len(params)
        self.front: List[ConvSpec] = []
        mods = list(model.frontend)
        convs = [m for m in mods if isinstance(m, nn.Conv2d)]
        for j, m in enumerate(convs):
            k = mods.index(m)
            pool_after = any(isinstance(mods[t], nn.MaxPool2d) for t in range(k + 1, min(k + 3, len(mods))))
            self.front.append(ConvSpec(j, m, m.in_channels, m.out_channels, 3, 1, first=(j == 0),
                                       pool_after=pool_after, w_index=pid[id(m.weight)], b_index=pid[id(m.bias)]))
        self.back: List[ConvSpec] = []
        for j, m in enumerate([m for m in model._modules["backend"] if isinstance(m, nn.Conv2d)]):
            self.back.append(ConvSpec(j, m, m.in_channels, m.out_channels, 3, m.dilation[0],
                                      w_index=pid[id(m.weight)], b_index=pid[id(m.bias)]))
        self.head = model.output_layer
        self.head_w_index, self.head_b_index = pid[id(self.head.weight)], pid[id(self.head.bias)]
        self.ctx1 = {s: getattr(model, f"conv{s}_1") for s in CONTEXT_SCALES}
        self.ctx2 = {s: getattr(model, f"conv{s}_2") for s in CONTEXT_SCALES}
        self.ctx1_index = {s: pid[id(self.ctx1[s].weight)] for s in CONTEXT_SCALES}
        self.ctx2_index = {s: pid[id(self.ctx2[s].weight)] for s in CONTEXT_SCALES}
        self.packs: Dict[int, tuple] = {}
        self._pack_version = None
        self._pack_desc = None          # device descriptor rows of the batched pack launch
        self._pack_desc_ptrs = None
        self.ws = None
        self._w1g_buf = None            # conv1_1 weight-gradient slabs of the fused conv1_2 data gradient
        self.stream_override = None
        self._side = None

    def grad_ready_order(self) -> List[int]:
        """Parameter indices in the order backward_features produces them."""
        order = [self.head_w_index, self.head_b_index]
        for s in reversed(self.back):
            order += [s.w_index, s.b_index]
        order += [self.ctx2_index[sc] for sc in CONTEXT_SCALES]
        order += [self.ctx1_index[sc] for sc in CONTEXT_SCALES]
        for s in reversed(self.front):
            order += [s.w_index, s.b_index]
        return order

    # ----------------------------------------------------------- weights
    def _params(self):
        return list(self.model.parameters())

    def _weights_version(self):
        return tuple(p._version for p in self._params())

    def _alloc_packs(self, device):
        for s in self.front + self.back:
            w = s.module.weight
            if s.first:
                # k = tap*4 + c: the pack kernel writes only c < 3, tap < 9 -> pad must be zero
                fwd = torch.zeros(s.cout, 64, dtype=self.act, device=device)
                dgr = None
            else:
                fwd = torch.empty(s.cout, s.ksize * s.ksize * s.cin, dtype=self.act, device=device)
                dgr = torch.empty(s.cin, s.ksize * s.ksize * s.cout, dtype=self.act, device=device)
            self.packs[id(w)] = (fwd, dgr)
        # the four conv{S}_2 packs are items of one [4, 512, 512] buffer each (one batched launch per pass)
        self.ctx2_fwd = torch.empty(len(CONTEXT_SCALES), 512, 512, dtype=self.act, device=device)
        self.ctx2_dgr = torch.empty_like(self.ctx2_fwd)
        for i, sc in enumerate(CONTEXT_SCALES):
            self.packs[id(self.ctx2[sc].weight)] = (self.ctx2_fwd[i], self.ctx2_dgr[i])
        # the linearised context module's interleaved packs: W2cat[4c + si] = W2_S[c] and its transpose
        nsc = len(CONTEXT_SCALES)
        self.ctx2cat_fwd = torch.empty(nsc * 512, 512, dtype=self.act, device=device)
        self.ctx2cat_dgr = torch.empty(512, nsc * 512, dtype=self.act, device=device)

    def refresh_packs(self, force: bool = False):
        """Re-pack the 16-bit weight copies from the fp32 masters (one launch for all layers)."""
        ver = self._weights_version()
        if not force and ver == self._pack_version and self.packs:
            return
        dev = self.head.weight.device
        if not self.packs:
            self._alloc_packs(dev)
        st = self._stream()
        if self._pack_desc is None:
            rows = []
            for s in self.front + self.back:
                fwd, dgr = self.packs[id(s.module.weight)]
                rows.append([s.module.weight.data_ptr(), fwd.data_ptr(), dgr.data_ptr() if dgr is not None else 0,
                             s.cout, s.cin, s.ksize * s.ksize, int(s.first), 0])
            for sc in CONTEXT_SCALES:
                fwd, dgr = self.packs[id(self.ctx2[sc].weight)]
                rows.append([self.ctx2[sc].weight.data_ptr(), fwd.data_ptr(), dgr.data_ptr(), 512, 512, 1, 0, 0])
            for si, sc in enumerate(CONTEXT_SCALES):
                rows.append([self.ctx2[sc].weight.data_ptr(), self.ctx2cat_fwd.data_ptr(),
                             self.ctx2cat_dgr.data_ptr(), 512, 512, 1, 0, 1 + si])
            self._pack_desc = torch.tensor(rows, dtype=torch.int64, device=dev)
            self._pack_desc_ptrs = tuple(r[0] for r in rows)
            self._pack_tiles = max(((r[3] + 31) // 32) * ((r[4] + 31) // 32) for r in rows)
        # one launch for every layer (descriptor rows hold the fp32 master pointers,
        # which the flat arena keeps fixed; rebuilt if a weight tensor moved)
        cur = tuple(s.module.weight.data_ptr() for s in self.front + self.back) + \
            tuple(self.ctx2[sc].weight.data_ptr() for sc in CONTEXT_SCALES) * 2
        if cur != self._pack_desc_ptrs:
            self._pack_desc = None
            return self.refresh_packs(force=True)
        self.C.pack_multi(self._pack_desc.data_ptr(), self._pack_desc.shape[0], self._pack_tiles, self.dt, st)
        self._pack_version = ver

    def mark_weights_updated(self):
        """Called by the fused optimizer after it has re-packed (keeps versions in sync)."""
        self._pack_version = self._weights_version()

    def _stream(self):
        return self.stream_override if self.stream_override is not None else _ext.stream_ptr()

    def workspace(self, n, h, w):
        """Size the shared wgrad slab workspace for an input of [n,3,h,w] (call before graph capture)."""
        if self.ws is None:
            self.ws = C.WgradWorkspace(self.head.weight.device)
        need = 0
        hh, ww = h, w
        for s in self.front:
            _, _, _, nd = self.ws.plan(n * hh * ww, 4 if s.first else s.cin, s.cout, 3, s.first, 1, ww)
            need = max(need, nd)
            if s.pool_after:
                hh, ww = hh // 2, ww // 2
        for s in self.back:
            need = max(need, self.ws.plan(n * hh * ww, s.cin, s.cout, 3, False, s.dil, ww)[3])
        need = max(need, self.ws.plan(n * hh * ww, 512, 512, 1, False)[3])
        need = max(need, self.ws.plan(n * hh * ww, 512, 4 * 512, 1, False)[3])    # linearised context dW2cat
        need = max(need, max(C.wgrad_1x1_batched_plan(n * hh * ww, 4, 512, 512, ncu=c)[2] for c in (128, 192, 224, 256)))
        self.ws.reserve(need)
        if dispatch.current().w1g:
            self._w1g_slabs(self.head.weight.device)
        return self.ws

    def _w1g_ok(self, x) -> bool:
        """conv1_1's weight gradient fused into conv1_2's data gradient (conv_dgrad_w1g; CANNET_W1G=0: separate
        weight-gradient launch on the side stream).  Measured 453.5 -> 456.7 img/s, peak HBM 8.75 -> 7.95 GB
        (profiles/r2/ab_w1g.txt)."""
        f0, f1 = self.front[0], self.front[1]
        return (dispatch.current().w1g and f0.first and f0.cout == 64 and f1.cin == 64
                and f1.cout == 64 and not f0.pool_after and x.dim() == 4 and x.shape[-1] == 64)

    def _w1g_slabs(self, device):
        if self._w1g_buf is None or self._w1g_buf[0].device != device:
            cap = C.w1g_slab_cap(device)
            self._w1g_buf = (torch.empty(cap, 36 * 64, dtype=torch.float32, device=device),
                             torch.empty(cap, 64, dtype=torch.float32, device=device))
        return self._w1g_buf

    # ----------------------------------------------------------- forward
    def _conv(self, s: ConvSpec, x, epi=C.EPI_BIAS_RELU):
        fwd, _ = self.packs[id(s.module.weight)]
        return C.conv_igemm(x, fwd, s.module.bias.detach(), ksize=s.ksize, dil=s.dil, epi=epi, first=s.first)

    def _pool_fused(self, s: ConvSpec, x) -> bool:
        """The 2x2 max-pool after this conv runs in the conv's epilogue (LDS-DMA kernels; conv1_2: the halo
        kernel's epilogue through an LDS staging tile).  Dispatch pool_fwd_fused = 0: separate pool kernel."""
        return (s.pool_after and not s.first and s.dil == 1 and (s.cin != 64 or s.cout == 64)
                and dispatch.current().pool_fwd_fused and C.conv_pool_fwd_ok(x, s.cout, s.ksize))

    def _maxpool(self, x):
        """(pooled, max-pool codes): the codes replace the pool input in the saved state."""
        n, h, w, c = x.shape
        y = torch.empty(n, h // 2, w // 2, c, dtype=self.act, device=x.device)
        codes = torch.empty(n, h // 2, w // 2, c // 8, dtype=torch.int32, device=x.device)
        self.C.maxpool_fwd(x.data_ptr(), y.data_ptr(), n, h, w, c, self.dt, self._stream(), codes.data_ptr())
        return y, codes

    def _img(self, img):
        if img.dim() == 4 and img.shape[-1] == 4 and img.dtype in C.ACT_DTYPES:
            if img.dtype != self.act:
                raise ValueError(f"NHWC4 input is {img.dtype}, the executor computes in {self.act}")
            # already in the first layer's NHWC4 layout (ops/preprocess.py)
            if img.shape[1] % 8 or img.shape[2] % 8:
                raise ValueError("H, W must be multiples of 8")
            return img.contiguous()
        if img.dim() != 4 or img.shape[1] != 3:
            raise ValueError("input must be [N,3,H,W]")
        n, _, h, w = img.shape
        if h % 8 or w % 8:
            raise ValueError(f"H, W must be multiples of 8 (got {h}x{w}); resize as CrowdDataset does")
        img = img.float().contiguous()
        x4 = torch.empty(n, h, w, 4, dtype=self.act, device=img.device)
        self.C.img_to_nhwc4(img.data_ptr(), x4.data_ptr(), n, h, w, self.dt, self._stream())
        return x4

    def forward_features(self, img, save: bool):
        """Runs everything up to the last backend ReLU. Returns (b6 [N,h,w,64], saved dict)."""
        self.refresh_packs()
        sv = {} if save else None
        x = self._img(img)
        acts = []   # conv inputs of the frontend
        pre_pool = {}
        for s in self.front:
            acts.append(x)
            if self._pool_fused(s, x):
                # conv + ReLU + pool in one kernel; only the pooled map and the max-pool codes are written
                # (the full-resolution output is never stored: the backward needs the codes alone)
                fwd, _ = self.packs[id(s.module.weight)]
                _, x, codes = C.conv_pool_fwd(x, fwd, s.module.bias.detach(), ksize=s.ksize, dil=s.dil,
                                              keep_full=False, codes=save)
                if save:
                    pre_pool[s.idx] = codes
                continue
            else:
                y = self._conv(s, x)
            if s.pool_after:
                x, codes = self._maxpool(y)
                pre_pool[s.idx] = codes
            else:
                x = y
        fv = x
        cat, ctx_saved = self._context_fwd(fv, save)
        x = cat
        back_in = []
        for s in self.back:
            back_in.append(x)
            x = self._conv(s, x)
        if save:
            sv.update(front_in=acts, pre_pool=pre_pool, fv=fv, ctx=ctx_saved, back_in=back_in, b6=x)
        return x, sv

    @staticmethod
    def _ctx_linear(fv) -> bool:
        """The context module as one GEMM each way (conv_igemm.hip "Linearised context module"); dispatch ctx_linear =
        0 or a map narrower than 64 columns: the direct per-scale form (expand -> 4 sigmoid GEMMs -> fuse)."""
        return bool(dispatch.current().ctx_linear) and C.ctx_linear_ok(fv)

    def _context_fwd(self, fv, save):
        if self._ctx_linear(fv):
            return self._context_fwd_linear(fv, save)
        n, h, w, c = fv.shape
        st = self._stream()
        rowacc = torch.empty(n, h, 12, c, dtype=torch.float32, device=fv.device)
        ave = torch.empty(n, 50, c, dtype=torch.float32, device=fv.device)
        self.C.ctx_reduce(0, fv.data_ptr(), 0, 0, rowacc.data_ptr(), ave.data_ptr(), n, h, w, c, self.dt, st)
        # conv{S}_1 on the pooled grids: the four scales' fp32 GEMMs in one launch
        table = torch.empty_like(ave)
        self.C.ctx_gemm(0, ave.data_ptr(), 0, self._ctx1_ptrs(), table.data_ptr(), [], n, c, 0.0, 1.0, 0, st)
        cs = torch.empty(4, n, h, w, c, dtype=self.act, device=fv.device)
        self.C.ctx_expand(fv.data_ptr(), table.data_ptr(), cs.data_ptr(), n, h, w, c, self.dt, st)
        wts = torch.empty(4, n, h, w, c, dtype=self.act, device=fv.device)
        if self._ctx_batched(h, w):
            C.conv_igemm_batched(cs, self.ctx2_fwd, ksize=1, epi=C.EPI_SIGMOID, out=wts)   # one launch
        else:
            for i, sc in enumerate(CONTEXT_SCALES):
                fwd, _ = self.packs[id(self.ctx2[sc].weight)]
                C.conv_igemm(cs[i], fwd, None, ksize=1, epi=C.EPI_SIGMOID, out=wts[i])
        cat = torch.empty(n, h, w, 2 * c, dtype=self.act, device=fv.device)
        self.C.ctx_fuse(fv.data_ptr(), wts.data_ptr(), table.data_ptr(), cat.data_ptr(), n, h, w, c, self.dt, st)
        saved = dict(ave=ave, table=table, cs=cs, wts=wts, rowacc=rowacc) if save else None
        return cat, saved

    def _context_fwd_linear(self, fv, save):
        n, h, w, c = fv.shape
        st = self._stream()
        rowacc = torch.empty(n, h, 12, c, dtype=torch.float32, device=fv.device)
        ave = torch.empty(n, 50, c, dtype=torch.float32, device=fv.device)
        self.C.ctx_reduce(0, fv.data_ptr(), 0, 0, rowacc.data_ptr(), ave.data_ptr(), n, h, w, c, self.dt, st)
        u = torch.empty_like(ave)            # conv{S}_1 on the pooled cells
        self.C.ctx_gemm(0, ave.data_ptr(), 0, self._ctx1_ptrs(), u.data_ptr(), [], n, c, 0.0, 1.0, 0, st)
        t = torch.empty_like(ave)            # conv{S}_2 on the same cells (its upsample is z's first term)
        self.C.ctx_gemm(0, u.data_ptr(), 0, self._ctx2_ptrs(), t.data_ptr(), [], n, c, 0.0, 1.0, 0, st)
        wts, cat = C.conv_ctx_fwd(fv, self.ctx2cat_fwd, t, u)
        saved = dict(linear=True, ave=ave, u=u, wts=wts) if save else None
        return cat, saved

    def _ctx2_ptrs(self):
        ws = [self.ctx2[sc].weight for sc in CONTEXT_SCALES]
        for w_ in ws:
            if not (w_.is_contiguous() and w_.dtype == torch.float32):
                raise ValueError("conv{S}_2 weights must be contiguous fp32")
        return [w_.data_ptr() for w_ in ws]

    @staticmethod
    def _ctx_batched(h, w):
        """The four conv{S}_2 1x1 convs as one batched launch (dispatch ctx_batched = 0: four launches)."""
        return h >= 2 and w >= 2 and bool(dispatch.current().ctx_batched)

    def _ctx1_ptrs(self):
        ws = [self.ctx1[sc].weight for sc in CONTEXT_SCALES]
        for w_ in ws:
            if not (w_.is_contiguous() and w_.dtype == torch.float32):
                raise ValueError("conv{S}_1 weights must be contiguous fp32")
        return [w_.data_ptr() for w_ in ws]

    def head_forward(self, b6):
        n, h, w, _ = b6.shape
        et = torch.empty(n, 1, h, w, dtype=torch.float32, device=b6.device)
        self.C.head_fwd(b6.data_ptr(), self.head.weight.detach().data_ptr(), self.head.bias.detach().data_ptr(),
                        et.data_ptr(), n * h * w, self.dt, self._stream())
        return et

    @torch.no_grad()
    def forward_eval(self, img):
        b6, _ = self.forward_features(img, save=False)
        return self.head_forward(b6)

    # ----------------------------------------------------------- backward
    def backward_features(self, sv, d_b6: torch.Tensor, grads: Sequence[Optional[torch.Tensor]],
                          on_grad_ready: Optional[Callable[[List[int]], None]] = None, beta: float = 0.0,
                          scale: float = 1.0, dscale: Optional[torch.Tensor] = None):
        """d_b6: grad wrt the PRE-activation of the last backend conv (ReLU already applied).

        grads[i] is the fp32 output tensor for model.parameters()[i] (written, or
        accumulated when beta=1).  Entries for the head must already be filled.
        dscale: optional fp32 device scalar multiplied into every weight gradient
        (1 / loss scale when d_b6 carries a loss scale, fp16 step).
        (A data-gradient chain on a high-priority stream measured neutral: profiles/r4/ab_confirm.txt.)
        """
        st = self._stream()
        ws = self.ws or self.workspace(*self._shape_from(sv))
        ready = on_grad_ready or (lambda idx: None)
        side = self._side_stream()
        hold = []          # operands of side-stream work, kept alive until the join below

        # the data-gradient epilogues also sum the bias gradient of the dY they write, so the weight-gradient
        # launch need not re-read dY for db (the bias column sums were ~1 ms/step of weight-gradient-stream
        # time).  Round 2 measured it negative (421-423 vs 427 img/s, profiles/r2/README.md); after the round-3
        # kernel changes it is ahead in every interleaved round (485.5-485.8 vs 483.3-485.1 img/s,
        # profiles/r3/ab_bias_fused.txt), so it is the default; dispatch bias_fused = 0 re-reads dY
        fuse_bias = bool(dispatch.current().bias_fused)

        def wg(spec_or_w, dy, x, ksize, dil, first, wi, bi, bp=None, wbeta=None, mark=True):
            # bp: bias partials of dy summed by the data-gradient epilogue that wrote it (None: the weight-
            # gradient launch re-reads dy for the bias); wbeta / mark: a later image chunk accumulates (beta 1) and
            # only the last one marks the gradient ready
            def run():
                C.conv_wgrad(dy, x, grads[wi], grads[bi] if bi is not None else None, ksize=ksize, dil=dil,
                             first=first, ws=ws, beta=beta if wbeta is None else wbeta, scale=scale, dscale=dscale,
                             bias_partials=bp)
                if mark:
                    ready([wi] + ([bi] if bi is not None else []))
            self._on_side(side, run, hold, dy, x, *(() if bp is None else (bp,)))

        def dgrad(dy, dgr, dil, epi, mask):
            """Data gradient; returns (dX, bias partials of dX or None)."""
            if fuse_bias:
                return C.conv_dgrad_with_bias(dy, dgr, ksize=3, dil=dil, epi=epi, mask=mask)
            return C.conv_igemm(dy, dgr, None, ksize=3, dil=dil, epi=epi, mask=mask), None

        # ---- backend, reverse
        dy, bp = d_b6, None
        for s in reversed(self.back):
            x = sv["back_in"][s.idx]
            wg(s, dy, x, 3, s.dil, False, s.w_index, s.b_index, bp)
            _, dgr = self.packs[id(s.module.weight)]
            if s.idx > 0:
                dy, bp = dgrad(dy, dgr, s.dil, C.EPI_MASK, x)
            else:
                dcat = C.conv_igemm(dy, dgr, None, ksize=3, dil=s.dil, epi=C.EPI_NONE)
        # ---- context module
        dy = self._context_bwd(sv["ctx"], sv["fv"], dcat, grads, ws, beta, scale, ready, dscale, side, hold)
        # ---- frontend, reverse
        bp = None
        for s in reversed(self.front):
            x = sv["front_in"][s.idx]
            wg(s, dy, x, 3, 1, s.first, s.w_index, s.b_index, bp)
            if s.idx == 0:
                break
            _, dgr = self.packs[id(s.module.weight)]
            prev = self.front[s.idx - 1]
            if s.idx == 1 and prev.first and self._w1g_ok(x):
                # conv1_2's data gradient with conv1_1's weight gradient fused (compute stream): conv1_1's dY is
                # consumed tile by tile inside the kernel, never written to or re-read from memory
                img = sv["front_in"][0]
                sl, bsl = self._w1g_slabs(x.device)
                C.conv_dgrad_w1g(dy, dgr, x, img, grads[prev.w_index], grads[prev.b_index], slabs=sl, bslabs=bsl,
                                 beta=beta, scale=scale, dscale=dscale)
                if side is not None:
                    # join before marking ready: the bucket holding conv1_1 also holds side-stream gradients, and a
                    # transport that orders its all-reduce after the marking stream must see them too
                    torch.cuda.current_stream(d_b6.device).wait_stream(side)
                ready([prev.w_index, prev.b_index])
                break
            if prev.pool_after:
                # data gradient at the pooled resolution, scattered through the max-pool backward
                # (+ ReLU mask of the pool input) in the conv epilogue: the pooled gradient never
                # round-trips through memory
                codes = sv["pre_pool"][prev.idx]
                # (conv2_1's data gradient / conv1_2's weight gradient in image halves measured -0.5 %:
                # profiles/r4/ab_tail_split.txt)
                if dispatch.current().poolbwd_fused:
                    dy, bp = dgrad(dy, dgr, 1, C.EPI_POOLBWD, codes)
                else:
                    dp = C.conv_igemm(dy, dgr, None, ksize=3, dil=1, epi=C.EPI_NONE)
                    dy, bp = C.maxpool_bwd_codes(codes, dp), None
            else:
                dy, bp = dgrad(dy, dgr, 1, C.EPI_MASK, x)
        if side is not None:
            torch.cuda.current_stream(d_b6.device).wait_stream(side)     # join: every gradient written
        hold.clear()

    def _side_stream(self):
        """Weight gradients run on a second stream, concurrently with the data-gradient chain (they only
        need the layer's dY and input).  The memory-bound slab reductions / bias column sums and the
        partial last waves of one chain fill the CUs the other leaves idle.  Fork/join through stream
        waits, so the pattern is hipGraph-capturable; dispatch wgrad_stream = 0 runs everything in order.  (A
        high-priority side stream measured negative, profiles/r2/ab_side_priority_negative.txt.)"""
        if not dispatch.current().wgrad_stream or self.stream_override is not None:
            return None
        dev = self.head.weight.device
        if self._side is None or self._side.device != dev:
            self._side = torch.cuda.Stream(dev)
        return self._side

    @staticmethod
    def _on_side(side, fn, hold, *keep):
        if side is None:
            fn()
            return
        side.wait_stream(torch.cuda.current_stream(side.device))           # fork after the producers
        with torch.cuda.stream(side):
            fn()
        hold.extend(keep)

    def _context_bwd_linear(self, ctx, fv, dcat, grads, ws, beta, scale, ready, dscale=None, side=None, hold=None):
        """Backward of the linearised context module (see _context_fwd_linear); returns d(F10 pre-activation)."""
        st = self._stream()
        n, h, w, c = fv.shape
        hold = [] if hold is None else hold
        dg, rowacc = C.ctx_bwd_lin(dcat, ctx["wts"], ctx["u"])        # dG = -dz, x-pass partials of up^T
        dt = torch.empty(n, 50, c, dtype=torch.float32, device=fv.device)
        du = torch.empty_like(dt)
        self.C.ctx_cells(rowacc[0].data_ptr(), dt.data_ptr(), n, h, c, st)     # dt_S = up^T(dz_S)
        self.C.ctx_cells(rowacc[1].data_ptr(), du.data_ptr(), n, h, c, st)     # du_S = up^T(ds_S)   (direct part)
        u, ave = ctx["u"], ctx["ave"]
        dw2 = [grads[self.ctx2_index[sc]] for sc in CONTEXT_SCALES]
        for g in dw2:
            if not (g.is_contiguous() and g.dtype == torch.float32):
                raise ValueError("conv{S}_2 gradient buffers must be contiguous fp32")
        if getattr(self, "_dw2cat", None) is None or self._dw2cat.device != fv.device:
            self._dw2cat = torch.empty(4 * c, c, 1, 1, dtype=torch.float32, device=fv.device)
        dw2cat = self._dw2cat
        dsp = dscale.data_ptr() if dscale is not None else 0

        # du_S += W2_S^T dt_S, then dave_S = W1_S^T du_S (fp32 cell GEMMs).  Both before the side-stream fork:
        # forked first, the dW2cat weight gradient takes every CU (one 128-KB-LDS block each) and these two short
        # launches wait ~190 us behind it on the critical path
        self.C.ctx_gemm(1, dt.data_ptr(), 0, self._ctx2_ptrs(), du.data_ptr(), [], n, c, 1.0, 1.0, 0, st)
        dave = torch.empty_like(du)
        self.C.ctx_gemm(1, du.data_ptr(), 0, self._ctx1_ptrs(), dave.data_ptr(), [], n, c, 0.0, 1.0, 0, st)

        def ctx2_wgrad():
            # dW2_S = dG_S^T fv (one GEMM over the interleaved columns) + dt_S^T u_S (the t = W2 u term)
            C.conv_wgrad(dg, fv, dw2cat, None, ksize=1, ws=ws, beta=0.0, scale=scale, dscale=dscale)
            self.C.ctx_w2_scatter(dw2cat.data_ptr(), [g.data_ptr() for g in dw2], c, float(beta), self._stream())
            self.C.ctx_gemm(2, dt.data_ptr(), u.data_ptr(), [], 0, [g.data_ptr() for g in dw2], n, c, 1.0,
                            float(scale), dsp, self._stream())
            ready([self.ctx2_index[sc] for sc in CONTEXT_SCALES])
        self._on_side(side, ctx2_wgrad, hold, dg, fv, dt, u)

        def ctx1_wgrad():
            gws = [grads[self.ctx1_index[sc]] for sc in CONTEXT_SCALES]
            for g in gws:
                if not (g.is_contiguous() and g.dtype == torch.float32):
                    raise ValueError("conv{S}_1 gradient buffers must be contiguous fp32")
            self.C.ctx_gemm(2, du.data_ptr(), ave.data_ptr(), [], 0, [g.data_ptr() for g in gws], n, c, float(beta),
                            float(scale), dsp, self._stream())
            ready([self.ctx1_index[sc] for sc in CONTEXT_SCALES])
        self._on_side(side, ctx1_wgrad, hold, du, ave)
        hold.append(rowacc)
        return C.conv_ctx_bwd(dg, self.ctx2cat_dgr, dave, dcat, fv)

    def _context_bwd(self, ctx, fv, dcat, grads, ws, beta, scale, ready, dscale=None, side=None, hold=None):
        """Backward of the context module; returns d(F10 pre-activation) (ReLU mask of fv applied)."""
        if ctx.get("linear"):
            return self._context_bwd_linear(ctx, fv, dcat, grads, ws, beta, scale, ready, dscale, side, hold)
        st = self._stream()
        n, h, w, c = fv.shape
        dz = torch.empty(4, n, h, w, c, dtype=self.act, device=fv.device)
        sdir = torch.empty_like(dz)
        self.C.ctx_bwd_e1(dcat.data_ptr(), ctx["wts"].data_ptr(), ctx["table"].data_ptr(), dz.data_ptr(),
                          sdir.data_ptr(), n, h, w, c, self.dt, st)
        dc = torch.empty_like(dz)
        if self._ctx_batched(h, w):
            C.conv_igemm_batched(dz, self.ctx2_dgr, ksize=1, epi=C.EPI_NONE, out=dc)
        else:
            for i, sc in enumerate(CONTEXT_SCALES):
                _, dgr = self.packs[id(self.ctx2[sc].weight)]
                C.conv_igemm(dz[i], dgr, None, ksize=1, epi=C.EPI_NONE, out=dc[i])
        # the four conv{S}_2 weight gradients: one batched GEMM when their arena slots are adjacent
        dws = [grads[self.ctx2_index[sc]] for sc in CONTEXT_SCALES]

        def ctx2_wgrad():
            if C.wgrad_1x1_batched_ok(dz, ctx["cs"], dws):
                C.conv_wgrad_1x1_batched(dz, ctx["cs"], dws, ws=ws, beta=beta, scale=scale, dscale=dscale)
            else:
                for i, sc in enumerate(CONTEXT_SCALES):
                    C.conv_wgrad(dz[i], ctx["cs"][i], dws[i], None, ksize=1, ws=ws, beta=beta, scale=scale,
                                 dscale=dscale)
            ready([self.ctx2_index[sc] for sc in CONTEXT_SCALES])
        hold = [] if hold is None else hold
        self._on_side(side, ctx2_wgrad, hold, dz)
        rowacc = ctx["rowacc"]
        dA = torch.empty(n, 50, c, dtype=torch.float32, device=fv.device)
        self.C.ctx_reduce(1, 0, sdir.data_ptr(), dc.data_ptr(), rowacc.data_ptr(), dA.data_ptr(), n, h, w, c, self.dt,
                          st)
        dave = torch.empty_like(dA)
        ave = ctx["ave"]

        def ctx1_wgrad():
            # dW1_S = dA_S^T @ ave_S for the four scales, one launch (on the weight-gradient stream)
            gws = [grads[self.ctx1_index[sc]] for sc in CONTEXT_SCALES]
            for g in gws:
                if not (g.is_contiguous() and g.dtype == torch.float32):
                    raise ValueError("conv{S}_1 gradient buffers must be contiguous fp32")
            self.C.ctx_gemm(2, dA.data_ptr(), ave.data_ptr(), [], 0, [g.data_ptr() for g in gws], n, c, float(beta),
                            float(scale), dscale.data_ptr() if dscale is not None else 0, self._stream())
            ready([self.ctx1_index[sc] for sc in CONTEXT_SCALES])
        self._on_side(side, ctx1_wgrad, hold, dA, ave)
        self.C.ctx_gemm(1, dA.data_ptr(), 0, self._ctx1_ptrs(), dave.data_ptr(), [], n, c, 0.0, 1.0, 0, st)
        dfv = torch.empty(n, h, w, c, dtype=self.act, device=fv.device)
        self.C.ctx_bwd_final(dcat.data_ptr(), dc.data_ptr(), dave.data_ptr(), fv.data_ptr(), dfv.data_ptr(), n, h, w,
                             c, self.dt, st)
        return dfv

    @staticmethod
    def _shape_from(sv):
        x0 = sv["front_in"][0]
        return x0.shape[0], x0.shape[1], x0.shape[2]

    @staticmethod
    def input_hw(img):
        """(N, H, W) of an NCHW image batch or an NHWC4 prepacked batch."""
        if img.dim() == 4 and img.shape[-1] == 4 and img.dtype in C.ACT_DTYPES:
            return img.shape[0], img.shape[1], img.shape[2]
        return img.shape[0], img.shape[2], img.shape[3]

    # ----------------------------------------------------------- training head
    def head_train(self, b6, gt, grads, gscale: float = 1.0, beta: float = 0.0,
                   lscale: Optional[torch.Tensor] = None, flags: Optional[torch.Tensor] = None):
        """Fused: et, MSE(sum) loss, d(et), d(b6 pre-act) (ReLU-masked), head grads. Returns (loss, et, d_b6).
        lscale: optional fp32 device scalar (loss scale) applied to d_b6 only; head grads stay unscaled.
        flags: optional fp32 device vector; the loss is written to flags[1] and its non-finite flag
        (1.0 / 0.0) to flags[0] by the same reduction kernel (the returned loss is then flags[1:2])."""
        n, h, w, c = b6.shape
        if tuple(gt.shape) != (n, 1, h, w):
            raise ValueError(f"gt shape {tuple(gt.shape)} != {(n, 1, h, w)}")
        gt = gt.float().contiguous()
        P = n * h * w
        et = torch.empty(n, 1, h, w, dtype=torch.float32, device=b6.device)
        d_b6 = torch.empty_like(b6)
        nblk = max(1, min(1024, (P * 8 + 255) // 256))
        part = torch.empty(nblk, 66, dtype=torch.float32, device=b6.device)
        if flags is not None:
            if not (flags.dtype == torch.float32 and flags.is_contiguous() and flags.numel() >= 2):
                raise ValueError("flags must be a contiguous fp32 vector of >= 2 elements")
            loss, nf = flags[1:2], flags.data_ptr()
        else:
            loss, nf = torch.empty(1, dtype=torch.float32, device=b6.device), 0
        self.C.head_train(b6.data_ptr(), self.head.weight.detach().data_ptr(), self.head.bias.detach().data_ptr(),
                          gt.data_ptr(), et.data_ptr(), d_b6.data_ptr(), part.data_ptr(), nblk,
                          grads[self.head_w_index].data_ptr(), grads[self.head_b_index].data_ptr(), loss.data_ptr(),
                          P, float(gscale), float(beta), lscale.data_ptr() if lscale is not None else 0, nf, self.dt,
                          self._stream())
        return loss, et, d_b6

    # ----------------------------------------------------------- autograd entry
    def __call__(self, img: torch.Tensor) -> torch.Tensor:
        if not torch.is_grad_enabled() or not any(p.requires_grad for p in self._params()):
            return self.forward_eval(img)
        return _CANNetFn.apply(img, self, *self._params())


class _CANNetFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, img, ex: CANNetExecutor, *params):
        b6, sv = ex.forward_features(img, save=True)
        et = ex.head_forward(b6)
        ctx.ex = ex
        ctx.sv = sv
        ctx.b6 = b6
        return et

    @staticmethod
    def backward(ctx, g_et):
        ex: CANNetExecutor = ctx.ex
        params = ex._params()
        grads = [torch.empty_like(p, dtype=torch.float32) for p in params]
        b6 = ctx.b6
        n, h, w, c = b6.shape
        g = g_et.float().reshape(n, h, w, 1)
        b6f = b6.float()
        hw = ex.head.weight.detach().view(1, c)
        d_b6 = (g * hw * (b6f > 0)).to(ex.act).contiguous()
        grads[ex.head_w_index].copy_((g * b6f).sum(dim=(0, 1, 2)).view_as(params[ex.head_w_index]))
        grads[ex.head_b_index].copy_(g.sum().view(1))
        ex.workspace(*CANNetExecutor._shape_from(ctx.sv))
        ex.backward_features(ctx.sv, d_b6, grads)
        ctx.sv = None
        return (None, None) + tuple(gr.to(p.dtype) for gr, p in zip(grads, params))
