"""Per-component numerics of the native executor vs plain fp32 PyTorch, and determinism."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
BF16 = torch.bfloat16


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def test_maxpool_fwd_bwd():
    from can_distributed_pytorch_amd.ops import _ext
    C = _ext.require()
    torch.manual_seed(0)
    n, h, w, c = 2, 12, 20, 64
    x = torch.relu(torch.randn(n, h, w, c, device="cuda")).to(BF16)
    y = torch.empty(n, h // 2, w // 2, c, dtype=BF16, device="cuda")
    C.maxpool_fwd(x.data_ptr(), y.data_ptr(), n, h, w, c, 0, _ext.stream_ptr())
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    yr = F.max_pool2d(xr, 2, 2)
    assert torch.equal(y.float(), yr.detach().permute(0, 2, 3, 1))
    g = torch.randn(n, h // 2, w // 2, c, device="cuda").to(BF16)
    (gx,) = torch.autograd.grad(yr, xr, g.float().permute(0, 3, 1, 2))
    ref = gx.permute(0, 2, 3, 1) * (x.float() > 0)
    dx = torch.empty_like(x)
    C.maxpool_bwd_relu(x.data_ptr(), g.data_ptr(), dx.data_ptr(), n, h, w, c, 0, _ext.stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(dx.float(), ref)
    # max-pool codes: the backward from the codes alone (the pool input is not kept) is the same map
    from can_distributed_pytorch_amd.ops import conv as CV
    x[:, ::2, ::2, ::3] = 0                                   # ties (first max wins) and zero windows
    y2, codes = CV.maxpool_codes(x)
    assert torch.equal(y2.float(), F.max_pool2d(x.float().permute(0, 3, 1, 2), 2).permute(0, 2, 3, 1))
    dx2 = CV.maxpool_bwd_codes(codes, g)
    C.maxpool_bwd_relu(x.data_ptr(), g.data_ptr(), dx.data_ptr(), n, h, w, c, 0, _ext.stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(dx2, dx)


def _ctx_ref(fv, w1, w2):
    """Reference context module (model/CANNet.py:42-87) on NCHW fp32."""
    h, w = fv.shape[2], fv.shape[3]
    num = den = None
    for s in (1, 2, 3, 6):
        ave = F.conv2d(F.adaptive_avg_pool2d(fv, (s, s)), w1[s])
        up = F.interpolate(ave, size=(h, w), mode="bilinear", align_corners=True)
        wt = torch.sigmoid(F.conv2d(up - fv, w2[s]))
        num = wt * up if num is None else num + wt * up
        den = wt if den is None else den + wt
    return torch.cat((fv, num / (den + 1e-12)), 1)


@pytest.mark.parametrize("n,h,w", [(2, 12, 16), (1, 13, 22), (2, 96, 128), (1, 67, 45)])
def test_context_fwd_bwd(n, h, w):
    from can_distributed_pytorch_amd.models import CANNet
    from can_distributed_pytorch_amd.ops.executor import CANNetExecutor
    torch.manual_seed(1)
    model = CANNet().cuda()
    for s in (1, 2, 3, 6):
        torch.nn.init.normal_(getattr(model, f"conv{s}_1").weight, std=0.05)
        torch.nn.init.normal_(getattr(model, f"conv{s}_2").weight, std=0.05)
    ex = CANNetExecutor(model)
    ex.refresh_packs(force=True)
    fv = torch.relu(torch.randn(n, h, w, 512, device="cuda")).to(BF16)
    cat, saved = ex._context_fwd(fv, save=True)
    w1 = {s: getattr(model, f"conv{s}_1").weight.detach() for s in (1, 2, 3, 6)}
    w2 = {s: getattr(model, f"conv{s}_2").weight.detach().to(BF16).float() for s in (1, 2, 3, 6)}
    fvr = fv.float().permute(0, 3, 1, 2).contiguous().requires_grad_(True)
    w1r = {s: v.clone().requires_grad_(True) for s, v in w1.items()}
    w2r = {s: v.clone().requires_grad_(True) for s, v in w2.items()}
    ref = _ctx_ref(fvr, w1r, w2r)
    e = _rel(cat.float().permute(0, 3, 1, 2), ref)
    assert e < 1e-2, f"context fwd rel err {e}"
    # backward through the executor's context path only
    dcat = torch.randn(n, h, w, 1024, device="cuda").to(BF16)
    grads = [torch.zeros_like(p) for p in model.parameters()]
    gref = torch.autograd.grad(ref, [fvr] + [w1r[s] for s in (1, 2, 3, 6)] + [w2r[s] for s in (1, 2, 3, 6)],
                               dcat.float().permute(0, 3, 1, 2))
    dfv = ex._context_bwd(saved, fv, dcat, grads, ex.workspace(n, 8 * h, 8 * w), beta=0.0, scale=1.0,
                          ready=lambda idx: None)
    ref_dfv = gref[0].permute(0, 2, 3, 1) * (fv.float() > 0)
    e = _rel(dfv, ref_dfv)
    assert e < 3e-2, f"dfv rel err {e}"
    for k, s in enumerate((1, 2, 3, 6)):
        e1 = _rel(grads[ex.ctx1_index[s]], gref[1 + k])
        e2 = _rel(grads[ex.ctx2_index[s]], gref[5 + k])
        assert e1 < 3e-2 and e2 < 3e-2, (s, e1, e2)


def test_head_train():
    from can_distributed_pytorch_amd.models import CANNet
    from can_distributed_pytorch_amd.ops.executor import CANNetExecutor
    torch.manual_seed(2)
    model = CANNet().cuda()
    torch.nn.init.normal_(model.output_layer.weight, std=0.1)
    torch.nn.init.constant_(model.output_layer.bias, 0.3)
    ex = CANNetExecutor(model)
    n, h, w = 2, 9, 14
    b6 = torch.relu(torch.randn(n, h, w, 64, device="cuda")).to(BF16)
    gt = torch.rand(n, 1, h, w, device="cuda")
    grads = [torch.zeros_like(p) for p in model.parameters()]
    loss, et, d_b6 = ex.head_train(b6, gt, grads)
    x = b6.float().permute(0, 3, 1, 2).requires_grad_(True)
    wr = model.output_layer.weight.detach().clone().requires_grad_(True)
    br = model.output_layer.bias.detach().clone().requires_grad_(True)
    out = F.conv2d(x, wr, br)
    lr = ((out - gt) ** 2).sum()
    gx, gw, gb = torch.autograd.grad(lr, (x, wr, br))
    assert abs(loss.item() - lr.item()) / lr.item() < 1e-4
    assert _rel(et, out) < 1e-4
    assert _rel(d_b6.float(), gx.permute(0, 2, 3, 1) * (b6.float() > 0)) < 1e-2
    assert _rel(grads[ex.head_w_index], gw) < 1e-4 and _rel(grads[ex.head_b_index], gb) < 1e-4


def test_kernels_deterministic():
    """Same inputs -> bitwise identical outputs (no races in the LDS-DMA pipelines)."""
    from can_distributed_pytorch_amd.ops import conv as C
    torch.manual_seed(3)
    for (n, h, w, ci, co, dil) in [(2, 48, 64, 256, 512, 2), (1, 96, 128, 64, 64, 1), (2, 24, 32, 512, 256, 1)]:
        x = torch.randn(n, h, w, ci, device="cuda").to(BF16)
        dy = torch.randn(n, h, w, co, device="cuda").to(BF16)
        wt = torch.randn(co, ci, 3, 3, device="cuda") * 0.05
        wf = C.pack_weight_fwd(wt)
        y1 = C.conv_igemm(x, wf, torch.zeros(co, device="cuda"), ksize=3, dil=dil)
        y2 = C.conv_igemm(x, wf, torch.zeros(co, device="cuda"), ksize=3, dil=dil)
        assert torch.equal(y1, y2)
        d1, d2 = torch.empty_like(wt), torch.empty_like(wt)
        b1, b2 = torch.empty(co, device="cuda"), torch.empty(co, device="cuda")
        C.conv_wgrad(dy, x, d1, b1, ksize=3, dil=dil)
        C.conv_wgrad(dy, x, d2, b2, ksize=3, dil=dil)
        torch.cuda.synchronize()
        assert torch.equal(d1, d2) and torch.equal(b1, b2)


def test_executor_deterministic():
    from can_distributed_pytorch_amd.models import CANNet
    torch.manual_seed(4)
    m = CANNet().cuda()
    x = torch.randn(2, 3, 64, 96, device="cuda")
    gt = torch.rand(2, 1, 8, 12, device="cuda")
    outs = []
    for _ in range(2):
        m.zero_grad(set_to_none=True)
        loss = torch.nn.MSELoss(reduction="sum")(m(x), gt)
        loss.backward()
        outs.append([loss.detach().clone()] + [p.grad.clone() for p in m.parameters()])
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_density_gpu_matches_cpu():
    import numpy as np
    from can_distributed_pytorch_amd.data.density import density_map_gpu, gaussian_filter_density
    rng = np.random.default_rng(5)
    h, w = 96, 128
    pts = np.stack([rng.random(300) * w, rng.random(300) * h], 1).astype(np.float32)
    ref = gaussian_filter_density((h, w), pts)
    got = density_map_gpu(pts, h, w).cpu().numpy()
    assert np.abs(got - ref).max() < 1e-4
    assert abs(got.sum() - ref.sum()) < 1e-2


@pytest.mark.parametrize("npts", [1, 3])
def test_density_gpu_large_radius_matches_cpu(npts):
    """Footprints wider than 1023 px: the single-head case sigma = (H+W)/8 = 224 at 768x1024 (R = 896) and
    three heads far apart (kNN sigmas ~ 0.1 * (d1+d2) >> 128).  Exact radius, mass outside the image dropped
    after normalising, as scipy's gaussian_filter on a delta (radius was clamped at 511)."""
    import numpy as np
    from can_distributed_pytorch_amd.data.density import density_map_gpu, gaussian_filter_density
    h, w = 768, 1024
    pts = np.array([[500.3, 380.7], [20.0, 30.0], [1000.0, 750.0]], dtype=np.float32)[:npts]
    ref = gaussian_filter_density((h, w), pts)
    got = density_map_gpu(pts, h, w).cpu().numpy()
    assert np.abs(got - ref).max() < 1e-7 + 1e-4 * np.abs(ref).max()
    assert abs(got.sum() - ref.sum()) < 1e-4 * npts


def test_no_uninitialized_reads_poisoned_allocator():
    """Regression: fill the caching allocator with NaN bit patterns before every
    buffer the executor allocates; outputs must not change (a NaN read from an
    unwritten pad once got silently zeroed by fmaxf in a ReLU epilogue)."""
    from can_distributed_pytorch_amd.models import CANNet
    torch.manual_seed(6)
    x = torch.randn(2, 3, 64, 96, device="cuda")
    outs = []
    for bits in (0, 0x7FC07FC0):
        m = CANNet().cuda()
        torch.manual_seed(7)
        for mod in m.modules():
            if isinstance(mod, torch.nn.Conv2d):
                torch.nn.init.normal_(mod.weight, std=0.05)
        t = torch.empty(256 * 1024 * 1024 // 4, dtype=torch.int32, device="cuda")
        t.fill_(bits)
        del t
        with torch.no_grad():
            outs.append(m(x))
        torch.cuda.synchronize()
    assert not torch.isnan(outs[1]).any()
    assert torch.equal(outs[0], outs[1])


def test_packed_batch_preprocess_matches_cpu_transform():
    """CrowdDataset(raw=True) items -> PackedCollate (in the loader workers) -> preprocess_packed (one H2D copy
    of the images, ONE launch for the batch) == data/transforms.prepare_pair per sample (cv2 INTER_LINEAR
    semantics), incl. flips, mixed source sizes that resize to one shape, gray images."""
    import numpy as np
    from can_distributed_pytorch_amd.data.dataset import density_to_gt
    from can_distributed_pytorch_amd.data.transforms import prepare_pair
    from can_distributed_pytorch_amd.ops.preprocess import PackedCollate, preprocess_packed
    rng = np.random.default_rng(9)
    shapes = [(77, 101, 3), (72, 96, 3), (79, 103, 1), (72, 100, 3)]        # all -> 72 x 96
    samples, refs = [], []
    for i, (h, w, c) in enumerate(shapes):
        img = (rng.random((h, w, c) if c > 1 else (h, w)) * 255).astype(np.uint8)
        dm = rng.random((h, w)).astype(np.float32)
        flip = bool(i % 2)
        samples.append((torch.from_numpy(img), torch.from_numpy(density_to_gt(dm, h, w, 8, flip)), flip))
        refs.append(prepare_pair(img, dm, 8, flip))
    packed = PackedCollate()(samples)
    x4, gt = preprocess_packed(packed, "cuda")
    assert tuple(x4.shape) == (4, 72, 96, 4) and tuple(gt.shape) == (4, 1, 9, 12)
    for i, (ri, rg) in enumerate(refs):
        got = x4[i, ..., :3].float().permute(2, 0, 1).cpu().numpy()
        assert np.abs(got - ri).max() < 0.03
        assert np.abs(gt[i].cpu().numpy() - rg).max() < 1e-5
    assert bool((x4[..., 3] == 0).all())


def test_synthetic_gpu_generator():
    """GPU-rendered synthetic crowds: count-preserving ground truth (sum = number of heads inside, up to the
    border mass), reproducible per seed to fp32 rounding (the density splat adds with fp32 atomics, so the
    last bits may differ run to run), NHWC4 with channel 3 zero, statistics of the CPU recipe."""
    from can_distributed_pytorch_amd.data.synthetic import make_synthetic_batch, make_synthetic_batch_gpu
    x4, gt = make_synthetic_batch_gpu(2, 128, 192, seeds=[5, 6], heads=(50, 60))
    x4b, gtb = make_synthetic_batch_gpu(2, 128, 192, seeds=[5, 6], heads=(50, 60))
    torch.cuda.synchronize()
    assert torch.allclose(x4.float(), x4b.float(), atol=2e-2) and torch.allclose(gt, gtb, rtol=1e-5, atol=1e-6)
    assert bool((x4[..., 3] == 0).all())
    counts = gt.flatten(1).sum(1)
    assert bool(((counts > 20) & (counts < 61)).all()), counts          # heads clamped to the border lose mass
    img_cpu, gt_cpu = make_synthetic_batch(2, 128, 192, seed=5, heads=(50, 60))
    assert abs(float(x4[..., :3].float().mean()) - float(img_cpu.mean())) < 0.5


def test_gpu_preprocess_matches_cpu_transform():
    """ops/preprocess (HIP) == data/transforms.prepare_pair (cv2 INTER_LINEAR semantics), incl. flip."""
    import numpy as np
    from can_distributed_pytorch_amd.data.transforms import prepare_pair
    from can_distributed_pytorch_amd.ops.preprocess import preprocess_batch
    rng = np.random.default_rng(8)
    for (h, w, c) in [(77, 101, 3), (64, 96, 3), (50, 70, 1)]:
        img = (rng.random((h, w, c) if c > 1 else (h, w)) * 255).astype(np.uint8)
        dm = rng.random((h, w)).astype(np.float32)
        for flip in (False, True):
            ref_img, ref_gt = prepare_pair(img, dm, 8, flip)
            x4, gt = preprocess_batch([torch.from_numpy(img)], [torch.from_numpy(dm)], [flip], "cuda")
            got = x4[0, ..., :3].float().permute(2, 0, 1).cpu().numpy()
            assert np.abs(got - ref_img).max() < 0.03          # bf16 storage of the normalised image
            assert bool((x4[0, ..., 3] == 0).all())
            assert np.abs(gt[0].cpu().numpy() - ref_gt).max() < 1e-3


@pytest.mark.parametrize("arena", [False, True])
def test_weight_packs_bitwise(arena):
    """One-launch weight packing (pack_multi: 16-B vector path for whole 32x32 tiles, element-wise otherwise) ==
    the Python packs of every layer, bitwise; arena=True: fp32 masters that are not 16-B aligned (element-wise
    loads, vector stores)."""
    from can_distributed_pytorch_amd.models import CANNet
    from can_distributed_pytorch_amd.ops import conv as C
    from can_distributed_pytorch_amd.ops.executor import CANNetExecutor
    torch.manual_seed(3)
    model = CANNet().cuda()
    for p in model.parameters():
        torch.nn.init.normal_(p, std=0.3)
    if arena:
        # masters as views at a 1-float offset of one buffer: no slot 16-B aligned -> element-wise loads
        ps = list(model.parameters())
        buf = torch.zeros(1 + sum(p.numel() for p in ps), device="cuda")
        off = 1
        with torch.no_grad():
            for p in ps:
                n = p.numel()
                buf[off:off + n].copy_(p.reshape(-1))
                p.data = buf[off:off + n].view_as(p)
                off += n
        assert any(p.data_ptr() % 16 for p in ps if p.dim() == 4 and p.shape[1] >= 64)
    ex = CANNetExecutor(model)
    ex.refresh_packs(force=True)
    torch.cuda.synchronize()
    for s in ex.front + ex.back:
        fwd, dgr = ex.packs[id(s.module.weight)]
        w = s.module.weight
        if s.first:
            assert torch.equal(fwd, C.pack_weight_first(w))
            continue
        assert torch.equal(fwd, C.pack_weight_fwd(w)), s.idx
        assert torch.equal(dgr, C.pack_weight_dgrad(w)), s.idx
    for sc in (1, 2, 3, 6):
        fwd, dgr = ex.packs[id(ex.ctx2[sc].weight)]
        assert torch.equal(fwd, C.pack_weight_fwd(ex.ctx2[sc].weight))
        assert torch.equal(dgr, C.pack_weight_dgrad(ex.ctx2[sc].weight))
