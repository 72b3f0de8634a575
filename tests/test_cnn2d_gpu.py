"""Per-frame 2-D CNN video backbones of the reference VideoEncoder (`video_backbone` 'resnet18' / 'mobilenet_v2',
src/models/models.py:163-173,208-216) on the MI355X, against the CPU restatement oracle/cnn2d_cpu.py (F.conv2d /
F.batch_norm / F.max_pool2d / F.relu6 on torchvision's architectures; parity unpinned w.r.t. the reference: torchvision
is absent here).

Kernels: MaxPool2d(3, 2, 1) forward and gather backward are exact (max / sums of ≤ 4 routed values) incl. tied
maxima (torch's first-maximum rule, checked against torch's CPU kernel); depthwise conv forward / input gradient /
weight gradient ≤ 1e-5 rel in fp32 (stride 1 and 2, 32..960 channels); channels-last BatchNorm with channel counts
that are not 8·2^j and ReLU6 ≤ 1e-5; weight packs bit-exact.  Backbones: fp32 features ≤ 1e-4 rel, every parameter
gradient ≤ 2e-3 rel, running statistics ≤ 1e-5; bf16 within 3× (+2e-3) of the error bf16 storage alone causes per
parameter (oracle re-run with bf16 rounding at the storage points); VideoEncoder output (per-frame projection + temporal
mean) ≤ 1e-4."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _equal_nan(a, b):
    return bool(((a == b) | (a.isnan() & b.isnan())).all())


def rel(a, b):
    a, b = torch.as_tensor(a).detach().double().cpu(), torch.as_tensor(b).detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize('nan', [False, True])
@pytest.mark.parametrize('dt', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('N,C,H,W', [(3, 64, 56, 56), (2, 16, 13, 11)])
def test_maxpool_fwd_bwd_with_ties(dt, N, C, H, W, nan):
    """`nan`: ~3 % NaN inputs — the NaN propagates as in torch (output NaN, gradient to the window's last
    NaN), instead of being skipped."""
    from cmhar import _lib as L
    torch.manual_seed(0)
    x = torch.randint(-3, 4, (N, C, H, W)).float()          # many tied maxima
    if nan:
        x[torch.rand(x.shape) < 0.03] = float('nan')
    xr = x.clone().requires_grad_(True)
    ref = F.max_pool2d(xr, 3, 2, 1)
    dy = torch.randint(-4, 5, ref.shape).float()
    ref.backward(dy)
    xc = x.permute(0, 2, 3, 1).contiguous().to(DEV, dt)
    Ho, Wo = ref.shape[2], ref.shape[3]
    y = torch.empty(N * Ho * Wo, C, dtype=dt, device=DEV)
    arg = torch.empty(N * Ho * Wo, C, dtype=torch.uint8, device=DEV)
    L.call('cmhar_maxpool2d_cl_fwd', L.dtype_code(dt), N, H, W, C, 3, 2, 1, xc.data_ptr(), y.data_ptr(),
           arg.data_ptr(), L.stream(xc.device))
    assert _equal_nan(y.float().cpu().view(N, Ho, Wo, C).permute(0, 3, 1, 2), ref.detach())
    assert (ref.isnan().any().item()) == nan
    dyc = dy.permute(0, 2, 3, 1).contiguous().to(DEV, dt)
    dx = torch.empty(N * H * W, C, dtype=dt, device=DEV)
    L.call('cmhar_maxpool2d_cl_bwd', L.dtype_code(dt), N, H, W, C, 3, 2, 1, dyc.data_ptr(), arg.data_ptr(),
           dx.data_ptr(), L.stream(xc.device))
    assert torch.equal(dx.float().cpu().view(N, H, W, C).permute(0, 3, 1, 2), xr.grad)


@pytest.mark.parametrize('C,s,HW', [(32, 1, (17, 19)), (144, 2, (28, 28)), (960, 1, (7, 7)), (96, 2, (15, 9))])
def test_depthwise_conv_fwd_dgrad_wgrad_fp32(C, s, HW):
    from cmhar import _lib as L
    from cmhar import kernels as K
    torch.manual_seed(1)
    N = 3
    H, W = HW
    x = torch.randn(N, C, H, W, requires_grad=True)
    w = (torch.randn(C, 1, 3, 3) * 0.3).requires_grad_(True)
    ref = F.conv2d(x, w, stride=s, padding=1, groups=C)
    dz = torch.randn_like(ref)
    ref.backward(dz)
    Ho, Wo = ref.shape[2:]
    xc = x.detach().permute(0, 2, 3, 1).contiguous().to(DEV)
    wc = w.detach().to(DEV)
    z = torch.empty(N * Ho * Wo, C, device=DEV)
    st = L.stream(xc.device)
    L.call('cmhar_dwconv2d_cl_fwd', L.F32, N, H, W, C, 3, s, 1, xc.data_ptr(), wc.data_ptr(), z.data_ptr(), st)
    assert rel(z.cpu().view(N, Ho, Wo, C).permute(0, 3, 1, 2), ref) < 1e-5
    dzc = dz.permute(0, 2, 3, 1).contiguous().to(DEV)
    dx = torch.empty_like(xc)
    L.call('cmhar_dwconv2d_cl_dgrad', L.F32, N, H, W, C, 3, s, 1, dzc.data_ptr(), wc.data_ptr(), dx.data_ptr(), st)
    assert rel(dx.cpu().permute(0, 3, 1, 2), x.grad) < 1e-5
    dw = torch.empty(C, 1, 3, 3, device=DEV)
    ws = K.workspace(L.lib().cmhar_dwconv2d_cl_wgrad_ws(N, H, W, C, 3, s, 1), xc.device)
    L.call('cmhar_dwconv2d_cl_wgrad', L.F32, N, H, W, C, 3, s, 1, xc.data_ptr(), dzc.data_ptr(), dw.data_ptr(),
           ws.data_ptr(), st)
    assert rel(dw, w.grad) < 1e-5


@pytest.mark.parametrize('C,s,HW', [(32, 1, (17, 19)), (144, 2, (28, 28)), (96, 2, (15, 9))])
def test_depthwise_conv_bf16_matches_fp32(C, s, HW):
    """bf16 depthwise conv (the MobileNetV2 path: all K² tap loads through a buffer resource, the padding taps at an
    out-of-range offset that reads zero) vs the fp32 conv on the same bf16-rounded operands: forward and input
    gradient within bf16 output rounding (5e-3 rel), weight gradient (fp32 accumulation) within 1e-4."""
    from cmhar import _lib as L
    from cmhar import kernels as K
    torch.manual_seed(3)
    N = 3
    H, W = HW
    x = torch.randn(N, C, H, W).bfloat16().float().requires_grad_(True)
    w = (torch.randn(C, 1, 3, 3) * 0.3).requires_grad_(True)
    ref = F.conv2d(x, w, stride=s, padding=1, groups=C)
    dz = torch.randn_like(ref).bfloat16().float()
    ref.backward(dz)
    Ho, Wo = ref.shape[2:]
    xc = x.detach().permute(0, 2, 3, 1).contiguous().to(DEV).bfloat16()
    wc = w.detach().to(DEV)
    st = L.stream(xc.device)
    z = torch.empty(N * Ho * Wo, C, device=DEV, dtype=torch.bfloat16)
    L.call('cmhar_dwconv2d_cl_fwd', L.BF16, N, H, W, C, 3, s, 1, xc.data_ptr(), wc.data_ptr(), z.data_ptr(), st)
    assert rel(z.float().cpu().view(N, Ho, Wo, C).permute(0, 3, 1, 2), ref) < 5e-3
    dzc = dz.permute(0, 2, 3, 1).contiguous().to(DEV).bfloat16()
    dx = torch.empty_like(xc)
    L.call('cmhar_dwconv2d_cl_dgrad', L.BF16, N, H, W, C, 3, s, 1, dzc.data_ptr(), wc.data_ptr(), dx.data_ptr(), st)
    assert rel(dx.float().cpu().permute(0, 3, 1, 2), x.grad) < 5e-3
    dw = torch.empty(C, 1, 3, 3, device=DEV)
    ws = K.workspace(L.lib().cmhar_dwconv2d_cl_wgrad_ws(N, H, W, C, 3, s, 1), xc.device)
    L.call('cmhar_dwconv2d_cl_wgrad', L.BF16, N, H, W, C, 3, s, 1, xc.data_ptr(), dzc.data_ptr(), dw.data_ptr(),
           ws.data_ptr(), st)
    assert rel(dw, w.grad) < 1e-4


def test_depthwise_conv_past_2gib_matches_buffer_form():
    """Past 2^31 bytes of input the depthwise forward keeps its 64-bit-address form; on the first and last frames it
    equals, bit for bit, the buffer-resource form run on those frames alone (each frame is independent)."""
    from cmhar import _lib as L
    torch.manual_seed(5)
    N, H, W, C = 900, 112, 112, 96                      # 2.17 GB of bf16 input
    x = torch.randn(N, H, W, C, device=DEV, dtype=torch.bfloat16)
    assert x.numel() * 2 > (1 << 31)
    wc = torch.randn(C, 1, 3, 3, device=DEV) * 0.3
    st = L.stream(x.device)
    z = torch.empty(N * H * W, C, device=DEV, dtype=torch.bfloat16)
    L.call('cmhar_dwconv2d_cl_fwd', L.BF16, N, H, W, C, 3, 1, 1, x.data_ptr(), wc.data_ptr(), z.data_ptr(), st)
    per = H * W
    for f0, f1 in ((0, 2), (N - 1, N)):
        xs = x[f0:f1].contiguous()
        zs = torch.empty((f1 - f0) * per, C, device=DEV, dtype=torch.bfloat16)
        L.call('cmhar_dwconv2d_cl_fwd', L.BF16, f1 - f0, H, W, C, 3, 1, 1, xs.data_ptr(), wc.data_ptr(), zs.data_ptr(),
               st)
        assert torch.equal(z[f0 * per:f1 * per], zs)
    torch.cuda.synchronize()


@pytest.mark.parametrize('C,act,res', [(96, 2, True), (144, 2, False), (1280, 2, False), (24, 0, True), (320, 1, False)])
def test_bn_channels_last_any_width_relu6(C, act, res):
    from cmhar import _lib as L
    from cmhar import kernels as K
    from cmhar import r3d
    torch.manual_seed(2)
    M = 2999
    x = (torch.randn(M, C) * 3 + 1.5).to(DEV)
    r = torch.randn(M, C, device=DEV) * 4 if res else None
    bn = torch.nn.BatchNorm2d(C).to(DEV)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 3.0)
        bn.bias.uniform_(-0.5, 3.0)
    y, sm, sr = r3d._bn_fwd(x, bn, r, act, True)
    xr = x.clone().requires_grad_(True)
    w = bn.weight.detach().clone().requires_grad_(True)
    b = bn.bias.detach().clone().requires_grad_(True)
    ref = F.batch_norm(xr, None, None, w, b, training=True, eps=1e-5)
    if res:
        ref = ref + r
    ref = F.relu6(ref) if act == 2 else (F.relu(ref) if act == 1 else ref)
    assert rel(y, ref) < 1e-5
    assert rel(bn.running_var, 0.9 + 0.1 * x.var(0, unbiased=True)) < 1e-5
    dy = torch.randn(M, C, device=DEV)
    ref.backward(dy)
    dx = torch.empty_like(x)
    dw = torch.empty(C, device=DEV)
    db = torch.empty(C, device=DEV)
    ws = K.workspace(L.lib().cmhar_bn_cl_ws(M, C), x.device)
    L.call('cmhar_bn_cl_bwd', L.F32, M, C, x.data_ptr(), y.data_ptr(), dy.data_ptr(), bn.weight.data_ptr(),
           sm.data_ptr(), sr.data_ptr(), dx.data_ptr(), None, dw.data_ptr(), db.data_ptr(), 1, act, ws.data_ptr(),
           L.stream(x.device))
    assert rel(dx, xr.grad) < 1e-5
    assert rel(dw, w.grad) < 1e-5 and rel(db, b.grad) < 1e-5
    # channel mean of the pool kernel at these widths
    from cmhar import _lib as Lb
    out = torch.empty(3, C, device=DEV)
    xs = x[:3 * 999].contiguous()
    Lb.call('cmhar_avgpool_cl', Lb.F32, 3, 999, C, xs.data_ptr(), out.data_ptr(), Lb.stream(x.device))
    assert rel(out, xs.view(3, 999, C).mean(1)) < 1e-6


def _case(backbone, dtype, training=True, B=2, T=2, S=64, emulate=False, fp64=False):
    from cmhar.cnn2d import MobileNetV2Features, ResNet18Features, run_cnn2d
    from oracle import cnn2d_cpu as O
    from oracle.r3d_cpu import bf16_storage, bf16_weight
    torch.manual_seed(3)
    m = (ResNet18Features if backbone == 'resnet18' else MobileNetV2Features)(compute_dtype=dtype)
    with torch.no_grad():
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm2d):
                mod.weight.uniform_(0.5, 1.5)
                mod.bias.uniform_(-0.2, 0.2)
                mod.running_mean.uniform_(-0.1, 0.1)
                mod.running_var.uniform_(0.5, 1.5)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    video = torch.randn(B, T, 3, S, S)
    R = torch.randn(B * T, m.feature_dim)
    f = O.resnet18_features if backbone == 'resnet18' else O.mobilenet_v2_features

    def oracle(q, dt=torch.float32, qw=None):
        sd_p = {k: (v.clone().to(dt).requires_grad_(True) if v.is_floating_point() and 'running' not in k
                    else (v.clone().to(dt) if v.is_floating_point() else v.clone())) for k, v in sd.items()}
        stats = {}
        ref = f(sd_p, video.reshape(B * T, 3, S, S).to(dt), training, stats, q, qw).mean(dim=(2, 3))
        (ref * R.to(dt)).sum().backward()
        return sd_p, stats, ref

    sd_p, stats, ref = oracle(None)
    m = m.to(DEV).train(training)
    feat = run_cnn2d(m, video.to(DEV), training)
    (feat * R.to(DEV)).sum().backward()
    out = [m, sd_p, stats, ref, feat]
    if emulate:
        out.append(oracle(bf16_storage, qw=bf16_weight))
    if fp64:
        out.append(oracle(None, torch.float64))
    return tuple(out)


@pytest.mark.parametrize('backbone,S', [('resnet18', 64), ('mobilenet_v2', 128)])
def test_backbone_fp32_matches_oracle(backbone, S):
    """fp32 path vs the oracle.  Training-mode BatchNorm after BatchNorm makes some gradients ill-conditioned (in
    MobileNetV2 the projection BNs' biases are exactly shift-invariant — their true gradient is 0 — and the CPU fp32
    oracle itself is 2e-3..7e-3 off its fp64 run on the stem / early BNs, even though torch's CPU BatchNorm accumulates
    its statistics in double while the HIP kernels accumulate in fp32), so each gradient is checked against the fp64
    oracle with the bound max(5e-3, 16·rel(cpu fp32, cpu fp64)); mathematically-zero gradients must be ≈ 0.  The
    well-conditioned eval-mode gradients are held to 2e-3 (test_backbone_eval_running_stats_and_grads)."""
    m, sd_p, stats, ref, feat, (sd64, _, ref64) = _case(backbone, 'fp32', S=S, fp64=True)
    assert rel(feat, ref) < 1e-4
    gscale = max(sd64[k].grad.abs().max().item() for k, _ in m.named_parameters())
    worst = []
    for k, p in m.named_parameters():
        assert p.grad is not None, k
        g64 = sd64[k].grad
        if g64.abs().max().item() < 1e-6 * gscale:                   # mathematically zero (shift invariance)
            assert p.grad.abs().max().item() < 1e-4 * gscale, k
            continue
        cond = rel(sd_p[k].grad, g64)
        err = rel(p.grad, g64)
        worst.append((err, cond, k))
        assert err < max(5e-3, 16 * cond), (k, err, cond)
    print(backbone, 'worst (gpu vs fp64, cpu fp32 vs fp64, param):', sorted(worst, reverse=True)[:3])
    bufs = dict(m.named_buffers())
    for pre, (rm, rv) in stats.items():
        assert rel(bufs[pre + 'running_mean'], rm) < 1e-5, pre
        assert rel(bufs[pre + 'running_var'], rv) < 1e-5, pre
        assert int(bufs[pre + 'num_batches_tracked']) == 1


@pytest.mark.parametrize('backbone', ['resnet18', 'mobilenet_v2'])
def test_backbone_bf16_error_is_bf16_storage(backbone):
    """bf16 path vs the fp32 oracle, bounded per parameter by the error bf16 storage alone causes (the oracle re-run
    with bf16 rounding at the HIP path's storage points; see tests/test_r3d_gpu.py::bf16_storage_bound)."""
    from test_r3d_gpu import bf16_storage_bound
    m, sd_p, _, ref, feat, (sd_q, _, ref_q) = _case(backbone, 'bf16', B=2, T=2, S=128, emulate=True)
    e_feat = rel(ref_q, ref)
    assert rel(feat, ref) < 3 * e_feat + 2e-3, (rel(feat, ref), e_feat)
    grads = {k: p.grad for k, p in m.named_parameters()}
    rows = bf16_storage_bound(grads, {k: sd_p[k].grad for k in grads}, {k: sd_q[k].grad for k in grads})
    print(backbone, 'worst (gpu err, bf16-storage err, param):', rows[:4])


@pytest.mark.parametrize('backbone', ['resnet18', 'mobilenet_v2'])
def test_backbone_eval_running_stats_and_grads(backbone):
    """Eval-mode BatchNorm (running statistics): forward ≤ 1e-4 and — the backward being well-conditioned without
    batch statistics — every parameter gradient ≤ 2e-3 rel, in fp32 (depthwise dgrad / wgrad, ReLU6 masks, residual
    routing, max-pool gather all on the path)."""
    m, sd_p, _, ref, feat = _case(backbone, 'fp32', training=False, S=96)
    assert rel(feat, ref) < 1e-4
    for k, p in m.named_parameters():
        assert rel(p.grad, sd_p[k].grad) < 2e-3, (k, rel(p.grad, sd_p[k].grad))
    bufs = dict(m.named_buffers())
    assert all(int(v) == 0 for k, v in bufs.items() if k.endswith('num_batches_tracked'))


@pytest.mark.parametrize('backbone', ['resnet18', 'mobilenet_v2'])
def test_video_encoder_and_crossmodal_step(backbone):
    """VideoEncoder (models.py:208-216: per-frame projection, temporal mean) vs the oracle, then one CrossModalModel
    training step through the CNN backbone."""
    from cmhar.config import Config
    from cmhar.losses import SigmoidContrastiveLoss
    from cmhar.models import CrossModalModel, VideoEncoder
    from oracle import cnn2d_cpu as O
    cfg = Config()
    cfg.model.video_backbone = backbone
    cfg.model.video_pretrained = False
    cfg.model.compute_dtype = 'fp32'
    cfg.data.video_frames_per_window = 3
    cfg.data.video_resize = (64, 64)
    torch.manual_seed(4)
    venc = VideoEncoder(cfg)
    assert venc.feature_dim == (512 if backbone == 'resnet18' else 1280) and not venc.is_videomae
    sd = {k: v.clone() for k, v in venc.state_dict().items()}
    video = torch.randn(2, 3, 3, 64, 64)
    with torch.no_grad():
        ref = O.video_encoder_cnn(sd, video, backbone, training=False)
        got = venc.to(DEV).eval()(video.to(DEV))
    assert rel(got, ref) < 1e-4
    cfg.model.compute_dtype = 'bf16'
    model = CrossModalModel(cfg).to(DEV).train()
    a, b = model(torch.randn(4, 6, 200, device=DEV), torch.randn(4, 3, 3, 64, 64, device=DEV))
    loss = SigmoidContrastiveLoss().to(DEV)(a, b)
    loss.backward()
    assert torch.isfinite(loss)
    for k, p in model.named_parameters():
        if k.startswith('video_encoder.'):
            assert p.grad is not None and torch.isfinite(p.grad).all(), k


@pytest.mark.parametrize('co,ci,k', [(64, 3, (3, 7, 7)), (512, 256, (3, 3, 3)), (96, 144, (1, 1, 1)), (40, 24, (1, 3, 3)),
                                     (64, 3, (1, 7, 7))])
@pytest.mark.parametrize('dt', [torch.float32, torch.bfloat16])
def test_conv_pack_weight_both_forms(co, ci, k, dt):
    """cmhar_conv_pack_weight vs torch's permute / flip of the same master: bit-exact (a pure data movement)."""
    from cmhar import _lib as L
    from cmhar import r3d
    torch.manual_seed(6)
    w = torch.randn(co, ci, *k, device=DEV)
    taps = k[0] * k[1] * k[2]
    kp = r3d._r8(ci * taps)
    wp = torch.empty(co, kp, dtype=dt, device=DEV)
    wf = torch.empty(ci, taps * co, dtype=dt, device=DEV)
    L.call('cmhar_conv_pack_weight', L.dtype_code(dt), co, ci, *k, kp, w.data_ptr(), wp.data_ptr(), wf.data_ptr(),
           L.stream(w.device))
    ref = torch.zeros(co, kp, device=DEV)
    ref[:, :ci * taps] = w.permute(0, 2, 3, 4, 1).reshape(co, -1)
    assert torch.equal(wp, ref.to(dt))
    reff = w.flip(2, 3, 4).permute(1, 2, 3, 4, 0).reshape(ci, -1)
    assert torch.equal(wf, reff.to(dt))


@pytest.mark.parametrize('dt', [torch.float32, torch.bfloat16])
def test_conv_pack_weights_multi_launch(dt):
    """cmhar_conv_pack_weights: 30 packs (more than one launch's 24 jobs) of mixed geometry — vector and scalar forms,
    with and without the flipped copy, the out-only form — equal to torch's permute / flip bit for bit."""
    import ctypes
    from cmhar import _lib as L
    from cmhar import r3d
    torch.manual_seed(7)
    geo = [(64, 3, (3, 7, 7)), (512, 256, (3, 3, 3)), (96, 144, (1, 1, 1)), (40, 24, (1, 3, 3)), (64, 64, (3, 3, 3)),
           (128, 64, (1, 1, 1))]
    jobs = [(geo[i % len(geo)], i % 3 != 0) for i in range(30)]
    dims = (ctypes.c_int * (6 * len(jobs)))()
    ptrs = (ctypes.c_void_p * (3 * len(jobs)))()
    bufs = []
    for i, ((co, ci, k), flip) in enumerate(jobs):
        w = torch.randn(co, ci, *k, device=DEV)
        taps = k[0] * k[1] * k[2]
        kp = r3d._r8(ci * taps)
        wp = torch.full((co, kp), 7.0, dtype=dt, device=DEV)
        wf = torch.empty(ci, taps * co, dtype=dt, device=DEV) if flip else None
        dims[6 * i:6 * i + 6] = [co, ci, *k, kp]
        ptrs[3 * i:3 * i + 3] = [w.data_ptr(), wp.data_ptr(), None if wf is None else wf.data_ptr()]
        bufs.append((w, wp, wf, ci, taps))
    L.call('cmhar_conv_pack_weights', L.dtype_code(dt), len(jobs), dims, ptrs, L.stream(torch.device(DEV)))
    torch.cuda.synchronize()
    for w, wp, wf, ci, taps in bufs:
        ref = torch.zeros(wp.shape, device=DEV)
        ref[:, :ci * taps] = w.permute(0, 2, 3, 4, 1).reshape(w.shape[0], -1)
        assert torch.equal(wp, ref.to(dt))
        if wf is not None:
            assert torch.equal(wf, w.flip(2, 3, 4).permute(1, 2, 3, 4, 0).reshape(ci, -1).to(dt))
