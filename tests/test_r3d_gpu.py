"""R3D-18 video backbone (north_star extension; parity unpinned w.r.t. the reference, which has no 3-D CNN) against
the CPU restatement oracle/r3d_cpu.py (F.conv3d / F.batch_norm) on identical weights and inputs.

Kernel level (fp32, exact-fp32 GEMM): conv3d = im2col + GEMM vs F.conv3d (≤ 1e-5 rel) for the scalar (C = 3) and
vectorised (C % 8 == 0) paths with stride/padding; col2im is the adjoint of im2col (<im2col x, c> = <x, col2im c>);
channels-last BatchNorm3d (+ residual + ReLU) forward / backward vs torch autograd (≤ 1e-5).
Backbone: fp32 mode features ≤ 1e-4 rel, running stats ≤ 1e-5, every parameter gradient ≤ 2e-3 rel; bf16 mode
(throughput): every parameter gradient within 3× (+2e-3) of the error bf16 storage alone causes for that parameter
(the fp32 oracle re-run with bf16 rounding at the HIP path's storage points — `bf16_storage_bound` documents why the
stem / early-BN gradients are the ill-conditioned ones); eval mode (running statistics) ≤ 1e-4 rel.  The stem
weight gradient's ~1024-way split-K at production row counts ≤ 1e-4 vs the fp32 product of the same operands."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def rel(a, b):
    a, b = torch.as_tensor(a).detach().double().cpu(), torch.as_tensor(b).detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize('cin,cout,k,s,p', [(3, 64, (3, 7, 7), (1, 2, 2), (1, 3, 3)), (16, 32, (3, 3, 3), (2, 2, 2), (1, 1, 1)),
                                            (16, 64, (1, 1, 1), (2, 2, 2), (0, 0, 0))])
def test_conv3d_im2col_gemm_matches_conv3d(cin, cout, k, s, p):
    from cmhar import r3d
    torch.manual_seed(0)
    conv = torch.nn.Conv3d(cin, cout, k, s, p, bias=False)
    x = torch.randn(2, cin, 5, 13, 11)
    ref = F.conv3d(x, conv.weight, stride=s, padding=p)
    conv = conv.to(DEV)
    xc = x.permute(0, 2, 3, 4, 1).contiguous().to(DEV)
    shape = tuple(xc.shape)
    Kp = r3d._r8(conv.weight[0].numel())
    col = r3d._im2col(xc, shape, conv, Kp, math.prod(r3d._out_shape(shape, conv)[:4]))
    wp = r3d._pack(conv, torch.float32)
    z = torch.empty(col.shape[0], cout, device=DEV)
    from cmhar import kernels as K
    K.gemm(0, col, wp, z)
    osh = r3d._out_shape(shape, conv)
    got = z.reshape(osh).permute(0, 4, 1, 2, 3).cpu()
    assert got.shape == ref.shape
    assert rel(got, ref) < 1e-5
    # col2im is the adjoint of im2col
    from cmhar import _lib as L
    c = torch.randn_like(col)
    dx = torch.empty_like(xc)
    L.call('cmhar_conv3d_col2im', L.F32, r3d._dims(shape, conv, Kp), c.data_ptr(), dx.data_ptr(), 0,
           L.stream(dx.device))
    lhs = (col.double() * c.double()).sum().item()
    rhs = (xc.double() * dx.double()).sum().item()
    assert abs(lhs - rhs) <= 1e-5 * (abs(lhs) + 1.0)


@pytest.mark.parametrize('C,relu,res', [(64, True, True), (512, False, False), (128, True, False)])
def test_bn_channels_last_fwd_bwd(C, relu, res):
    from cmhar import r3d
    torch.manual_seed(1)
    M = 3001
    x = (torch.randn(M, C) * 3 + 1.5).to(DEV)
    r = torch.randn(M, C, device=DEV) if res else None
    bn = torch.nn.BatchNorm3d(C).to(DEV)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    y, sm, sr = r3d._bn_fwd(x, bn, r, relu, True)
    xr = x.clone().requires_grad_(True)
    rr = r.clone().requires_grad_(True) if res else None
    w = bn.weight.detach().clone().requires_grad_(True)
    b = bn.bias.detach().clone().requires_grad_(True)
    ref = F.batch_norm(xr, None, None, w, b, training=True, eps=1e-5)
    if res:
        ref = ref + rr
    if relu:
        ref = F.relu(ref)
    assert rel(y, ref) < 1e-5
    assert rel(bn.running_mean, 0.1 * x.mean(0)) < 1e-5
    assert rel(bn.running_var, 0.9 + 0.1 * x.var(0, unbiased=True)) < 1e-5
    assert int(bn.num_batches_tracked) == 1
    dy = torch.randn(M, C, device=DEV)
    ref.backward(dy)
    from cmhar import _lib as L
    dx = torch.empty_like(x)
    dres = torch.empty_like(x) if res else None
    dw = torch.empty(C, device=DEV)
    db = torch.empty(C, device=DEV)
    from cmhar import kernels as K
    ws = K.workspace(L.lib().cmhar_bn_cl_ws(M, C), x.device)
    L.call('cmhar_bn_cl_bwd', L.F32, M, C, x.data_ptr(), y.data_ptr(), dy.data_ptr(), bn.weight.data_ptr(),
           sm.data_ptr(), sr.data_ptr(), dx.data_ptr(), None if dres is None else dres.data_ptr(), dw.data_ptr(),
           db.data_ptr(), 1, int(relu), ws.data_ptr(), L.stream(x.device))
    assert rel(dx, xr.grad) < 1e-5
    assert rel(dw, w.grad) < 1e-5
    assert rel(db, b.grad) < 1e-5
    if res:
        assert rel(dres, rr.grad) < 1e-6


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('C,relu', [(64, 1), (96, 2), (192, 1), (512, 1)])
@pytest.mark.parametrize('training', [1, 0])
def test_bn_bwd_nores_matches_y_mask(dtype, C, relu, training):
    """cmhar_bn_cl_bwd_nores recomputes the activation mask from z in bn_cl_apply's arithmetic: dx / dw / db must
    equal cmhar_bn_cl_bwd's (which reads the stored y) bit for bit.  C = 96 / 192: C/8 does not divide 256 (the
    per-vector constant loads); 64 / 512 the hoisted ones.  z is offset so that many pre-activations sit near 0."""
    from cmhar import _lib as L
    from cmhar import kernels as K
    from cmhar import r3d
    torch.manual_seed(3)
    M = 4099
    z = (torch.randn(M, C) * 2 + 0.3).to(DEV).to(dtype)
    bn = torch.nn.BatchNorm3d(C).to(DEV)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 3.5)
        bn.bias.uniform_(-0.5, 3.0)
        bn.running_mean.uniform_(-0.2, 0.2)
        bn.running_var.uniform_(0.5, 1.5)
    y, sm, sr = r3d._bn_fwd(z, bn, None, relu, bool(training))
    frac_off = float(((y.float() <= 0) | (y.float() >= 6)).float().mean()) if relu == 2 else float((y <= 0).float().mean())
    assert 0.05 < frac_off < 0.95
    dy = torch.randn(M, C, device=DEV).to(dtype)
    ws = K.workspace(L.lib().cmhar_bn_cl_ws(M, C), z.device)
    outs = []
    for nores in (False, True):
        dx = torch.empty_like(z)
        dw = torch.empty(C, device=DEV)
        db = torch.empty(C, device=DEV)
        if nores:
            L.call('cmhar_bn_cl_bwd_nores', L.dtype_code(dtype), M, C, z.data_ptr(), dy.data_ptr(),
                   bn.weight.data_ptr(), bn.bias.data_ptr(), sm.data_ptr(), sr.data_ptr(), dx.data_ptr(),
                   dw.data_ptr(), db.data_ptr(), training, relu, ws.data_ptr(), L.stream(z.device))
        else:
            L.call('cmhar_bn_cl_bwd', L.dtype_code(dtype), M, C, z.data_ptr(), y.data_ptr(), dy.data_ptr(),
                   bn.weight.data_ptr(), sm.data_ptr(), sr.data_ptr(), dx.data_ptr(), None, dw.data_ptr(),
                   db.data_ptr(), training, relu, ws.data_ptr(), L.stream(z.device))
        torch.cuda.synchronize()
        outs.append((dx, dw, db))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def _backbone_case(dtype, training=True, B=2, T=4, S=32, emulate=False):
    from cmhar.r3d import R3D18, run_r3d
    from oracle.r3d_cpu import BF16, r3d18_features
    torch.manual_seed(2)
    m = R3D18(None, compute_dtype=dtype)
    with torch.no_grad():     # non-trivial BN affine parameters / running stats
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm3d):
                mod.weight.uniform_(0.5, 1.5)
                mod.bias.uniform_(-0.2, 0.2)
                mod.running_mean.uniform_(-0.1, 0.1)
                mod.running_var.uniform_(0.5, 1.5)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    video = torch.randn(B, T, 3, S, S)      # (B, T, C, H, W)
    R = torch.randn(B, 512)

    def oracle(hooks):
        sd_p = {k: (v.clone().requires_grad_(True) if v.is_floating_point() and 'running' not in k else v.clone())
                for k, v in sd.items()}
        stats = {}
        ref = r3d18_features(sd_p, video.transpose(1, 2), training=training, stats=stats, **(hooks or {}))
        (ref * R).sum().backward()
        return sd_p, stats, ref

    sd_p, stats, ref = oracle(None)
    m = m.to(DEV).train(training)
    feat = run_r3d(m, video.to(DEV), training)
    (feat * R.to(DEV)).sum().backward()
    if emulate:
        return m, sd_p, stats, ref, feat, oracle(BF16)
    return m, sd_p, stats, ref, feat


def test_r3d18_fp32_matches_oracle():
    m, sd_p, stats, ref, feat = _backbone_case('fp32')
    assert rel(feat, ref) < 1e-4
    names = dict(m.named_parameters())
    for k, p in names.items():
        assert p.grad is not None, k
        assert rel(p.grad, sd_p[k].grad) < 2e-3, (k, rel(p.grad, sd_p[k].grad))
    bufs = dict(m.named_buffers())
    for pre, (rm, rv) in stats.items():
        assert rel(bufs[pre + 'running_mean'], rm) < 1e-5, pre
        assert rel(bufs[pre + 'running_var'], rv) < 1e-5, pre
        assert int(bufs[pre + 'num_batches_tracked']) == 1


def bf16_storage_bound(gpu_grads, fp32_grads, emul_grads, slack=3.0, floor=2e-3):
    """Per-parameter check of a bf16-storage path against the fp32 oracle, with the bound set by the error that bf16
    STORAGE ITSELF causes for that parameter: the fp32 restatement run with bf16 rounding at the HIP path's storage
    points (oracle q = bf16_storage) shows e_p = rel(emulated, fp32).  Root cause of the large stem / early-BN errors
    (r01's 0.35): the next training-mode BatchNorm's backward removes each channel's mean gradient, so the gradients of
    the layers before it are small residuals of large cancelling sums, and the 2^-9 relative rounding of the stored
    dz / dx does not cancel — e_p is large exactly for those parameters and ~1e-2 elsewhere.  A kernel error shows as
    rel(gpu, fp32) >> e_p on a well-conditioned parameter."""
    rows = []
    for k in fp32_grads:
        e_p = rel(emul_grads[k], fp32_grads[k])
        e_g = rel(gpu_grads[k], fp32_grads[k])
        rows.append((e_g, e_p, k))
        assert e_g <= slack * e_p + floor, (k, e_g, e_p)
    return sorted(rows, reverse=True)


def test_r3d18_bf16_error_is_bf16_storage():
    m, sd_p, _, ref, feat, (sd_q, _, ref_q) = _backbone_case('bf16', B=4, T=4, S=48, emulate=True)
    e_feat = rel(ref_q, ref)
    assert rel(feat, ref) < 3 * e_feat + 2e-3, (rel(feat, ref), e_feat)
    grads = {k: p.grad for k, p in m.named_parameters()}
    rows = bf16_storage_bound(grads, {k: sd_p[k].grad for k in grads}, {k: sd_q[k].grad for k in grads})
    print('worst (gpu err, bf16-storage err, param):', rows[:4])


def test_r3d_stem_weight_gradient_split_k_production_rows():
    """the stem weight gradient (C = 3, Kp = 448 → 64 × 448 over ~1.6 M rows) at the production clip
    geometry, i.e. the ~1024-way split-K of r3d.py's stem path (K.gemm layout 2 with `splits`), against the fp32
    product of the same bf16 operands (torch matmul on the device): ≤ 1e-4 rel."""
    from cmhar import kernels as K
    from cmhar import r3d
    torch.manual_seed(7)
    rows = 32 * 16 * 56 * 56                                  # B = 32 clips, 16 × 112² → 16 × 56² outputs
    Kp, Cc = 448, 64
    col = torch.randn(rows, Kp, device=DEV).bfloat16()
    dz = torch.randn(rows, Cc, device=DEV).bfloat16()
    tiles = -(-Cc // 128) * -(-Kp // 128)
    splits = max(1, min(1024 // tiles, rows // 4096))
    assert splits >= 256
    dw = torch.empty(Cc, Kp, device=DEV)
    K.gemm(2, dz, col, dw, splits=splits)
    ref = dz.float().T @ col.float()
    assert rel(dw, ref) < 1e-4
    assert r3d._r8(3 * 3 * 7 * 7) == Kp                      # the stem's padded K


def test_r3d_implicit_stem_production_geometry():
    """The implicit stem kernels at the bench geometry (32 clips of 16 × 112² → 7168 row tiles, ~171-way split weight
    gradient) against fp32 products of the same bf16 operands on the device: the column matrix is built by
    cmhar_conv3d_im2col (itself checked against F.conv3d above), z_ref = col · Wᵀ (≤ 5e-3 rel, bf16 output) and
    dW_ref = dzᵀ · col (≤ 1e-4 rel, fp32 output), plus the epilogue BatchNorm statistics vs the two-pass kernel."""
    from cmhar import _lib as L
    from cmhar import kernels as K
    from cmhar import r3d
    torch.manual_seed(8)
    conv = torch.nn.Conv3d(3, 64, (3, 7, 7), (1, 2, 2), (1, 3, 3), bias=False).to(DEV)
    x = torch.randn(32, 16, 112, 112, 3, device=DEV).bfloat16()
    shp = tuple(x.shape)
    assert r3d._stem_ok(x, shp, conv)
    osh = r3d._out_shape(shp, conv)
    M = math.prod(osh[:4])
    Kp = r3d._r8(conv.weight[0].numel())
    col = r3d._im2col(x, shp, conv, Kp, M)                           # [M, 448] bf16, k = ((it·7 + ih)·7 + iw)·3 + c
    wq = conv.weight.detach().bfloat16().float()                      # the bf16 operand the kernel multiplies
    wk = wq.permute(0, 2, 3, 4, 1).reshape(64, -1)                    # im2col k order
    w4 = r3d._pack_stem(conv)
    dims = r3d._dims(shp, conv, r3d._stem_kp(conv))
    ntile = L.lib().cmhar_conv3d_stem_tiles(dims, 64)
    assert ntile == 32 * 16 * 14
    ts = torch.empty(L.lib().cmhar_conv3d_stem_stats_floats(dims, 64), device=DEV)
    z = torch.empty(M, 64, dtype=torch.bfloat16, device=DEV)
    L.call('cmhar_conv3d_stem_fwd', dims, 64, x.data_ptr(), w4.data_ptr(), z.data_ptr(), ts.data_ptr(),
           L.stream(x.device))
    z_ref = col[:, :wk.shape[1]].float() @ wk.T
    assert rel(z.float(), z_ref) < 5e-3
    bn_a, bn_b = torch.nn.BatchNorm3d(64).to(DEV), torch.nn.BatchNorm3d(64).to(DEV)
    _, sma, sra = r3d._bn_fwd(z, bn_a, None, True, True)
    _, smb, srb = r3d._bn_fwd_tiles(z, bn_b, None, True, ts, ntile)
    assert rel(smb, sma) < 1e-5 and rel(srb, sra) < 1e-5
    dz = torch.randn(M, 64, device=DEV).bfloat16()
    dw4 = torch.empty(64, r3d._stem_kp(conv), device=DEV)
    ws = K.workspace(L.lib().cmhar_conv3d_stem_wgrad_ws(dims, 64), x.device)
    L.call('cmhar_conv3d_stem_wgrad', dims, 64, x.data_ptr(), dz.data_ptr(), dw4.data_ptr(), ws.data_ptr(),
           L.stream(x.device))
    dw = dw4.view(64, 3, 7, 8, 4)[:, :, :, :7, :3].reshape(64, -1)
    dw_ref = dz.float().T @ col[:, :wk.shape[1]].float()
    assert rel(dw, dw_ref) < 1e-4


def test_r3d18_eval_running_stats():
    from cmhar.r3d import run_r3d
    from oracle.r3d_cpu import r3d18_features
    m, sd_p, _, _, _ = _backbone_case('fp32', training=False)
    video = torch.randn(2, 4, 3, 32, 32)
    with torch.no_grad():
        ref = r3d18_features({k: v.detach() for k, v in sd_p.items()}, video.transpose(1, 2), training=False)
        got = run_r3d(m.eval(), video.to(DEV), False)
    assert rel(got, ref) < 1e-4


def test_crossmodal_with_r3d_backbone_steps():
    from cmhar.config import Config
    from cmhar.losses import SigmoidContrastiveLoss
    from cmhar.models import CrossModalModel
    cfg = Config()
    cfg.model.video_backbone = 'r3d_18'
    cfg.data.video_frames_per_window = 4
    cfg.data.video_resize = (32, 32)
    torch.manual_seed(3)
    model = CrossModalModel(cfg).to(DEV).train()
    assert model.video_encoder.feature_dim == 512 and not model.video_encoder.is_videomae
    a, b = model(torch.randn(4, 6, 200, device=DEV), torch.randn(4, 4, 3, 32, 32, device=DEV))
    loss = SigmoidContrastiveLoss().to(DEV)(a, b)
    loss.backward()
    assert torch.isfinite(loss)
    for k, p in model.named_parameters():
        if k.startswith('video_encoder.backbone.'):
            assert p.grad is not None and torch.isfinite(p.grad).all(), k


@pytest.mark.parametrize('cin,cout,k,s,p,shape', [(64, 64, 3, 1, 1, (3, 5, 9, 7)), (64, 128, 3, 2, 1, (2, 6, 11, 10)),
                                                  (64, 64, 3, 1, 1, (2, 12, 40, 38)),
                                                  (128, 256, 1, 2, 0, (2, 4, 7, 9)), (192, 72, 3, 1, 1, (1, 3, 6, 5)),
                                                  (128, 128, 3, 1, 1, (2, 4, 28, 28)), (64, 64, 3, 1, 1, (1, 4, 10, 56)),
                                                  (256, 512, 3, 2, 1, (1, 4, 14, 14)), (256, 256, 3, 1, 1, (1, 3, 14, 14)),
                                                  (128, 192, 3, 1, 1, (1, 2, 30, 30))])
def test_conv3d_implicit_gemm_fwd_wgrad(cin, cout, k, s, p, shape):
    """Implicit-GEMM forward / weight gradient (bf16 operands, fp32 MFMA accumulation) vs F.conv3d in fp32 on the
    same bf16-rounded operands: forward ≤ 5e-3 rel (bf16 output rounding), wgrad ≤ 1e-4 rel (fp32 output).  The
    k = 3 cases with Cout % 64 == 0 take the row-slab weight gradient (conv3d_wgrad_rows: whole output rows per chunk
    — Wo = 7 / 38 / 56 / 28 give 9 / 1 / 1 / 2 rows per chunk, stride 2 slabs of 2·Wo + 1 positions, Cout tiles of
    64 and 128, one and two 64-channel slices); the stride-1 3x3x3 cases whose frames fill >= 3/4 of a 256-slot tile
    take the nine-tap forward (conv3d_fwd_rows3) on 64-wide Cout slices — 28², 14² (one 14-row tile of 4 slices),
    30² (Ho = 30 over 4 tiles of 8, 8, 8, 6 rows, 3 slices); 1x1x1 and Cout = 72 the generic gather kernel."""
    from cmhar import _lib as L
    from cmhar import kernels as K
    from cmhar import r3d
    torch.manual_seed(4)
    N, T, H, W = shape
    conv = torch.nn.Conv3d(cin, cout, k, s, p, bias=False)
    x = torch.randn(N, cin, T, H, W).bfloat16().float().requires_grad_(True)
    wq = conv.weight.detach().bfloat16().float().requires_grad_(True)
    ref = F.conv3d(x, wq, stride=s, padding=p)
    dz = torch.randn_like(ref).bfloat16().float()
    ref.backward(dz)
    conv = conv.to(DEV)
    xc = x.detach().permute(0, 2, 3, 4, 1).contiguous().to(DEV).bfloat16()
    shp = tuple(xc.shape)
    Kp = r3d._r8(conv.weight[0].numel())
    assert r3d._igemm_ok(xc, shp, conv, Kp)
    wp = r3d._pack(conv, torch.bfloat16)
    osh = r3d._out_shape(shp, conv)
    M = math.prod(osh[:4])
    z = torch.empty(M, cout, dtype=torch.bfloat16, device=DEV)
    dims = r3d._dims(shp, conv, Kp)
    ntm = L.lib().cmhar_conv3d_fwd_tiles(dims, cout)
    ts = torch.empty(L.lib().cmhar_conv3d_fwd_stats_floats(dims, cout), device=DEV)
    L.call('cmhar_conv3d_fwd', dims, cout, xc.data_ptr(), wp.data_ptr(), None, z.data_ptr(), ts.data_ptr(),
           L.stream(xc.device))
    got = z.float().reshape(osh).permute(0, 4, 1, 2, 3).cpu()
    assert rel(got, ref) < 5e-3
    # epilogue BatchNorm statistics (per-tile mean / M2 combined by cmhar_bn_cl_fwd_tiles) vs the two-pass kernel
    bn_a, bn_b = torch.nn.BatchNorm3d(cout).to(DEV), torch.nn.BatchNorm3d(cout).to(DEV)
    if cout % 8 == 0 and 256 % (cout // 8) == 0:
        ya, sma, sra = r3d._bn_fwd(z, bn_a, None, True, True)
        yb, smb, srb = r3d._bn_fwd_tiles(z, bn_b, None, True, ts, ntm)
        assert rel(smb, sma) < 1e-5 and rel(srb, sra) < 1e-5
        assert rel(bn_b.running_var, bn_a.running_var) < 1e-5 and int(bn_b.num_batches_tracked) == 1
        assert rel(yb.float(), ya.float()) < 1e-2
    dzc = dz.permute(0, 2, 3, 4, 1).reshape(M, cout).contiguous().to(DEV).bfloat16()
    dwp = torch.empty(cout, Kp, device=DEV)
    n = L.lib().cmhar_conv3d_wgrad_ws(dims, cout)
    ws = K.workspace(n, xc.device) if n > 0 else None
    L.call('cmhar_conv3d_wgrad', dims, cout, xc.data_ptr(), dzc.data_ptr(), dwp.data_ptr(),
           None if ws is None else ws.data_ptr(), L.stream(xc.device))
    kk = conv.weight[0].numel()
    dw = dwp[:, :kk].reshape(cout, *conv.kernel_size, cin).permute(0, 4, 1, 2, 3).cpu()
    assert rel(dw, wq.grad) < 1e-4


@pytest.mark.parametrize('cin,k,s,p,shape', [(3, (3, 7, 7), (1, 2, 2), (1, 3, 3), (1, 4, 112, 112)),
                                             (3, (3, 7, 7), (1, 2, 2), (1, 3, 3), (2, 3, 30, 34)),
                                             (3, (1, 7, 7), (1, 2, 2), (0, 3, 3), (2, 2, 40, 36)),
                                             (2, (3, 5, 5), (2, 1, 2), (1, 2, 2), (1, 5, 20, 24)),
                                             (4, (2, 3, 8), (1, 2, 2), (0, 1, 3), (2, 3, 11, 120))])
def test_conv3d_implicit_stem_fwd_wgrad(cin, k, s, p, shape):
    """Implicit stem (cmhar_conv3d_stem_*: C <= 4, kw <= 8 at w-stride 2, Cout = 64 — R3D-18's 3x7x7 (1,2,2) stem at
    the production 112² frame, ragged row tiles, ResNet-18's 7x7/2 stem as (1,7,7), h-stride 1, kw = 8 at the widest
    staged row) vs F.conv3d in fp32 on the same bf16-rounded operands: forward ≤ 5e-3 rel (bf16 output), epilogue
    BatchNorm statistics ≤ 1e-5 vs the two-pass kernel, weight gradient ≤ 1e-4 rel (fp32 output)."""
    from cmhar import _lib as L
    from cmhar import kernels as K
    from cmhar import r3d
    torch.manual_seed(6)
    N, T, H, W = shape
    conv = torch.nn.Conv3d(cin, 64, k, s, p, bias=False)
    x = torch.randn(N, cin, T, H, W).bfloat16().float().requires_grad_(True)
    wq = conv.weight.detach().bfloat16().float().requires_grad_(True)
    ref = F.conv3d(x, wq, stride=s, padding=p)
    dz = torch.randn_like(ref).bfloat16().float()
    ref.backward(dz)
    conv = conv.to(DEV)
    xc = x.detach().permute(0, 2, 3, 4, 1).contiguous().to(DEV).bfloat16()
    shp = tuple(xc.shape)
    assert r3d._stem_ok(xc, shp, conv)
    w4 = r3d._pack_stem(conv)
    osh = r3d._out_shape(shp, conv)
    M = math.prod(osh[:4])
    dims = r3d._dims(shp, conv, r3d._stem_kp(conv))
    ntile = L.lib().cmhar_conv3d_stem_tiles(dims, 64)
    ts = torch.empty(L.lib().cmhar_conv3d_stem_stats_floats(dims, 64), device=DEV)
    z = torch.empty(M, 64, dtype=torch.bfloat16, device=DEV)
    L.call('cmhar_conv3d_stem_fwd', dims, 64, xc.data_ptr(), w4.data_ptr(), z.data_ptr(), ts.data_ptr(),
           L.stream(xc.device))
    got = z.float().reshape(osh).permute(0, 4, 1, 2, 3).cpu()
    assert rel(got, ref) < 5e-3
    bn_a, bn_b = torch.nn.BatchNorm3d(64).to(DEV), torch.nn.BatchNorm3d(64).to(DEV)
    ya, sma, sra = r3d._bn_fwd(z, bn_a, None, True, True)
    yb, smb, srb = r3d._bn_fwd_tiles(z, bn_b, None, True, ts, ntile)
    assert rel(smb, sma) < 1e-5 and rel(srb, sra) < 1e-5
    assert rel(yb.float(), ya.float()) < 1e-2
    dzc = dz.permute(0, 2, 3, 4, 1).reshape(M, 64).contiguous().to(DEV).bfloat16()
    dw4 = torch.empty(64, r3d._stem_kp(conv), device=DEV)
    ws = K.workspace(L.lib().cmhar_conv3d_stem_wgrad_ws(dims, 64), xc.device)
    L.call('cmhar_conv3d_stem_wgrad', dims, 64, xc.data_ptr(), dzc.data_ptr(), dw4.data_ptr(), ws.data_ptr(),
           L.stream(xc.device))
    kt, kh, kw = k
    dw = dw4.view(64, kt, kh, 8, 4)[:, :, :, :kw, :cin].permute(0, 4, 1, 2, 3).cpu()
    assert rel(dw, wq.grad) < 1e-4
    # the zero padding of the packed layout (iw >= kw, c >= C) carries no gradient into the parameter view
    assert torch.equal(w4.view(64, kt, kh, 8, 4)[:, :, :, kw:, :].float().cpu(),
                       torch.zeros(64, kt, kh, 8 - kw, 4))


@pytest.mark.parametrize('cin,cout,shape,acc', [(64, 64, (2, 4, 9, 7), True), (128, 192, (1, 3, 5, 6), False),
                                                (128, 128, (2, 3, 14, 28), True), (192, 256, (1, 2, 14, 14), True)])
def test_conv3d_implicit_gemm_dgrad(cin, cout, shape, acc):
    """Stride-1 input gradient as the flipped-weight implicit GEMM (+ the residual-branch gradient in its epilogue)
    vs torch autograd of F.conv3d on the same bf16-rounded operands: ≤ 5e-3 rel."""
    from cmhar import r3d
    torch.manual_seed(5)
    N, T, H, W = shape
    conv = torch.nn.Conv3d(cin, cout, 3, 1, 1, bias=False)
    conv.weight.data = conv.weight.data.bfloat16().float()
    x = torch.randn(N, cin, T, H, W).bfloat16().float().requires_grad_(True)
    ref = F.conv3d(x, conv.weight, padding=1)
    dz = torch.randn_like(ref).bfloat16().float()
    ref.backward(dz)
    res = torch.randn(N, T, H, W, cin).bfloat16() if acc else None
    expect = x.grad.permute(0, 2, 3, 4, 1) + (res.float() if acc else 0)
    conv = conv.to(DEV)
    assert r3d._dgrad_igemm_ok(conv)
    xc = x.detach().permute(0, 2, 3, 4, 1).reshape(-1, cin).contiguous().to(DEV).bfloat16()
    dzc = dz.permute(0, 2, 3, 4, 1).reshape(-1, cout).contiguous().to(DEV).bfloat16()
    dx = r3d._dgrad_igemm(dzc, conv, (N, T, H, W, cout), xc,
                          None if res is None else res.reshape(-1, cin).contiguous().to(DEV))
    assert rel(dx.float().reshape(N, T, H, W, cin), expect) < 5e-3


@pytest.mark.parametrize('relu', [1, 2])
def test_bn_bwd_nores_rounding_boundaries(relu):
    """The z-mask's thresholds at the bf16 rounding boundaries of y = bf16(act(v)): with mean 0, rstd 1 (eval, eps 0)
    and z = 1 the pre-activation v is the channel's weight, chosen at each boundary and one fp32 ulp inside it —
    ReLU6's tie at 6 − 2^-6 (rounds to the even 6.0), the denormal 2^-134 (rounds to +0), ReLU's overflow to +inf at 0x1.ffp127 (active: [y > 0], as torch)
    — plus ordinary values.  The no-residual entry must give the y-reading entry's dx / dw / db bit for bit (whatever
    rsqrt(1) rounds to, both entries use the same saved statistics)."""
    from cmhar import _lib as L
    from cmhar import kernels as K
    from cmhar import r3d
    import numpy as np
    below = lambda v: float(np.nextafter(np.float32(v), np.float32(0)))      # one fp32 ulp toward 0  # noqa: E731
    ws = [5.984375, below(5.984375), 2.0 ** -134, 1.5 * 2.0 ** -134, float.fromhex('0x1.ffp127'),
          below(float.fromhex('0x1.ffp127')), float.fromhex('0x1.fep127'), 2.0 ** -133, 6.0, 0.75, 3.0, 2.0 ** -126,
          1e-3, -2.0 ** -140, 5.96875, -1.0]
    C = len(ws)
    M = 257
    bn = torch.nn.BatchNorm3d(C, eps=0.0).to(DEV)
    with torch.no_grad():
        bn.weight.copy_(torch.tensor(ws, dtype=torch.float64).float())
        bn.bias.zero_()
        bn.running_mean.zero_()
        bn.running_var.fill_(1.0)
    z = torch.ones(M, C, device=DEV, dtype=torch.bfloat16)
    z[M // 2:] = torch.randn(M - M // 2, C, device=DEV).to(torch.bfloat16)
    y, sm, sr = r3d._bn_fwd(z, bn, None, relu, False)
    dy = torch.randn(M, C, device=DEV).to(torch.bfloat16)
    wsp = K.workspace(L.lib().cmhar_bn_cl_ws(M, C), z.device)
    outs = []
    for nores in (False, True):
        dx = torch.empty_like(z)
        dw = torch.empty(C, device=DEV)
        db = torch.empty(C, device=DEV)
        if nores:
            L.call('cmhar_bn_cl_bwd_nores', L.BF16, M, C, z.data_ptr(), dy.data_ptr(), bn.weight.data_ptr(),
                   bn.bias.data_ptr(), sm.data_ptr(), sr.data_ptr(), dx.data_ptr(), dw.data_ptr(), db.data_ptr(), 0,
                   relu, wsp.data_ptr(), L.stream(z.device))
        else:
            L.call('cmhar_bn_cl_bwd', L.BF16, M, C, z.data_ptr(), y.data_ptr(), dy.data_ptr(), bn.weight.data_ptr(),
                   sm.data_ptr(), sr.data_ptr(), dx.data_ptr(), None, dw.data_ptr(), db.data_ptr(), 0, relu,
                   wsp.data_ptr(), L.stream(z.device))
        torch.cuda.synchronize()
        outs.append((dx, dw, db))
    for a, b in zip(*outs):      # bitwise (±0 and inf included)
        ai = a.view(torch.int16) if a.dtype == torch.bfloat16 else a.view(torch.int32)
        bi = b.view(torch.int16) if b.dtype == torch.bfloat16 else b.view(torch.int32)
        bad = (ai != bi).nonzero()
        assert bad.numel() == 0, [(tuple(i), ws[int(i[-1])], float(y.view(-1, C)[int(i[0]), int(i[-1])])
                                   if a.dim() == 2 else None, float(a[tuple(i)]), float(b[tuple(i)]))
                                  for i in bad[:6].tolist()]


@pytest.mark.parametrize('res', [False, True])
@pytest.mark.parametrize('geom', ['r3d_layer4', 'resnet18_layer4_kt1', 'r3d_layer4_stride2'])
def test_conv3d_fwd_split_layer4(res, geom):
    """The split-K implicit-GEMM forward at R3D-18 layer 4's geometry (batch 32: 32×2×7×7 = 3136 output rows, 512 → 512,
    3×3×3 'same'; the row-slab kernel split over its K-steps), at a 2-D (kt = 1) ResNet-18 layer-4 conv run through the
    conv3d machinery (32 frames of 7×7, (1,3,3) taps — ADVICE r04), and at layer 4's stride-2 conv (256 → 512 from
    32×4×14×14: the generic gather kernel, 100 128×128 tiles, split over its 64-wide K-steps): planned
    (`cmhar_conv3d_fwd_split_ws` > 0), against the fp32 conv of the same bf16 operands (+ the residual, as the dgrad
    call adds dx_acc) within the bf16 output rounding, and within one bf16 ulp (of the value or of the output's rms near
    zero) of the unsplit kernel (`cmhar_conv3d_fwd`, the same products summed in a different order)."""
    from cmhar import _lib as L
    from cmhar import kernels as K
    from cmhar import r3d
    torch.manual_seed(9)
    if geom == 'r3d_layer4':
        N, Ci, C, T, S, k, st, pd = 32, 512, 512, 2, 7, (3, 3, 3), 1, (1, 1, 1)
    elif geom == 'resnet18_layer4_kt1':
        N, Ci, C, T, S, k, st, pd = 32, 512, 512, 1, 7, (1, 3, 3), 1, (0, 1, 1)
    else:
        N, Ci, C, T, S, k, st, pd = 32, 256, 512, 4, 14, (3, 3, 3), 2, (1, 1, 1)
    conv = torch.nn.Conv3d(Ci, C, k, st, pd, bias=False)
    x = torch.randn(N, Ci, T, S, S).bfloat16().float()
    wq = conv.weight.detach().bfloat16().float()
    ref = F.conv3d(x.to(DEV), wq.to(DEV), stride=st, padding=pd)
    conv = conv.to(DEV)
    xc = x.permute(0, 2, 3, 4, 1).contiguous().to(DEV).bfloat16()
    shp = tuple(xc.shape)
    Kp = r3d._r8(conv.weight[0].numel())
    wp = r3d._pack(conv, torch.bfloat16)
    M = ref.shape[0] * ref.shape[2] * ref.shape[3] * ref.shape[4]
    dims = r3d._dims(shp, conv, Kp)
    n = L.lib().cmhar_conv3d_fwd_split_ws(dims, C)
    assert n > 0 and n % (M * C) == 0
    rr = torch.randn(M, C, device=DEV).bfloat16() if res else None
    z = torch.empty(M, C, dtype=torch.bfloat16, device=DEV)
    ws = K.workspace(n, xc.device)
    L.call('cmhar_conv3d_fwd_split', dims, C, xc.data_ptr(), wp.data_ptr(), None if rr is None else rr.data_ptr(),
           z.data_ptr(), ws.data_ptr(), L.stream(xc.device))
    z1 = torch.empty_like(z)
    L.call('cmhar_conv3d_fwd', dims, C, xc.data_ptr(), wp.data_ptr(), None if rr is None else rr.data_ptr(),
           z1.data_ptr(), None, L.stream(xc.device))
    torch.cuda.synchronize()
    want = ref.permute(0, 2, 3, 4, 1).reshape(M, C) + (rr.float() if res else 0.)
    assert rel(z.float(), want) < 5e-3
    # (near-zero outputs: the summation-order difference is absolute, ~1e-6 of the accumulated magnitude)
    tol = torch.maximum(z1.float().abs(), z1.float().pow(2).mean().sqrt()) * 2.0 ** -7
    assert bool(((z.float() - z1.float()).abs() <= tol).all())
