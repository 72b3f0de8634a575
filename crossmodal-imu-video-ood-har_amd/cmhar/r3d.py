"""R3D-18 video backbone on the cmhar HIP library (north_star extension "VideoEncoder 3D-conv/R3D").

The reference has no 3-D CNN (its CNN options are per-frame 2-D torchvision models, `models.py:160-216`, and
torchvision is absent here), so this module follows torchvision's `models.video.r3d_18` architecture and
state_dict names (`stem.0.weight`, `layer{i}.{j}.conv{1,2}.{0,1}.*`, `layer{i}.0.downsample.{0,1}.*`): BasicStem
Conv3d(3,64,(3,7,7),s=(1,2,2),p=(1,3,3)) + BN + ReLU, four stages of two BasicBlocks (64/128/256/512 channels,
stride 2 at stages 2-4 with a 1x1x1 strided downsample), global average pool; `fc` is dropped (the encoder's own
projection follows).  Parity: unpinned w.r.t. the reference (no reference code); checked against the CPU
restatement `oracle/r3d_cpu.py` (F.conv3d / F.batch_norm) in tests/test_r3d_gpu.py.

Execution (MI355X): activations channels-last NDHWC in the compute dtype.  Convs with C % 64 == 0 (all but the
stem) run as implicit GEMMs on MFMA (`cmhar_conv3d_fwd` / `cmhar_conv3d_wgrad`: the im2col gather happens in the
operand loads, no column matrix in HBM); the stem (C = 3) and the fp32 parity mode use im2col
(`cmhar_conv3d_im2col`, kept from the forward for the weight gradient) + the GEMM.  BatchNorm3d with fused
residual/ReLU (`cmhar_bn_cl_fwd`); backward: fused ReLU-mask BN backward (also emitting the residual-branch
gradient), dgrad = dz·W (layout 1) gathered by `cmhar_conv3d_col2im`.
"""
from __future__ import annotations

import ctypes
import math

import torch
import torch.nn as nn

from . import _lib as L
from . import kernels as K
from ._lib import call, ptr
from .heads import bn_momentum


def _r8(x):
    return (x + 7) // 8 * 8


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Sequential(nn.Conv3d(inplanes, planes, 3, stride, 1, bias=False), nn.BatchNorm3d(planes),
                                   nn.ReLU(inplace=True))
        self.conv2 = nn.Sequential(nn.Conv3d(planes, planes, 3, 1, 1, bias=False), nn.BatchNorm3d(planes))
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride


class R3D18(L.NoReplicate, nn.Module):
    """torchvision `r3d_18(num_classes)` layout; `fc=None` → feature extractor returning (B, 512) fp32."""

    def __init__(self, num_classes=None, compute_dtype='bf16'):
        super().__init__()
        self.compute_dtype = compute_dtype
        self.stem = nn.Sequential(nn.Conv3d(3, 64, (3, 7, 7), (1, 2, 2), (1, 3, 3), bias=False), nn.BatchNorm3d(64),
                                  nn.ReLU(inplace=True))
        self.inplanes = 64
        self.layer1 = self._make_layer(64, 1)
        self.layer2 = self._make_layer(128, 2)
        self.layer3 = self._make_layer(256, 2)
        self.layer4 = self._make_layer(512, 2)
        self.fc = nn.Linear(512, num_classes) if num_classes else None
        self.feature_dim = 512
        # keep every conv's im2col matrix from the forward for the weight gradient (~38 GB at 32 clips of 16x112²,
        # sized for the 288 GB of HBM) instead of rebuilding it in the backward
        self.keep_cols = True
        for m in self.modules():     # torchvision VideoResNet.__init__ initialisation
            if isinstance(m, nn.Conv3d):
                nn.init.kaiming_normal_(m.weight, mode='fan_out', nonlinearity='relu')
            elif isinstance(m, nn.BatchNorm3d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
            elif isinstance(m, nn.Linear):
                nn.init.normal_(m.weight, 0, 0.01)
                nn.init.constant_(m.bias, 0)

    def _make_layer(self, planes, stride):
        ds = None
        if stride != 1 or self.inplanes != planes:
            ds = nn.Sequential(nn.Conv3d(self.inplanes, planes, 1, stride, bias=False), nn.BatchNorm3d(planes))
        blocks = [BasicBlock(self.inplanes, planes, stride, ds), BasicBlock(planes, planes)]
        self.inplanes = planes
        return nn.Sequential(*blocks)

    def blocks(self):
        for layer in (self.layer1, self.layer2, self.layer3, self.layer4):
            yield from layer

    def forward(self, x):
        """x: (B, C, T, H, W) as torchvision's VideoResNet.forward."""
        feat = run_r3d(self, x.transpose(1, 2), self.training)
        if self.fc is not None:
            from .models import linear_fp32
            feat = linear_fp32(feat, self.fc)
        return feat


# ------------------------------------------------------------------------------------------------------------
# one Conv3d (+ BatchNorm3d [+ residual] [+ ReLU]) unit
# ------------------------------------------------------------------------------------------------------------
def _dims(shape, conv, Kp):
    N, T, H, W, C = shape
    kt, kh, kw = conv.kernel_size
    st, sh, sw = conv.stride
    pt, ph, pw = conv.padding
    return (ctypes.c_int * 15)(N, T, H, W, C, kt, kh, kw, st, sh, sw, pt, ph, pw, Kp)


def _out_shape(shape, conv):
    N, T, H, W, _ = shape
    o = [(s + 2 * p - k) // st + 1 for s, p, k, st in zip((T, H, W), conv.padding, conv.kernel_size, conv.stride)]
    return (N, o[0], o[1], o[2], conv.out_channels)


def _pack(conv, dt, flip=False):
    """[Cout, Cin, kt, kh, kw] fp32 master → [Cout, Kp] compute dtype in the im2col k order (kt, kh, kw, Cin), zero
    padded to Kp; with flip also the tap-flipped, in/out-transposed [Cin, taps·Cout] weight of the stride-1 input
    gradient — both from one cmhar_conv_pack_weight pass (no torch permute / copy kernels on the step).
    Returns wp, or (wp, wf) when flip."""
    w = conv.weight.detach()
    if not w.is_contiguous():
        w = w.contiguous()
    co, ci, kt, kh, kw = w.shape
    kp = _r8(w[0].numel())
    wp = torch.empty(co, kp, dtype=dt, device=w.device)
    wf = torch.empty(ci, kt * kh * kw * co, dtype=dt, device=w.device) if flip else None
    call('cmhar_conv_pack_weight', L.dtype_code(dt), co, ci, kt, kh, kw, kp, ptr(w), ptr(wp), ptr(wf),
         L.stream(w.device))
    return (wp, wf) if flip else wp


def _pack_all(jobs, dt, dev):
    """[(conv, flip)] → {conv: wp, or (wp, wf) when flip}: every pack of `_pack` from ONE cmhar_conv_pack_weights
    launch (R3D-18's 19 block convs were 19 serial launches of a few blocks each)."""
    n = len(jobs)
    dims = (ctypes.c_int * (6 * n))()
    ptrs = (ctypes.c_void_p * (3 * n))()
    out, keep = {}, []
    for i, (conv, flip) in enumerate(jobs):
        w = conv.weight.detach()
        if not w.is_contiguous():
            w = w.contiguous()
            keep.append(w)
        co, ci, kt, kh, kw = w.shape
        kp = _r8(w[0].numel())
        wp = torch.empty(co, kp, dtype=dt, device=dev)
        wf = torch.empty(ci, kt * kh * kw * co, dtype=dt, device=dev) if flip else None
        dims[6 * i:6 * i + 6] = [co, ci, kt, kh, kw, kp]
        ptrs[3 * i:3 * i + 3] = [w.data_ptr(), wp.data_ptr(), ptr(wf)]
        out[conv] = (wp, wf) if flip else wp
    if n:
        call('cmhar_conv_pack_weights', L.dtype_code(dt), n, dims, ptrs, L.stream(dev))
    return out


def _stem_ok(x, shape, conv):
    """Implicit stem kernel (cmhar_conv3d_stem_*): bf16, <= 4 input channels, kw <= 8 taps at w-stride 2, 64 outputs
    (R3D-18's 3x7x7 (1,2,2) stem, ResNet-18's 7x7/2 stem run as (1, 7, 7))."""
    if x.dtype != torch.bfloat16 or shape[4] > 4 or conv.out_channels != 64 or conv.kernel_size[2] > 8 or \
            conv.stride[2] != 2:
        return False
    return L.lib().cmhar_conv3d_stem_tiles(_dims(shape, conv, _stem_kp(conv)), 64) > 0


def _stem_kp(conv):
    kt, kh, _ = conv.kernel_size
    return kt * kh * 32


def _pack_stem(conv):
    """[64, C, kt, kh, kw] fp32 master → [64, kt·kh·32] bf16, element iw·4 + c of each (it, ih) tap row."""
    w = conv.weight.detach()
    if not w.is_contiguous():
        w = w.contiguous()
    co, ci, kt, kh, kw = w.shape
    w4 = torch.empty(co, kt * kh * 32, dtype=torch.bfloat16, device=w.device)
    call('cmhar_conv_pack_stem', co, ci, kt, kh, kw, ptr(w), ptr(w4), L.stream(w.device))
    return w4


def _pack_flip(conv, dt):
    w = conv.weight.detach().contiguous()
    co, ci, kt, kh, kw = w.shape
    wf = torch.empty(ci, kt * kh * kw * co, dtype=dt, device=w.device)
    call('cmhar_conv_pack_weight', L.dtype_code(dt), co, ci, kt, kh, kw, 0, ptr(w), None, ptr(wf), L.stream(w.device))
    return wf


def _im2col(x, shape, conv, Kp, rows):
    dims = _dims(shape, conv, Kp)
    M = math.prod(_out_shape(shape, conv)[:4])
    col = torch.empty(rows, Kp, dtype=x.dtype, device=x.device)
    if rows > M:
        col[M:].zero_()
    dc = L.dtype_code(x.dtype)
    call('cmhar_conv3d_im2col', dc, dc, dims, ptr(x), ptr(col), L.stream(x.device))
    return col


def _bn_fwd(z, bn, res, relu, training):
    M, Cc = z.shape
    y = torch.empty_like(z)
    sm = torch.empty(Cc, dtype=torch.float32, device=z.device)
    sr = torch.empty(Cc, dtype=torch.float32, device=z.device)
    ws = K.workspace(L.lib().cmhar_bn_cl_ws(M, Cc), z.device)
    upd = training and bn.track_running_stats
    use_batch = training or not bn.track_running_stats     # torch: eval without running stats → batch statistics
    call('cmhar_bn_cl_fwd', L.dtype_code(z.dtype), M, Cc, ptr(z), ptr(res), ptr(y), ptr(bn.weight), ptr(bn.bias),
         ptr(bn.running_mean) if upd or not use_batch else None,
         ptr(bn.running_var) if upd or not use_batch else None,
         ptr(sm), ptr(sr), int(use_batch), bn_momentum(bn, upd), bn.eps, int(relu),
         ptr(bn.num_batches_tracked) if upd else None, ptr(ws), L.stream(z.device))
    return y, sm, sr


def _bn_fwd_tiles(z, bn, res, relu, tstats, ntile):
    """Training BatchNorm3d of a conv output whose per-tile statistics the conv epilogue wrote into `tstats`
    (`ntile` tiles, layout of cmhar_conv3d_fwd_stats_floats)."""
    M, Cc = z.shape
    y = torch.empty_like(z)
    sm = torch.empty(Cc, dtype=torch.float32, device=z.device)
    sr = torch.empty(Cc, dtype=torch.float32, device=z.device)
    call('cmhar_bn_cl_fwd_tiles', M, Cc, ntile, ptr(tstats), ptr(z), ptr(res), ptr(y), ptr(bn.weight), ptr(bn.bias),
         ptr(bn.running_mean), ptr(bn.running_var), ptr(sm), ptr(sr),
         bn_momentum(bn, True), bn.eps, int(relu), ptr(bn.num_batches_tracked),
         L.stream(z.device))
    return y, sm, sr


class _Unit:
    """Forward state of one conv+BN unit (input, pre-BN output, BN output, batch statistics)."""
    __slots__ = ('conv', 'bn', 'relu', 'shape', 'oshape', 'x', 'z', 'y', 'sm', 'sr', 'Kp', 'rows', 'wp', 'col',
                 'igemm', 'wf', 'stem', 'res')


def _pointwise(conv, shape, Kp, M, rows):
    """1×1×1, stride 1, no padding, Kp == C, no row padding: the im2col matrix IS the input viewed [M, C]."""
    return tuple(conv.kernel_size) == (1, 1, 1) and tuple(conv.stride) == (1, 1, 1) and \
        tuple(conv.padding) == (0, 0, 0) and Kp == shape[4] and rows == M


def _igemm_ok(x, shape, conv, Kp):
    """Implicit-GEMM conv (no column matrix in HBM): bf16, C % 64 == 0 (a 64-wide K-tile stays in one tap)."""
    return x.dtype == torch.bfloat16 and shape[4] % 64 == 0 and Kp == conv.weight[0].numel()


def _conv_fwd(x, shape, conv, wp, stats):
    """The convolution of a unit, as the step launches it: z [M, Cout] (compute dtype) = conv(x) on the implicit stem
    (C <= 4), the split-K implicit GEMM (layer-4 geometries), the implicit GEMM (C % 64 == 0), the pointwise GEMM, or
    im2col + GEMM.  stats: also have the conv epilogue write BatchNorm tile statistics where the kernel can.
    Returns (z, col, wp, stem, igemm, tstats, ntile); col is the im2col matrix when one was built (or x itself for a
    pointwise conv), wp the weight pack the conv used (the stem packs its own layout)."""
    oshape = _out_shape(shape, conv)
    M = math.prod(oshape[:4])
    Kp = _r8(conv.weight[0].numel())
    rows = _r8(M) if x.dtype == torch.bfloat16 else M
    z = torch.empty(M, conv.out_channels, dtype=x.dtype, device=x.device)
    stem = _stem_ok(x, shape, conv)
    igemm = not stem and _igemm_ok(x, shape, conv, Kp)
    tstats, ntile, col = None, 0, None
    if stem:
        # implicit stem: no column matrix; the packed [64, kt·kh·32] weight replaces the im2col-order pack
        wp = _pack_stem(conv)
        dims = _dims(shape, conv, _stem_kp(conv))
        if stats:
            ntile = L.lib().cmhar_conv3d_stem_tiles(dims, 64)
            tstats = K.workspace(L.lib().cmhar_conv3d_stem_stats_floats(dims, 64), x.device)
        call('cmhar_conv3d_stem_fwd', dims, 64, ptr(x), ptr(wp), ptr(z), ptr(tstats), L.stream(x.device))
    elif igemm:
        dims = _dims(shape, conv, Kp)
        if not _conv_fwd_split(dims, conv.out_channels, x, wp, None, z):
            if stats:      # BN statistics from the conv epilogue (no statistics pass)
                ntile = L.lib().cmhar_conv3d_fwd_tiles(dims, conv.out_channels)
                tstats = K.workspace(L.lib().cmhar_conv3d_fwd_stats_floats(dims, conv.out_channels), x.device)
            call('cmhar_conv3d_fwd', dims, conv.out_channels, ptr(x), ptr(wp), None, ptr(z), ptr(tstats),
                 L.stream(x.device))
    elif _pointwise(conv, shape, Kp, M, rows):
        col = x.reshape(M, Kp)
        K.gemm(0, col, wp, z)
    else:
        col = _im2col(x, shape, conv, Kp, rows)
        K.gemm(0, col[:M], wp, z)
    return z, col, wp, stem, igemm, tstats, ntile


def _unit_fwd(x, shape, conv, bn, relu, training, save, res=None, wp=None, keep_col=True, wf=None):
    oshape = _out_shape(shape, conv)
    M = math.prod(oshape[:4])
    Kp = _r8(conv.weight[0].numel())
    rows = _r8(M) if x.dtype == torch.bfloat16 else M
    z, col, wp, stem, igemm, tstats, ntile = _conv_fwd(x, shape, conv, wp, training and bn.track_running_stats)
    if tstats is not None:
        y, sm, sr = _bn_fwd_tiles(z, bn, res, relu, tstats, ntile)
    else:
        y, sm, sr = _bn_fwd(z, bn, res, relu, training)
    u = None
    if save:
        u = _Unit()
        u.conv, u.bn, u.relu, u.shape, u.oshape, u.Kp, u.rows, u.wp = conv, bn, relu, shape, oshape, Kp, rows, wp
        u.x, u.z, u.y, u.sm, u.sr = x, z, y, sm, sr
        u.col = col if keep_col else None
        u.igemm = igemm
        u.wf = wf
        u.stem = stem
        u.res = res is not None
    return y, oshape, u


def _dgrad_igemm_ok(conv):
    return tuple(conv.stride) == (1, 1, 1) and conv.out_channels % 64 == 0 and \
        all(2 * p == k - 1 for p, k in zip(conv.padding, conv.kernel_size))


def _dgrad_igemm(dz, conv, oshape, x, dx_acc=None, wf=None):
    """Input gradient of a stride-1 'same' conv as the conv of dz (NDHWC [M, Cout] bf16) with the tap-flipped,
    in/out-transposed weight (padding k-1-p = p): an implicit GEMM, no dcol / col2im; dx_acc (the residual-branch
    gradient) is added in its epilogue.  Returns dx shaped like x."""
    cin, cout = conv.weight.shape[1], conv.weight.shape[0]
    if wf is None:
        wf = _pack_flip(conv, dz.dtype)
    N, To, Ho, Wo, _ = oshape
    kt, kh, kw = conv.kernel_size
    pt, ph, pw = conv.padding
    dims = (ctypes.c_int * 15)(N, To, Ho, Wo, cout, kt, kh, kw, 1, 1, 1, pt, ph, pw, wf.shape[1])
    dx = torch.empty_like(x)
    if not _conv_fwd_split(dims, cin, dz, wf, dx_acc, dx):
        call('cmhar_conv3d_fwd', dims, cin, ptr(dz), ptr(wf), ptr(dx_acc), ptr(dx), None, L.stream(dz.device))
    return dx


def _conv_fwd_split(dims, cout, x, w, res, z):
    """The split-K implicit-GEMM forward when the library plans one for this geometry (the small-M layer-4 convs:
    `cmhar_conv3d_fwd_split_ws` > 0); False otherwise.  No BatchNorm tile statistics come with it."""
    n = L.lib().cmhar_conv3d_fwd_split_ws(dims, cout)
    if n <= 0:
        return False
    ws = K.workspace(n, x.device)
    call('cmhar_conv3d_fwd_split', dims, cout, ptr(x), ptr(w), ptr(res), ptr(z), ptr(ws), L.stream(x.device))
    return True


def _grad_dest(grads, p, dev):
    """Where p's fp32 gradient is written: (destination, accumulate_into).  `grads` is a dict (a fresh tensor is
    recorded in it) or a gradient sink (cmhar.grads: AutogradSink, or the data-parallel FlatGradSink whose
    destination is p's slice of the flat bucket buffer).  When the sink asks for accumulation (β = 1: `.grad` already
    held a value) the gradient goes to a temporary that `_grad_acc` adds into the destination."""
    if isinstance(grads, dict) or not p.requires_grad:
        g = torch.empty(p.shape, dtype=torch.float32, device=dev)
        if isinstance(grads, dict):
            grads[p] = g
        return g, None                        # (a frozen parameter's gradient is computed and dropped)
    out, beta = grads.dest([p], tuple(p.shape), dev)
    if beta == 0.0:
        return out, None
    return torch.empty(p.shape, dtype=torch.float32, device=dev), out


def _grad_acc(tmp, acc):
    if acc is not None:
        acc.add_(tmp)


def _store_wgrad(conv, src, rs, cs, grads):
    """Packed fp32 weight gradient [Cout, Kp] → a contiguous gradient in the parameter's own layout (one HIP pass;
    a strided view here would make autograd's gradient accumulation copy it with a torch kernel)."""
    w = conv.weight
    co, ci, kt, kh, kw = w.shape
    p = getattr(conv, 'param', None)          # a 2-D conv run as (1, kh, kw): gradient in the parameter's shape
    g, acc = _grad_dest(grads, w if p is None else p, src.device)
    call('cmhar_conv_grad_unpack', co, ci, kt * kh, kw, src.shape[1], rs, cs, ptr(src), ptr(g), L.stream(src.device))
    _grad_acc(g, acc)


def _unit_grads_done(grads, u):
    """A unit's three parameter gradients (BN weight, BN bias, conv weight) are final: tell a gradient sink (the
    data-parallel reducer all-reduces a bucket as soon as every gradient in it is written)."""
    if not isinstance(grads, dict):
        p = getattr(u.conv, 'param', None)
        grads.done([u.bn.weight, u.bn.bias, u.conv.weight if p is None else p])


def unit_param_order(m: 'R3D18'):
    """Backward-production order of the R3D-18 parameters (`_backward_impl`: blocks last→first, per block conv2,
    downsample, conv1, then the stem; per unit BN weight, BN bias, conv weight) — the flat gradient buffer's layout,
    so that the reducer's buckets fill in order during the backward."""
    order = []
    for blk in reversed(list(m.blocks())):
        seqs = [blk.conv2] + ([blk.downsample] if blk.downsample is not None else []) + [blk.conv1]
        for sq in seqs:
            order += [sq[1].weight, sq[1].bias, sq[0].weight]
    order += [m.stem[1].weight, m.stem[1].bias, m.stem[0].weight]
    return order


def _bn_bwd(u, dy, dz, dres, dw_bn, db_bn, training):
    """BatchNorm(+residual)+activation backward of a unit into dz (and dres).  Without a residual input the
    activation mask is recomputed from z in the forward's arithmetic (`cmhar_bn_cl_bwd_nores`: y not re-read)."""
    M, Cc = u.z.shape
    dt = u.z.dtype
    ws = K.workspace(L.lib().cmhar_bn_cl_ws(M, Cc), dy.device)
    use_batch = int(training or not u.bn.track_running_stats)
    if u.relu and not u.res and dres is None:
        call('cmhar_bn_cl_bwd_nores', L.dtype_code(dt), M, Cc, ptr(u.z), ptr(dy), ptr(u.bn.weight), ptr(u.bn.bias),
             ptr(u.sm), ptr(u.sr), ptr(dz), ptr(dw_bn), ptr(db_bn), use_batch, int(u.relu), ptr(ws),
             L.stream(dy.device))
    else:
        call('cmhar_bn_cl_bwd', L.dtype_code(dt), M, Cc, ptr(u.z), ptr(u.y), ptr(dy), ptr(u.bn.weight), ptr(u.sm),
             ptr(u.sr), ptr(dz), ptr(dres), ptr(dw_bn), ptr(db_bn), use_batch, int(u.relu), ptr(ws),
             L.stream(dy.device))


def _unit_bwd(u, dy, grads, training, need_dx, want_dres, dx_acc=None):
    """Returns (dx or None, dres or None); dx accumulates into dx_acc when given."""
    M, Cc = u.z.shape
    dt = u.z.dtype
    dz = torch.empty(u.rows, Cc, dtype=dt, device=dy.device)
    if u.rows > M:
        dz[M:].zero_()
    dres = torch.empty(M, Cc, dtype=dt, device=dy.device) if want_dres else None
    dw_bn, acc_w = _grad_dest(grads, u.bn.weight, dy.device)
    db_bn, acc_b = _grad_dest(grads, u.bn.bias, dy.device)
    _bn_bwd(u, dy, dz, dres, dw_bn, db_bn, training)
    _grad_acc(dw_bn, acc_w)
    _grad_acc(db_bn, acc_b)
    if u.stem and need_dx:
        raise RuntimeError('the implicit stem has no input gradient (its input is the video)')
    dwp = _conv_wgrad(u, dz)
    w = u.conv.weight
    if u.stem:
        _store_wgrad(u.conv, dwp, 32, 4, grads)
    else:
        _store_wgrad(u.conv, dwp, w.shape[4] * w.shape[1], w.shape[1], grads)
    _unit_grads_done(grads, u)
    dx = _conv_dgrad(u, dz, dx_acc) if need_dx else None
    return dx, dres


def _conv_wgrad(u, dz):
    """Weight gradient of a unit's conv from dz ([rows, Cout], rows past M zero): fp32 in the packed layout the
    forward used — [Cout, Kp] in the im2col k order, or [64, kt·kh·32] for the implicit stem.  Implicit stem / row
    slab / nine-tap / gather kernels with their split reduces, or dzᵀ · col on the GEMM (split-K)."""
    Cc = dz.shape[1]
    dev = dz.device
    if u.stem:
        dims = _dims(u.shape, u.conv, _stem_kp(u.conv))
        dw4 = torch.empty(Cc, _stem_kp(u.conv), dtype=torch.float32, device=dev)
        ws = K.workspace(L.lib().cmhar_conv3d_stem_wgrad_ws(dims, Cc), dev)
        call('cmhar_conv3d_stem_wgrad', dims, Cc, ptr(u.x), ptr(dz), ptr(dw4), ptr(ws), L.stream(dev))
        return dw4
    dwp = torch.empty(Cc, u.Kp, dtype=torch.float32, device=dev)
    if u.igemm:
        dims = _dims(u.shape, u.conv, u.Kp)
        n = L.lib().cmhar_conv3d_wgrad_ws(dims, Cc)
        ws = K.workspace(n, dev) if n > 0 else None
        call('cmhar_conv3d_wgrad', dims, Cc, ptr(u.x), ptr(dz), ptr(dwp), ptr(ws), L.stream(dev))
    else:
        col = u.col if u.col is not None else _im2col(u.x, u.shape, u.conv, u.Kp, u.rows)
        u.col = None
        splits = None
        if dz.dtype == torch.bfloat16:
            # the stem's weight gradient is a 64 x 448 output over ~1.6 M rows: ~1024 split-K slices of >= 4096 rows
            # (the generic heuristic caps at 32 splits = 128 workgroups for this 4-tile output)
            tiles = -(-Cc // 128) * -(-u.Kp // 128)
            splits = max(1, min(1024 // tiles, u.rows // 4096))
        K.gemm(2, dz, col, dwp, splits=splits)
        del col
    return dwp


def _conv_dgrad(u, dz, dx_acc=None):
    """Input gradient of a unit's conv (+ dx_acc, the residual-branch gradient, when given): the flipped-weight
    implicit GEMM for stride-1 'same' convs (split-K where the forward plan splits), dz · W for a pointwise conv,
    else dcol = dz · W on the GEMM + col2im.  Returns dx shaped like u.x (dx_acc itself when accumulating in place)."""
    M = math.prod(u.oshape[:4])
    dt = dz.dtype
    dev = dz.device
    if u.igemm and _dgrad_igemm_ok(u.conv):
        return _dgrad_igemm(dz, u.conv, u.oshape, u.x, dx_acc, u.wf)
    if _pointwise(u.conv, u.shape, u.Kp, M, u.rows):
        # 1×1 stride-1: dx = dz·W directly (the col2im of a pointwise conv is the identity); the residual-branch
        # gradient is added in the GEMM epilogue (element-wise read-then-write of the same buffer)
        if dx_acc is not None:
            dxv = dx_acc.reshape(M, u.Kp)
            K.gemm(1, dz[:M], u.wp, dxv, residual=dxv)
            return dx_acc
        dx = torch.empty_like(u.x)
        K.gemm(1, dz[:M], u.wp, dx.reshape(M, u.Kp))
        return dx
    dcol = torch.empty(M, u.Kp, dtype=dt, device=dev)
    K.gemm(1, dz[:M], u.wp, dcol)
    dx = dx_acc if dx_acc is not None else torch.empty_like(u.x)
    call('cmhar_conv3d_col2im', L.dtype_code(dt), _dims(u.shape, u.conv, u.Kp), ptr(dcol), ptr(dx),
         int(dx_acc is not None), L.stream(dev))
    return dx


# ------------------------------------------------------------------------------------------------------------
# whole backbone
# ------------------------------------------------------------------------------------------------------------
def _forward_impl(m: R3D18, video, training, save):
    """video (B, T, C, H, W) fp32 → features (B, 512) fp32 (+ saved units)."""
    dt = torch.bfloat16 if m.compute_dtype == 'bf16' else torch.float32
    B, T, Cc, H, W = video.shape
    x = torch.empty(B, T, H, W, Cc, dtype=dt, device=video.device)
    call('cmhar_video_to_ndhwc', L.dtype_code(dt), B, T, Cc, H, W, ptr(video), ptr(x), L.stream(video.device))
    shape = (B, T, H, W, Cc)
    units = []
    # every block conv's pack from one launch; the backward's flipped weight (stride-1 input gradient on the
    # implicit-GEMM kernels) from the same pass
    seqs = [sq for blk in m.blocks() for sq in ([blk.conv1] + ([blk.downsample] if blk.downsample is not None else [])
                                                 + [blk.conv2])]
    packs = _pack_all([(sq[0], save and dt == torch.bfloat16 and _dgrad_igemm_ok(sq[0]) and
                        sq[0].in_channels % 64 == 0) for sq in seqs], dt, video.device)

    def unit(xin, shp, seq, relu, res=None):
        conv, bn = seq[0], seq[1]
        wf = None
        if _stem_ok(xin, shp, conv):
            wp = None                                # _unit_fwd packs the stem's own layout
        elif conv in packs:
            wp = packs[conv]
            if isinstance(wp, tuple):
                wp, wf = wp
        else:
            wp = _pack(conv, dt)
        y, osh, u = _unit_fwd(xin, shp, conv, bn, relu, training, save, res=res, wp=wp, keep_col=m.keep_cols, wf=wf)
        units.append(u)
        return y, osh

    h, shape = unit(x, shape, m.stem, True)
    for blk in m.blocks():
        x_in, s_in = h, shape
        h1, s1 = unit(x_in, s_in, blk.conv1, True)
        if blk.downsample is not None:
            idn, _ = unit(x_in, s_in, blk.downsample, False)
        else:
            idn = x_in
        h, shape = unit(h1, s1, blk.conv2, True, res=idn)
    N, To, Ho, Wo, Co = shape
    feat = torch.empty(N, Co, dtype=torch.float32, device=video.device)
    call('cmhar_avgpool_cl', L.dtype_code(dt), N, To * Ho * Wo, Co, ptr(h), ptr(feat), L.stream(video.device))
    st = (units, shape) if save else None
    return feat, st


def _backward_impl(m: R3D18, st, dfeat, training, grads=None):
    """Parameter gradients into `grads` (a dict, returned; or a gradient sink, cmhar.grads)."""
    units, shape = st
    if grads is None:
        grads = {}
    N, To, Ho, Wo, Co = shape
    dt = units[-1].z.dtype
    dh = torch.empty(N * To * Ho * Wo, Co, dtype=dt, device=dfeat.device)
    call('cmhar_avgpool_cl_bwd', L.dtype_code(dt), N, To * Ho * Wo, Co, ptr(dfeat.contiguous()), ptr(dh),
         L.stream(dfeat.device))
    i = len(units) - 1
    for blk in reversed(list(m.blocks())):
        has_ds = blk.downsample is not None
        u2 = units[i]
        u_ds = units[i - 1] if has_ds else None
        u1 = units[i - 2] if has_ds else units[i - 1]
        i -= 3 if has_ds else 2
        dh1, dres = _unit_bwd(u2, dh, grads, training, True, True)
        if has_ds:
            dx, _ = _unit_bwd(u_ds, dres, grads, training, True, False)
            dx, _ = _unit_bwd(u1, dh1, grads, training, True, False, dx_acc=dx)
        else:
            dx, _ = _unit_bwd(u1, dh1, grads, training, True, False, dx_acc=dres)
        dh = dx.reshape(-1, dx.shape[-1])
    _unit_bwd(units[0], dh, grads, training, False, False)     # stem: no pixel gradient
    return grads


class _R3DFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, video, module, training, *params):
        feat, st = _forward_impl(module, video.contiguous().float(), training, save=True)
        ctx.module, ctx.st, ctx.training = module, st, training
        return feat

    @staticmethod
    def backward(ctx, dfeat):
        m = ctx.module
        from .grads import AutogradSink
        sink = getattr(m, '_grad_sink', None) or AutogradSink()
        _backward_impl(m, ctx.st, dfeat, ctx.training, sink)
        ctx.st = None
        out = []
        for p in m.parameters():
            if m.fc is not None and (p is m.fc.weight or p is m.fc.bias):
                out.append(None)
            else:
                out.append(sink.result(p) if p.requires_grad else None)
        return (None, None, None, *out)


def run_r3d(m: R3D18, video_btchw: torch.Tensor, training: bool) -> torch.Tensor:
    """video (B, T, C, H, W) fp32 on the GPU → (B, 512) fp32 pooled features (autograd-aware)."""
    if not video_btchw.is_cuda:
        raise RuntimeError('R3D18 runs on the cmhar HIP library: move the module and input to the GPU')
    params = list(m.parameters())
    if torch.is_grad_enabled() and any(p.requires_grad for p in params):
        return _R3DFn.apply(video_btchw, m, training, *params)
    feat, _ = _forward_impl(m, video_btchw.contiguous().float(), training, save=False)
    return feat
