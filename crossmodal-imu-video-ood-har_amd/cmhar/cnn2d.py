"""Per-frame 2-D CNN video backbones of the reference's `VideoEncoder` (`src/models/models.py:163-173`, forward
`:208-216`): `video_backbone='resnet18'` → torchvision `resnet18` without avgpool/fc (`children()[:-2]`, 512 features)
and `'mobilenet_v2'` → torchvision `mobilenet_v2().features` (1280 features), applied to every frame of the
(B·T, 3, H, W) batch, then `adaptive_avg_pool2d` → per-frame `projection` → mean over T.

Module trees and state_dict names follow torchvision exactly (`backbone.0.weight` = conv1, `backbone.4.0.conv1.weight`,
`backbone.5.0.downsample.0.weight`, …; `backbone.1.conv.0.0.weight`, `backbone.18.1.running_var`, …), so a torchvision
checkpoint of the same network loads with `strict=True`.  torchvision itself is absent here, so parity is against the
build's own CPU restatement (`oracle/cnn2d_cpu.py`: F.conv2d / F.batch_norm / F.max_pool2d / F.relu6 on the same
architecture) — "parity unpinned" w.r.t. the reference.

Execution (MI355X): frames channels-last NHWC in the compute dtype; every dense Conv2d is the conv3d machinery with
kt = 1 (implicit GEMM on MFMA when C % 64 == 0, else im2col + GEMM; 1×1 stride-1 convs use the activation itself as
the GEMM operand); BatchNorm2d + ReLU / ReLU6 (+ residual) fused in one apply pass; MaxPool2d and the depthwise
convolutions of MobileNetV2's inverted residuals are `csrc/cnn2d.hip` kernels.  The whole backbone forward/backward
is one autograd node, as `cmhar.r3d`.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _lib as L
from . import kernels as K
from ._lib import call, ptr
from .r3d import _bn_bwd, _bn_fwd, _dgrad_igemm_ok, _grad_acc, _grad_dest, _pack, _stem_ok, _unit_bwd, _unit_fwd

RELU, RELU6 = 1, 2


class _As3d:
    """A Conv2d seen as the (1, kh, kw) Conv3d the NDHWC kernels run on frames (T = 1); gradients are keyed by the
    real parameter (`param`) in its own 4-D shape."""

    def __init__(self, conv: nn.Conv2d):
        self.conv2d = conv
        self.param = conv.weight
        self.kernel_size = (1,) + tuple(conv.kernel_size)
        self.stride = (1,) + tuple(conv.stride)
        self.padding = (0,) + tuple(conv.padding)
        self.out_channels = conv.out_channels

    @property
    def weight(self):
        return self.param.unsqueeze(2)


def _init_torchvision(modules):
    for m in modules:
        if isinstance(m, nn.Conv2d):
            nn.init.kaiming_normal_(m.weight, mode='fan_out', nonlinearity='relu')
            if m.bias is not None:
                nn.init.zeros_(m.bias)
        elif isinstance(m, (nn.BatchNorm2d, nn.GroupNorm)):
            nn.init.ones_(m.weight)
            nn.init.zeros_(m.bias)


# ---------------------------------------------------------------------------------------------------------------
# ResNet-18 (torchvision.models.resnet18, children()[:-2])
# ---------------------------------------------------------------------------------------------------------------
class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride


def _resnet_layer(inplanes, planes, stride):
    ds = None
    if stride != 1 or inplanes != planes:
        ds = nn.Sequential(nn.Conv2d(inplanes, planes, 1, stride, bias=False), nn.BatchNorm2d(planes))
    return nn.Sequential(BasicBlock(inplanes, planes, stride, ds), BasicBlock(planes, planes))


class ResNet18Features(L.NoReplicate, nn.Sequential):
    """conv1, bn1, relu, maxpool, layer1..layer4 — `nn.Sequential(*list(resnet18().children())[:-2])`."""
    feature_dim = 512

    def __init__(self, compute_dtype='bf16'):
        super().__init__(nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64), nn.ReLU(inplace=True),
                         nn.MaxPool2d(3, 2, 1), _resnet_layer(64, 64, 1), _resnet_layer(64, 128, 2),
                         _resnet_layer(128, 256, 2), _resnet_layer(256, 512, 2))
        self.compute_dtype = compute_dtype
        _init_torchvision(self.modules())


# ---------------------------------------------------------------------------------------------------------------
# MobileNetV2 (torchvision.models.mobilenet_v2().features)
# ---------------------------------------------------------------------------------------------------------------
class Conv2dNormActivation(nn.Sequential):
    def __init__(self, cin, cout, kernel_size=3, stride=1, groups=1):
        pad = (kernel_size - 1) // 2
        super().__init__(nn.Conv2d(cin, cout, kernel_size, stride, pad, groups=groups, bias=False),
                         nn.BatchNorm2d(cout), nn.ReLU6(inplace=True))


class InvertedResidual(nn.Module):
    def __init__(self, inp, oup, stride, expand_ratio):
        super().__init__()
        self.stride = stride
        hidden = int(round(inp * expand_ratio))
        self.use_res_connect = stride == 1 and inp == oup
        layers = []
        if expand_ratio != 1:
            layers.append(Conv2dNormActivation(inp, hidden, kernel_size=1))
        layers.extend([Conv2dNormActivation(hidden, hidden, stride=stride, groups=hidden),
                       nn.Conv2d(hidden, oup, 1, 1, 0, bias=False), nn.BatchNorm2d(oup)])
        self.conv = nn.Sequential(*layers)
        self.out_channels = oup


class MobileNetV2Features(L.NoReplicate, nn.Sequential):
    """torchvision `mobilenet_v2(width_mult=1.0).features`: 19 entries, last channel 1280."""
    feature_dim = 1280
    SETTING = [[1, 16, 1, 1], [6, 24, 2, 2], [6, 32, 3, 2], [6, 64, 4, 2], [6, 96, 3, 1], [6, 160, 3, 2],
               [6, 320, 1, 1]]

    def __init__(self, compute_dtype='bf16'):
        layers = [Conv2dNormActivation(3, 32, stride=2)]
        cin = 32
        for t, c, n, s in self.SETTING:
            for i in range(n):
                layers.append(InvertedResidual(cin, c, s if i == 0 else 1, t))
                cin = c
        layers.append(Conv2dNormActivation(cin, 1280, kernel_size=1))
        super().__init__(*layers)
        self.compute_dtype = compute_dtype
        _init_torchvision(self.modules())


# ---------------------------------------------------------------------------------------------------------------
# units: dense conv (+BN, act, residual) via r3d's unit, depthwise conv (+BN, act), max pool
# ---------------------------------------------------------------------------------------------------------------
class _DwUnit:
    __slots__ = ('conv', 'bn', 'relu', 'shape', 'oshape', 'x', 'z', 'y', 'sm', 'sr', 'res')


def _geom(shape, conv):
    N, _, H, W, C = shape
    k, s, p = conv.kernel_size[0], conv.stride[0], conv.padding[0]
    if conv.kernel_size[0] != conv.kernel_size[1] or conv.stride[0] != conv.stride[1] or \
            conv.padding[0] != conv.padding[1]:
        raise ValueError('square depthwise kernels / strides / padding only')
    return N, H, W, C, k, s, p, (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1


def _dw_fwd(x, shape, conv, bn, relu, training, save):
    N, H, W, C, k, s, p, Ho, Wo = _geom(shape, conv)
    z = torch.empty(N * Ho * Wo, C, dtype=x.dtype, device=x.device)
    call('cmhar_dwconv2d_cl_fwd', L.dtype_code(x.dtype), N, H, W, C, k, s, p, ptr(x), ptr(conv.weight.detach()),
         ptr(z), L.stream(x.device))
    y, sm, sr = _bn_fwd(z, bn, None, relu, training)
    oshape = (N, 1, Ho, Wo, C)
    u = None
    if save:
        u = _DwUnit()
        u.conv, u.bn, u.relu, u.shape, u.oshape, u.x, u.z, u.y, u.sm, u.sr = conv, bn, relu, shape, oshape, x, z, y, \
            sm, sr
        u.res = False
    return y, oshape, u


def _dw_bwd(u, dy, grads, training):
    M, C = u.z.shape
    dt = u.z.dtype
    dev = dy.device
    dz = torch.empty(M, C, dtype=dt, device=dev)
    dw_bn, acc_w = _grad_dest(grads, u.bn.weight, dev)
    db_bn, acc_b = _grad_dest(grads, u.bn.bias, dev)
    _bn_bwd(u, dy, dz, None, dw_bn, db_bn, training)
    _grad_acc(dw_bn, acc_w)
    _grad_acc(db_bn, acc_b)
    N, H, W, C_, k, s, p, _, _ = _geom(u.shape, u.conv)
    dwt, acc = _grad_dest(grads, u.conv.weight, dev)
    n = L.lib().cmhar_dwconv2d_cl_wgrad_ws(N, H, W, C, k, s, p)
    wsw = K.workspace(n, dev)
    call('cmhar_dwconv2d_cl_wgrad', L.dtype_code(dt), N, H, W, C, k, s, p, ptr(u.x), ptr(dz), ptr(dwt), ptr(wsw),
         L.stream(dev))
    _grad_acc(dwt, acc)
    if not isinstance(grads, dict):
        grads.done([u.bn.weight, u.bn.bias, u.conv.weight])
    dx = torch.empty_like(u.x)
    call('cmhar_dwconv2d_cl_dgrad', L.dtype_code(dt), N, H, W, C, k, s, p, ptr(dz), ptr(u.conv.weight.detach()),
         ptr(dx), L.stream(dev))
    return dx


def _maxpool_fwd(x, shape, pool):
    N, _, H, W, C = shape
    k, s, p = pool.kernel_size, pool.stride, pool.padding
    if pool.dilation != 1 or pool.ceil_mode:
        raise ValueError('MaxPool2d: dilation 1, floor mode only')
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    y = torch.empty(N * Ho * Wo, C, dtype=x.dtype, device=x.device)
    arg = torch.empty(N * Ho * Wo, C, dtype=torch.uint8, device=x.device)
    call('cmhar_maxpool2d_cl_fwd', L.dtype_code(x.dtype), N, H, W, C, k, s, p, ptr(x), ptr(y), ptr(arg),
         L.stream(x.device))
    return y, (N, 1, Ho, Wo, C), (shape, (k, s, p), arg)


def _maxpool_bwd(st, dy, dt):
    (N, _, H, W, C), (k, s, p), arg = st
    dx = torch.empty(N * H * W, C, dtype=dt, device=dy.device)
    call('cmhar_maxpool2d_cl_bwd', L.dtype_code(dt), N, H, W, C, k, s, p, ptr(dy), ptr(arg), ptr(dx),
         L.stream(dy.device))
    return dx


# ---------------------------------------------------------------------------------------------------------------
# whole backbones
# ---------------------------------------------------------------------------------------------------------------
def _dtype(m):
    return torch.bfloat16 if m.compute_dtype == 'bf16' else torch.float32


def _frames_nhwc(video, dt):
    B, T, Cc, H, W = video.shape
    x = torch.empty(B * T, H, W, Cc, dtype=dt, device=video.device)
    call('cmhar_video_to_ndhwc', L.dtype_code(dt), B, T, Cc, H, W, ptr(video), ptr(x), L.stream(video.device))
    return x, (B * T, 1, H, W, Cc)


def _unit(units, xin, shp, conv2d, bn, relu, training, save, res=None):
    conv = _As3d(conv2d)
    wf = None
    if _stem_ok(xin, shp, conv):
        wp = None                                   # _unit_fwd packs the implicit stem's own layout
    elif save and xin.dtype == torch.bfloat16 and _dgrad_igemm_ok(conv) and shp[4] % 64 == 0:
        wp, wf = _pack(conv, xin.dtype, flip=True)
    else:
        wp = _pack(conv, xin.dtype)
    y, osh, u = _unit_fwd(xin, shp, conv, bn, relu, training, save, res=res, wp=wp, keep_col=True, wf=wf)
    units.append(u)
    return y, osh


def _resnet_forward(m: ResNet18Features, video, training, save):
    dt = _dtype(m)
    x, shape = _frames_nhwc(video, dt)
    units = []
    h, shape = _unit(units, x, shape, m[0], m[1], RELU, training, save)
    h, shape, pool_st = _maxpool_fwd(h, shape, m[3])
    for layer in list(m)[4:8]:
        for blk in layer:
            x_in, s_in = h, shape
            h1, s1 = _unit(units, x_in, s_in, blk.conv1, blk.bn1, RELU, training, save)
            if blk.downsample is not None:
                idn, _ = _unit(units, x_in, s_in, blk.downsample[0], blk.downsample[1], 0, training, save)
            else:
                idn = x_in
            h, shape = _unit(units, h1, s1, blk.conv2, blk.bn2, RELU, training, save, res=idn)
    return h, shape, ((units, pool_st, shape) if save else None)


def _resnet_backward(m: ResNet18Features, st, dh, training, grads):
    units, pool_st, _ = st
    i = len(units) - 1
    for layer in reversed(list(m)[4:8]):
        for blk in reversed(list(layer)):
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
    dh = _maxpool_bwd(pool_st, dh, dh.dtype)
    _unit_bwd(units[0], dh, grads, training, False, False)        # stem: no pixel gradient
    return grads


def _mobilenet_forward(m: MobileNetV2Features, video, training, save):
    dt = _dtype(m)
    x, shape = _frames_nhwc(video, dt)
    units = []
    stem = m[0]
    h, shape = _unit(units, x, shape, stem[0], stem[1], RELU6, training, save)
    for blk in list(m)[1:-1]:     # (no Sequential slicing: it would re-run __init__)
        x_in, s_in = h, shape
        seq = list(blk.conv)
        if len(seq) == 4:                    # expand 1×1 → depthwise → project 1×1 → BN
            h, shape = _unit(units, h, shape, seq[0][0], seq[0][1], RELU6, training, save)
            dw = seq[1]
        else:                                # expand ratio 1: depthwise → project
            dw = seq[0]
        h, shape, u = _dw_fwd(h, shape, dw[0], dw[1], RELU6, training, save)
        units.append(u)
        h, shape = _unit(units, h, shape, seq[-2], seq[-1], 0, training, save,
                         res=x_in if blk.use_res_connect else None)
    last = m[-1]
    h, shape = _unit(units, h, shape, last[0], last[1], RELU6, training, save)
    return h, shape, ((units,) if save else None)


def _mobilenet_backward(m: MobileNetV2Features, st, dh, training, grads):
    (units,) = st
    i = len(units) - 1
    dh, _ = _unit_bwd(units[i], dh, grads, training, True, False)
    i -= 1
    for blk in reversed(list(m)[1:-1]):
        expand = len(blk.conv) == 4
        u_proj, u_dw = units[i], units[i - 1]
        u_exp = units[i - 2] if expand else None
        i -= 3 if expand else 2
        d_proj, dres = _unit_bwd(u_proj, dh, grads, training, True, blk.use_res_connect)
        d_dw = _dw_bwd(u_dw, d_proj.reshape(-1, d_proj.shape[-1]), grads, training)
        if expand:
            dx, _ = _unit_bwd(u_exp, d_dw.reshape(-1, d_dw.shape[-1]), grads, training, True, False, dx_acc=dres)
        else:
            dx = d_dw
            if dres is not None:
                K.copy2d(dres, dx.view(dres.shape), beta=1.0)
        dh = dx.reshape(-1, dx.shape[-1])
    _unit_bwd(units[0], dh, grads, training, False, False)        # stem: no pixel gradient
    return grads


_IMPL = {ResNet18Features: (_resnet_forward, _resnet_backward),
         MobileNetV2Features: (_mobilenet_forward, _mobilenet_backward)}


def unit_param_order(m):
    """Backward-production order of a per-frame CNN backbone's parameters (`_resnet_backward` /
    `_mobilenet_backward`: units last→first, per unit BN weight, BN bias, conv weight) — the layout of the
    data-parallel reducer's flat gradient buffer (cmhar.dist)."""
    order = []

    def unit(conv, bn):
        order.extend([bn.weight, bn.bias, conv.weight])
    if isinstance(m, ResNet18Features):
        for layer in reversed(list(m)[4:8]):
            for blk in reversed(list(layer)):
                unit(blk.conv2, blk.bn2)
                if blk.downsample is not None:
                    unit(blk.downsample[0], blk.downsample[1])
                unit(blk.conv1, blk.bn1)
        unit(m[0], m[1])
    else:
        unit(m[-1][0], m[-1][1])
        for blk in reversed(list(m)[1:-1]):
            seq = list(blk.conv)
            unit(seq[-2], seq[-1])
            dw = seq[1] if len(seq) == 4 else seq[0]
            unit(dw[0], dw[1])
            if len(seq) == 4:
                unit(seq[0][0], seq[0][1])
        unit(m[0][0], m[0][1])
    return order


def _pool(h, shape, dev):
    N, _, Ho, Wo, Cf = shape
    feat = torch.empty(N, Cf, dtype=torch.float32, device=dev)
    call('cmhar_avgpool_cl', L.dtype_code(h.dtype), N, Ho * Wo, Cf, ptr(h), ptr(feat), L.stream(dev))
    return feat


class _CNNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, video, module, training, *params):
        fwd, _ = _IMPL[type(module)]
        h, shape, st = fwd(module, video.contiguous().float(), training, save=True)
        ctx.module, ctx.st, ctx.shape, ctx.training, ctx.dt = module, st, shape, training, h.dtype
        return _pool(h, shape, video.device)

    @staticmethod
    def backward(ctx, dfeat):
        m = ctx.module
        N, _, Ho, Wo, Cf = ctx.shape
        dh = torch.empty(N * Ho * Wo, Cf, dtype=ctx.dt, device=dfeat.device)
        call('cmhar_avgpool_cl_bwd', L.dtype_code(ctx.dt), N, Ho * Wo, Cf, ptr(dfeat.contiguous()), ptr(dh),
             L.stream(dfeat.device))
        _, bwd = _IMPL[type(m)]
        from .grads import AutogradSink
        sink = getattr(m, '_grad_sink', None) or AutogradSink()
        bwd(m, ctx.st, dh, ctx.training, sink)
        ctx.st = None
        return (None, None, None, *[sink.result(p) if p.requires_grad else None for p in m.parameters()])


def run_cnn2d(m, video: torch.Tensor, training: bool) -> torch.Tensor:
    """video (B, T, C, H, W) fp32 on the GPU → (B·T, feature_dim) fp32 per-frame pooled features
    (`adaptive_avg_pool2d(backbone(x.view(B·T, C, H, W)), 1)`, models.py:208-210), autograd-aware."""
    if not video.is_cuda:
        raise RuntimeError(f'{type(m).__name__} runs on the cmhar HIP library: move the module and input to the GPU')
    if m.compute_dtype not in ('bf16', 'fp32'):
        raise ValueError(f'{type(m).__name__}: compute_dtype bf16 or fp32')
    params = list(m.parameters())
    if torch.is_grad_enabled() and any(p.requires_grad for p in params):
        return _CNNFn.apply(video, m, training, *params)
    fwd, _ = _IMPL[type(m)]
    h, shape, _ = fwd(m, video.contiguous().float(), training, save=False)
    return _pool(h, shape, video.device)
