"""ORACLE — test infrastructure only.  CPU fp32 restatement of the R3D-18 video backbone (north_star extension).

Only `tests/` may import this module, as the checker.  Parity unpinned w.r.t. the reference: the reference has no
3-D CNN (its CNN options are per-frame 2-D torchvision models, `src/models/models.py:160-216`) and torchvision is
not installed here, so this restates torchvision `models/video/resnet.py` (VideoResNet with BasicStem,
Conv3DSimple, BasicBlock [2, 2, 2, 2]; BN3d eps 1e-5, momentum 0.1; AdaptiveAvgPool3d(1)) functionally with
`F.conv3d` / `F.batch_norm` on parameters taken from a `cmhar.r3d.R3D18` state_dict (same key names as torchvision).

`q` (optional): a rounding applied at every point where the HIP bf16 path stores a tensor in bf16 — the network input,
each conv output z (and, in the backward, dz), each BN/activation output y (and the gradient flowing into it) —
`bf16_storage` emulates that storage in the fp32 restatement.  `qw` (optional): the rounding of the conv weights the
HIP bf16 path multiplies (`cmhar/r3d.py` `_pack` / `_pack_stem` / `_pack_flip` write bf16 packs; the weight gradient
itself is accumulated and stored in fp32, so `bf16_weight` rounds the forward value only).  `BF16` holds both hooks.  It separates the error bf16 storage itself causes
(ill-conditioned gradients amplify it) from any kernel error (tests/test_r3d_gpu.py, tests/test_cnn2d_gpu.py).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


class _RoundBF16(torch.autograd.Function):
    """Forward value and backward gradient both rounded to bf16 (round-to-nearest-even), kept in fp32."""

    @staticmethod
    def forward(ctx, x):
        return x.bfloat16().float()

    @staticmethod
    def backward(ctx, g):
        return g.bfloat16().float()


def bf16_storage(x):
    return _RoundBF16.apply(x)


class _RoundFwdBF16(torch.autograd.Function):
    """Forward value rounded to bf16, gradient passed through unrounded (a bf16 weight pack over an fp32 master)."""

    @staticmethod
    def forward(ctx, x):
        return x.bfloat16().float()

    @staticmethod
    def backward(ctx, g):
        return g


def bf16_weight(x):
    return _RoundFwdBF16.apply(x)


BF16 = dict(q=bf16_storage, qw=bf16_weight)


def _id(x):
    return x


def _bn(x, sd, pre, training, stats):
    rm, rv = sd[pre + 'running_mean'].clone(), sd[pre + 'running_var'].clone()
    y = F.batch_norm(x, rm, rv, sd[pre + 'weight'], sd[pre + 'bias'], training=training, momentum=0.1, eps=1e-5)
    stats[pre] = (rm, rv)
    return y


def r3d18_features(sd, video_bcthw, training=True, stats=None, q=None, qw=None, trace=None):
    """video (B, 3, T, H, W) fp32 → pooled (B, 512).  `stats` collects updated running (mean, var) per BN prefix;
    `q` / `qw` mark the bf16 storage points / bf16 weight packs of the HIP path (module docstring); `trace` (a list)
    collects (conv output z, unit output y) per conv unit in the HIP path's unit order (stem, then per block conv1,
    downsample, conv2) for per-layer comparisons."""
    stats = {} if stats is None else stats
    q = q or _id
    qw = qw or _id
    tr = trace.append if trace is not None else (lambda t: None)
    z = q(F.conv3d(q(video_bcthw), qw(sd['stem.0.weight']), stride=(1, 2, 2), padding=(1, 3, 3)))
    x = q(F.relu(_bn(z, sd, 'stem.1.', training, stats)))
    tr((z, x))
    for li in range(1, 5):
        for bi in range(2):
            p = f'layer{li}.{bi}.'
            stride = 2 if (li > 1 and bi == 0) else 1
            z1 = q(F.conv3d(x, qw(sd[p + 'conv1.0.weight']), stride=stride, padding=1))
            h = q(F.relu(_bn(z1, sd, p + 'conv1.1.', training, stats)))
            tr((z1, h))
            z2 = q(F.conv3d(h, qw(sd[p + 'conv2.0.weight']), stride=1, padding=1))
            h = _bn(z2, sd, p + 'conv2.1.', training, stats)
            if p + 'downsample.0.weight' in sd:
                zd = q(F.conv3d(x, qw(sd[p + 'downsample.0.weight']), stride=stride))
                idn = q(_bn(zd, sd, p + 'downsample.1.', training, stats))
                tr((zd, idn))
            else:
                idn = x
            x = q(F.relu(h + idn))
            tr((z2, x))
    return x.mean(dim=(2, 3, 4))
