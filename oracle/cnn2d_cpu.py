"""ORACLE — test infrastructure only.  CPU fp32 restatement of the reference VideoEncoder's per-frame CNN branch.

Only `tests/` may import this module, as the checker.  The reference (`src/models/models.py:163-173,208-216`) builds
torchvision `resnet18(...).children()[:-2]` / `mobilenet_v2(...).features`, applies it to `x.view(B*T, C, H, W)`,
then `F.adaptive_avg_pool2d(fmap, 1)` → `view(B, T, F)` → `projection` (Linear F→d, per frame) → transpose →
`AdaptiveAvgPool1d(1)` over T.  torchvision is not installed here, so its two networks are restated functionally
(torchvision models/resnet.py BasicBlock [2, 2, 2, 2], MaxPool2d(3, 2, 1); models/mobilenetv2.py InvertedResidual
with the (t, c, n, s) table, Conv2dNormActivation = Conv2d + BN + ReLU6; BN eps 1e-5, momentum 0.1) with
`F.conv2d` / `F.batch_norm` / `F.max_pool2d` / `F.relu6` on parameters from a `cmhar.cnn2d` state_dict (torchvision
key names).  Parity unpinned w.r.t. the reference (no torchvision to import, no reference fixtures for this branch).
`q` (optional, e.g. `oracle.r3d_cpu.bf16_storage`) is applied where the HIP bf16 path stores tensors in bf16; `qw`
(optional, `oracle.r3d_cpu.bf16_weight`) to the dense conv weights, which that path multiplies as bf16 packs (the
depthwise kernels read the fp32 weights).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .r3d_cpu import _id

MOBILENET_V2_SETTING = [[1, 16, 1, 1], [6, 24, 2, 2], [6, 32, 3, 2], [6, 64, 4, 2], [6, 96, 3, 1], [6, 160, 3, 2],
                        [6, 320, 1, 1]]


def _bn(x, sd, pre, training, stats):
    rm, rv = sd[pre + 'running_mean'].clone(), sd[pre + 'running_var'].clone()
    y = F.batch_norm(x, rm, rv, sd[pre + 'weight'], sd[pre + 'bias'], training=training, momentum=0.1, eps=1e-5)
    stats[pre] = (rm, rv)
    return y


def resnet18_features(sd, frames, training=True, stats=None, q=None, qw=None):
    """frames (N, 3, H, W) → feature map (N, 512, h, w); sd keys as `nn.Sequential(*resnet18().children()[:-2])`."""
    stats = {} if stats is None else stats
    q = q or _id
    qw = qw or _id
    x = q(F.conv2d(q(frames), qw(sd['0.weight']), stride=2, padding=3))
    x = q(F.relu(_bn(x, sd, '1.', training, stats)))
    x = q(F.max_pool2d(x, 3, 2, 1))
    for li in range(4):
        for bi in range(2):
            p = f'{4 + li}.{bi}.'
            stride = 2 if (li > 0 and bi == 0) else 1
            h = q(F.relu(_bn(q(F.conv2d(x, qw(sd[p + 'conv1.weight']), stride=stride, padding=1)), sd, p + 'bn1.',
                             training, stats)))
            h = _bn(q(F.conv2d(h, qw(sd[p + 'conv2.weight']), padding=1)), sd, p + 'bn2.', training, stats)
            if p + 'downsample.0.weight' in sd:
                idn = q(_bn(q(F.conv2d(x, qw(sd[p + 'downsample.0.weight']), stride=stride)), sd, p + 'downsample.1.',
                            training, stats))
            else:
                idn = x
            x = q(F.relu(h + idn))
    return x


def mobilenet_v2_features(sd, frames, training=True, stats=None, q=None, qw=None):
    """frames (N, 3, H, W) → feature map (N, 1280, h, w); sd keys as `mobilenet_v2().features`."""
    stats = {} if stats is None else stats
    q = q or _id
    qw = qw or _id

    def cna(x, pre, stride=1, groups=1):
        w = sd[pre + '0.weight'] if groups > 1 else qw(sd[pre + '0.weight'])
        x = q(F.conv2d(x, w, stride=stride, padding=(w.shape[-1] - 1) // 2, groups=groups))
        return q(F.relu6(_bn(x, sd, pre + '1.', training, stats)))

    x = cna(q(frames), '0.', stride=2)
    cin, i = 32, 1
    for t, c, n, s in MOBILENET_V2_SETTING:
        for j in range(n):
            stride = s if j == 0 else 1
            p = f'{i}.conv.'
            h = x
            k = 0
            if t != 1:
                h = cna(h, f'{p}0.')
                k = 1
            hidden = cin * t
            h = cna(h, f'{p}{k}.', stride=stride, groups=hidden)
            h = q(F.conv2d(h, qw(sd[f'{p}{k + 1}.weight'])))
            h = _bn(h, sd, f'{p}{k + 2}.', training, stats)
            x = q(x + h if (stride == 1 and cin == c) else h)
            cin = c
            i += 1
    return cna(x, f'{i}.')


def video_encoder_cnn(sd, video, backbone, training=True, stats=None, q=None, qw=None):
    """models.py:208-216 on a whole `VideoEncoder` state_dict (keys `backbone.*`, `projection.*`):
    video (B, T, C, H, W) → (B, video_d_model)."""
    B, T, C, H, W = video.shape
    bsd = {k[len('backbone.'):]: v for k, v in sd.items() if k.startswith('backbone.')}
    f = resnet18_features if backbone == 'resnet18' else mobilenet_v2_features
    fmap = f(bsd, video.reshape(B * T, C, H, W), training, stats, q, qw)
    feats = F.adaptive_avg_pool2d(fmap, (1, 1)).squeeze(-1).squeeze(-1).view(B, T, -1)
    feats = F.linear(feats, sd['projection.weight'], sd['projection.bias'])
    return feats.transpose(1, 2).mean(-1)
