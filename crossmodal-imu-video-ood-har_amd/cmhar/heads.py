"""MLP heads on the cmhar HIP library: ProjectionHead (`src/models/models.py:221-234`), the IMUClassifier head
(`models.py:311-322`) and F.normalize (`models.py:288-289`).

A head is a chain [Linear → BatchNorm1d → ReLU (→ Dropout)]* → Linear over a (B, C) fp32 batch.  The whole chain
is one autograd node: fp32 GEMMs with bias epilogues, a fused BatchNorm1d+ReLU kernel that also updates the
running statistics / num_batches_tracked in place (train mode: batch statistics, momentum 0.1, unbiased running
variance), and counter-hash dropout.  Parameter containers are the reference's own torch modules, so
`state_dict()` keys (`net.0/1/3`, `classifier.0/1/4/5/8`) and initialisation are unchanged.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import kernels as K
from ._lib import NoReplicate


def _blocks(seq: nn.Sequential):
    """Parse a Sequential of (Linear, BN, ReLU, [Dropout])* Linear into ([(lin, bn, p)], final_lin)."""
    mods = list(seq)
    blocks, i = [], 0
    while i < len(mods) - 1:
        lin, bn, act = mods[i], mods[i + 1], mods[i + 2]
        if not (isinstance(lin, nn.Linear) and isinstance(bn, nn.BatchNorm1d) and isinstance(act, nn.ReLU)):
            raise TypeError('unsupported head structure')
        p, step = 0.0, 3
        if i + 3 < len(mods) and isinstance(mods[i + 3], nn.Dropout):
            p, step = mods[i + 3].p, 4
        blocks.append((lin, bn, p))
        i += step
    if not isinstance(mods[-1], nn.Linear):
        raise TypeError('head must end with a Linear')
    return blocks, mods[-1]


class _Seeds:
    def __init__(self):
        self.n = 0

    def next(self):
        self.n += 1
        return (0x5DEECE66D * self.n + 0xB) & ((1 << 62) - 1)


def bn_momentum(bn, updating: bool) -> float:
    """The running-statistics factor torch's _BatchNorm.forward uses: `momentum`, or with momentum=None the
    cumulative moving average 1 / num_batches_tracked (counted after this batch's increment; one host read)."""
    if bn.momentum is not None:
        return float(bn.momentum)
    if not updating or bn.num_batches_tracked is None:
        return 0.0
    return 1.0 / float(int(bn.num_batches_tracked.item()) + 1)


def _head_forward(seq, x, training, seed, save):
    blocks, final = _blocks(seq)
    h = x
    saved = []
    for bi, (lin, bn, p) in enumerate(blocks):
        z = K.linear(h, lin.weight, lin.bias)
        upd = training and bn.track_running_stats and bn.running_mean is not None
        use_batch = training or not bn.track_running_stats
        y, sm, sr = K.batchnorm_fwd(z, bn.weight, bn.bias, bn.running_mean if upd or not use_batch else None,
                                    bn.running_var if upd or not use_batch else None, use_batch,
                                    bn_momentum(bn, upd), bn.eps, True,
                                    bn.num_batches_tracked if upd else None)
        pd = p if training else 0.0
        if pd > 0:
            yd = torch.empty_like(y)
            K.copy2d(y, yd, pdrop=pd, seed=seed + bi)
        else:
            yd = y
        if save:
            saved.append((h, z, y, sm, sr, pd, use_batch))
        h = yd
    out = K.linear(h, final.weight, final.bias)
    return out, (saved, h)


def _head_backward(seq, st, dout, seed):
    blocks, final = _blocks(seq)
    saved, hlast = st
    grads = {final.weight: K.linear_wgrad(dout, hlast), final.bias: K.colsum(dout)}
    dh = K.linear_dgrad(dout, final.weight)
    for bi in reversed(range(len(blocks))):
        lin, bn, _ = blocks[bi]
        h, z, y, sm, sr, pd, use_batch = saved[bi]
        if pd > 0:
            K.copy2d(dh, dh, pdrop=pd, seed=seed + bi)
        dz, dgw, dgb = K.batchnorm_bwd(z, y, dh, bn.weight, sm, sr, use_batch, True)
        grads[bn.weight], grads[bn.bias] = dgw, dgb
        grads[lin.weight] = K.linear_wgrad(dz, h)
        grads[lin.bias] = K.colsum(dz)
        dh = K.linear_dgrad(dz, lin.weight)
    return dh, grads


class _HeadFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, seq, training, seed, *params):
        out, st = _head_forward(seq, x, training, seed, save=True)
        ctx.seq, ctx.st, ctx.seed, ctx.params = seq, st, seed, params
        return out

    @staticmethod
    def backward(ctx, dout):
        dx, grads = _head_backward(ctx.seq, ctx.st, dout.contiguous(), ctx.seed)
        ctx.st = None
        return (dx, None, None, None) + tuple(grads.get(p) if p.requires_grad else None for p in ctx.params)


def run_head(seq: nn.Sequential, x: torch.Tensor, training: bool, seeds: _Seeds) -> torch.Tensor:
    if training and x.shape[0] <= 1:
        raise ValueError(f'Expected more than 1 value per channel when training, got input size {tuple(x.shape)}')
    x = x.contiguous().float()
    params = [p for p in seq.parameters()]
    has_drop = any(isinstance(m, nn.Dropout) and m.p > 0 for m in seq)
    seed = seeds.next() if (training and has_drop) else 0
    if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in params)):
        return _HeadFn.apply(x, seq, training, seed, *params)
    with torch.no_grad():
        return _head_forward(seq, x, training, seed, save=False)[0]


class ProjectionHead(NoReplicate, nn.Module):
    """models.py:221-234: Linear → BatchNorm1d → ReLU → Linear."""

    def __init__(self, in_dim, hidden_dim, out_dim):
        super().__init__()
        self.net = nn.Sequential(
            nn.Linear(in_dim, hidden_dim),
            nn.BatchNorm1d(hidden_dim),
            nn.ReLU(inplace=True),
            nn.Linear(hidden_dim, out_dim),
        )
        self._seeds = _Seeds()

    def forward(self, x):
        return run_head(self.net, x, self.training, self._seeds)


class _L2NormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, eps):
        y, n = K.l2normalize_fwd(x, eps)
        ctx.save_for_backward(y, n)
        ctx.eps = eps
        return y

    @staticmethod
    def backward(ctx, dy):
        y, n = ctx.saved_tensors
        return K.l2normalize_bwd(y, dy, n, ctx.eps), None


def l2_normalize(x: torch.Tensor, eps: float = 1e-12) -> torch.Tensor:
    """F.normalize(x, dim=1) for (B, C) fp32 device tensors."""
    x = x.contiguous().float()
    if torch.is_grad_enabled() and x.requires_grad:
        return _L2NormFn.apply(x, eps)
    return K.l2normalize_fwd(x, eps)[0]
