"""ORACLE — test infrastructure only.  CPU fp32 restatement of the reference's pretraining hot path.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import this module, and only
as the checker / the timed CPU baseline.  The product path (`cmhar.*`) never imports it: the HIP library is
the only compute path and fails loudly when it is missing.

What it restates (functional, torch-eager fp32 on CPU, parameters taken from a reference-shaped state_dict):

* `imu_encoder`            — `src/models/models.py:16-132` (PatchEmbedding + IMUEncoder, incl. the
                             pos-table truncation at `:122-123` that keeps only CLS + channel-0 patches),
                             with `nn.TransformerEncoderLayer` post-LN semantics
                             (third-party torch `nn/modules/transformer.py`: x = norm1(x + sa(x));
                             x = norm2(x + ff(x)); ReLU; eps 1e-5).
* `videomae`               — third-party transformers `models/videomae/modeling_videomae.py`
                             (`:80-124` sinusoid table + tubelet Conv3d, `:209-358` pre-LN block,
                             `:398-466` model; LN eps 1e-12, erf-GELU, no final LN when use_mean_pooling).
* `video_encoder`          — `models.py:185-203` (token 0 of `last_hidden_state`, then `projection`).
* `projection_head`        — `models.py:221-234` (Linear → BatchNorm1d → ReLU → Linear).
* `crossmodal`             — `models.py:270-291` (+ `F.normalize(dim=1)`, eps 1e-12).
* `siglip_loss`            — `src/models/losses.py:25-54`, written literally (BCE-with-logits on
                             logits·labels vs (labels+1)/2) so the reference's degeneracy is reproduced.
* `imu_classifier`         — `models.py:296-348`.
* `adamw_step`/`clip_grad_norm` — torch.optim.AdamW / clip_grad_norm_ algorithms as used at
                             `src/train/trainer.py:74-78,138-141`.

Parity status: pinned against golden vectors produced by importing the reference itself
(`tests/golden/make_golden.py`, fixtures `tests/golden/*.npz`, checked by `tests/test_oracle_golden.py`).
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Tuple

import numpy as np
import torch
import torch.nn.functional as F

Tensor = torch.Tensor


# ----------------------------------------------------------------------------------------------------------
# IMU encoder  (models.py:16-132)
# ----------------------------------------------------------------------------------------------------------
def _dropout(x: Tensor, p: float, training: bool, gen: Optional[torch.Generator]) -> Tensor:
    if not training or p == 0.0:
        return x
    keep = (torch.rand(x.shape, generator=gen) >= p).to(x.dtype)
    return x * keep / (1.0 - p)


def imu_encoder(sd: Dict[str, Tensor], x: Tensor, *, patch_size: int, stride: int, nhead: int,
                num_layers: int, dropout: float = 0.0, training: bool = False,
                gen: Optional[torch.Generator] = None, prefix: str = 'imu_encoder.') -> Tuple[Tensor, Tensor]:
    """Returns (cls (B,D), encoded (B,1+N',D)) — models.py:100-132."""
    B, C, L = x.shape
    patches = x.unfold(2, patch_size, stride)                       # (B,C,N,P)   models.py:40
    emb = [F.linear(patches[:, c], sd[f'{prefix}patch_embed.projections.{c}.weight'],
                    sd[f'{prefix}patch_embed.projections.{c}.bias']) for c in range(C)]   # models.py:45-47
    emb = torch.stack(emb, 1)                                        # (B,C,N,D)
    _, _, N, D = emb.shape
    tokens = torch.cat([sd[f'{prefix}cls_token'].expand(B, -1, -1), emb.reshape(B, C * N, D)], 1)
    pos = sd[f'{prefix}pos_encoding']
    pos_len = min(tokens.shape[1], pos.shape[1])                     # models.py:122-123
    h = tokens[:, :pos_len] + pos[:, :pos_len]
    dh = D // nhead
    for i in range(num_layers):
        p = f'{prefix}transformer.layers.{i}.'
        # self-attention block (torch MultiheadAttention, batch_first)
        qkv = F.linear(h, sd[p + 'self_attn.in_proj_weight'], sd[p + 'self_attn.in_proj_bias'])
        q, k, v = qkv.split(D, dim=-1)
        T = h.shape[1]
        q = q.reshape(B, T, nhead, dh).transpose(1, 2)
        k = k.reshape(B, T, nhead, dh).transpose(1, 2)
        v = v.reshape(B, T, nhead, dh).transpose(1, 2)
        att = torch.softmax((q @ k.transpose(-1, -2)) / math.sqrt(dh), dim=-1)
        att = _dropout(att, dropout, training, gen)
        o = (att @ v).transpose(1, 2).reshape(B, T, D)
        o = F.linear(o, sd[p + 'self_attn.out_proj.weight'], sd[p + 'self_attn.out_proj.bias'])
        h = F.layer_norm(h + _dropout(o, dropout, training, gen), (D,), sd[p + 'norm1.weight'],
                         sd[p + 'norm1.bias'], 1e-5)
        f = F.relu(F.linear(h, sd[p + 'linear1.weight'], sd[p + 'linear1.bias']))
        f = F.linear(_dropout(f, dropout, training, gen), sd[p + 'linear2.weight'], sd[p + 'linear2.bias'])
        h = F.layer_norm(h + _dropout(f, dropout, training, gen), (D,), sd[p + 'norm2.weight'],
                         sd[p + 'norm2.bias'], 1e-5)
    enc = F.layer_norm(h, (D,), sd[f'{prefix}norm.weight'], sd[f'{prefix}norm.bias'], 1e-5)  # models.py:127
    return enc[:, 0], enc


# ----------------------------------------------------------------------------------------------------------
# VideoMAE (third-party transformers modeling_videomae.py)
# ----------------------------------------------------------------------------------------------------------
def sinusoid_table(n_position: int, d_hid: int) -> Tensor:
    """Fixed sin-cos table (modeling_videomae.py:80-91): angle = pos / 10000^(2*(j//2)/d), computed in f64."""
    pos = np.arange(n_position, dtype=np.float64)[:, None]
    j = np.arange(d_hid)[None, :]
    ang = pos / np.power(10000, 2 * (j // 2) / d_hid)
    tab = np.empty_like(ang)
    tab[:, 0::2] = np.sin(ang[:, 0::2])
    tab[:, 1::2] = np.cos(ang[:, 1::2])
    return torch.from_numpy(tab.astype(np.float32))


class _Round(torch.autograd.Function):
    """bf16 storage of a tensor: round-to-nearest-even of the forward value (`fwd`) and/or of the gradient that
    flows back into it (`bwd`), both kept in fp32."""

    @staticmethod
    def forward(ctx, x, fwd, bwd):
        ctx.bwd = bwd
        return x.bfloat16().float() if fwd else x.clone()

    @staticmethod
    def backward(ctx, g):
        return (g.bfloat16().float() if ctx.bwd else g), None, None


def _rq(x, fwd=True, bwd=True):
    return _Round.apply(x, fwd, bwd)


def _bf(x):
    return x.bfloat16().float()


class _FlashBF16(torch.autograd.Function):
    """Flash attention with bf16 MFMA operands (csrc/attention.hip): fp32 scores and softmax statistics, the
    probabilities rounded to bf16 before P·V (forward) and Pᵀ·dO (backward), dS rounded to bf16 before dS·K and
    dSᵀ·Q; δ = rowsum(dO ∘ O) from the bf16-stored O.  q, k, v: (B, H, L, D) bf16-valued fp32 tensors."""

    @staticmethod
    def forward(ctx, q, k, v, scale):
        s = (q @ k.transpose(-1, -2)) * scale
        m = s.amax(-1, keepdim=True)
        p = torch.exp(s - m)
        l = p.sum(-1, keepdim=True)
        o = (_bf(p) @ v) / l
        ctx.save_for_backward(q, k, v, o, m + l.log())
        ctx.scale = scale
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        scale = ctx.scale
        p = torch.exp((q @ k.transpose(-1, -2)) * scale - lse)
        dv = _bf(p).transpose(-1, -2) @ do
        dp = do @ v.transpose(-1, -2)
        delta = (do * _bf(o)).sum(-1, keepdim=True)
        ds = _bf(p * (dp - delta))
        dq = (ds @ k) * scale
        dk = (ds.transpose(-1, -2) @ q) * scale
        return dq, dk, dv, None


class _GeluBF16(torch.autograd.Function):
    """The FC1 epilogue of the bf16 path: stores bf16(gelu(a)) and bf16(gelu'(a)); the FC2 dgrad epilogue forms
    dpre = bf16(dY·W2 ∘ gelu'_bf16)."""

    @staticmethod
    def forward(ctx, a):
        ad = a.double()
        cdf = 0.5 * (1.0 + torch.erf(ad / math.sqrt(2.0)))
        pdf = torch.exp(-0.5 * ad * ad) / math.sqrt(2.0 * math.pi)
        ctx.save_for_backward(_bf((cdf + ad * pdf).float()))
        return _bf((ad * cdf).float())

    @staticmethod
    def backward(ctx, g):
        (gp,) = ctx.saved_tensors
        return _bf(g * gp)


def videomae(sd: Dict[str, Tensor], video: Tensor, *, num_heads: int, patch_size: int = 16, tubelet: int = 2,
             eps: float = 1e-12, use_mean_pooling: bool = True,
             prefix: str = 'video_encoder.backbone.', bf16: bool = False) -> Tensor:
    """last_hidden_state (B, L, Hd) of VideoMAEModel (modeling_videomae.py:398-466).

    `bf16=True` restates the HIP bf16 throughput path's STORAGE (not the reference): bf16 weight shadows, bf16
    video columns, every activation the path stores in bf16 (residual stream, LN outputs, Q/K/V with the keys
    pre-scaled by scale·log2(e), attention output, GELU output and GELU'), every stored gradient (dx, dh, dQKV, dO,
    dpre), and the flash kernels' bf16 P / dS operands; accumulation, softmax statistics and LayerNorm stay
    fp32.  Its distance to the fp32 run is the error bf16 storage itself causes — the bound the bf16 parity tests
    scale (tests/test_models_gpu.py)."""
    rw = (lambda t: _rq(t, True, False)) if bf16 else (lambda t: t)        # weight shadows: straight-through
    rq = _rq if bf16 else (lambda t, *a: t)
    w = sd[prefix + 'embeddings.patch_embeddings.projection.weight']
    hd = w.shape[0]
    x = video.permute(0, 2, 1, 3, 4)                                 # (B,C,T,H,W)  :165
    if bf16:
        x = _bf(x)
    emb = F.conv3d(x, rw(w), sd[prefix + 'embeddings.patch_embeddings.projection.bias'],
                   stride=(tubelet, patch_size, patch_size))
    emb = emb.flatten(2).transpose(1, 2)                             # (B,L,Hd)     :166
    h = rq(emb + sinusoid_table(emb.shape[1], hd)[None])             # :109-117
    B, L, _ = h.shape
    dh = hd // num_heads
    i = 0
    while f'{prefix}encoder.layer.{i}.layernorm_before.weight' in sd:
        p = f'{prefix}encoder.layer.{i}.'
        n = rq(F.layer_norm(h, (hd,), sd[p + 'layernorm_before.weight'], sd[p + 'layernorm_before.bias'], eps))
        def proj(name):
            return F.linear(n, rw(sd[p + f'attention.attention.{name}.weight']),
                            sd.get(p + f'attention.attention.{name}.bias')).reshape(B, L, num_heads, dh).transpose(1, 2)
        if bf16:
            c = dh ** -0.5 * math.log2(math.e)
            q, k, v = rq(proj('query')), rq(proj('key')), rq(proj('value'))
            k = _rq(k * c, True, False) / c                           # K' = bf16(c·K); dK of the unscaled key
            o = rq(_FlashBF16.apply(q, k, v, dh ** -0.5))
        else:
            q, k, v = proj('query'), proj('key'), proj('value')
            att = torch.softmax((q @ k.transpose(-1, -2)) * dh ** -0.5, dim=-1)
            o = att @ v
        o = o.transpose(1, 2).reshape(B, L, hd)
        o = F.linear(o, rw(sd[p + 'attention.output.dense.weight']), sd[p + 'attention.output.dense.bias'])
        h = rq(h + o)
        n2 = rq(F.layer_norm(h, (hd,), sd[p + 'layernorm_after.weight'], sd[p + 'layernorm_after.bias'], eps))
        a = F.linear(n2, rw(sd[p + 'intermediate.dense.weight']), sd[p + 'intermediate.dense.bias'])
        f = _GeluBF16.apply(a) if bf16 else F.gelu(a)
        h = rq(h + F.linear(f, rw(sd[p + 'output.dense.weight']), sd[p + 'output.dense.bias']))
        i += 1
    if not use_mean_pooling:
        h = rq(F.layer_norm(h, (hd,), sd[prefix + 'layernorm.weight'], sd[prefix + 'layernorm.bias'], eps))
    return h


def video_encoder(sd, video, *, num_heads, patch_size=16, tubelet=2, eps=1e-12, use_mean_pooling=True,
                  prefix='video_encoder.', bf16=False):
    """models.py:197-203: token 0 of last_hidden_state → projection (`bf16`: see `videomae`)."""
    h = videomae(sd, video, num_heads=num_heads, patch_size=patch_size, tubelet=tubelet, eps=eps,
                 use_mean_pooling=use_mean_pooling, prefix=prefix + 'backbone.', bf16=bf16)
    return F.linear(h[:, 0], sd[prefix + 'projection.weight'], sd[prefix + 'projection.bias'])


# ----------------------------------------------------------------------------------------------------------
# Heads, model, loss
# ----------------------------------------------------------------------------------------------------------
def batch_norm(x: Tensor, sd: Dict[str, Tensor], p: str, training: bool, momentum: float = 0.1,
               eps: float = 1e-5, update_stats: bool = True) -> Tensor:
    """nn.BatchNorm1d: batch statistics in train mode (biased var to normalise, unbiased var into the
    running buffer), running statistics in eval mode."""
    if training:
        if x.shape[0] <= 1:
            raise ValueError('Expected more than 1 value per channel when training')
        mean = x.mean(0)
        var = x.var(0, unbiased=False)
        if update_stats:
            with torch.no_grad():
                n = x.shape[0]
                sd[p + 'running_mean'].mul_(1 - momentum).add_(momentum * mean.detach())
                sd[p + 'running_var'].mul_(1 - momentum).add_(momentum * var.detach() * n / (n - 1))
                sd[p + 'num_batches_tracked'].add_(1)
        return (x - mean) / torch.sqrt(var + eps) * sd[p + 'weight'] + sd[p + 'bias']
    return (x - sd[p + 'running_mean']) / torch.sqrt(sd[p + 'running_var'] + eps) * sd[p + 'weight'] + sd[p + 'bias']


def projection_head(sd, x, prefix, training, update_stats=True):
    """models.py:221-234."""
    h = F.linear(x, sd[prefix + 'net.0.weight'], sd[prefix + 'net.0.bias'])
    h = F.relu(batch_norm(h, sd, prefix + 'net.1.', training, update_stats=update_stats))
    return F.linear(h, sd[prefix + 'net.3.weight'], sd[prefix + 'net.3.bias'])


def l2_normalize(x: Tensor, eps: float = 1e-12) -> Tensor:
    return x / x.norm(dim=1, keepdim=True).clamp_min(eps)


def crossmodal(sd, imu, video, mcfg, training=True, imu_dropout=0.0, gen=None, update_stats=True, bf16=False):
    """models.py:270-291 → (imu_proj, video_proj) unit rows (`bf16`: the video backbone with the HIP bf16 path's
    storage emulated, see `videomae`)."""
    cls, _ = imu_encoder(sd, imu, patch_size=mcfg['imu_patch_size'], stride=mcfg['imu_stride'],
                         nhead=mcfg['imu_nhead'], num_layers=mcfg['imu_num_layers'], dropout=imu_dropout,
                         training=training, gen=gen)
    vf = video_encoder(sd, video, num_heads=mcfg['video_num_heads'], patch_size=mcfg.get('video_patch_size', 16),
                       tubelet=mcfg.get('video_tubelet', 2), eps=mcfg.get('video_eps', 1e-12),
                       use_mean_pooling=mcfg.get('video_use_mean_pooling', True), bf16=bf16)
    a = projection_head(sd, cls, 'imu_proj.', training, update_stats)
    b = projection_head(sd, vf, 'video_proj.', training, update_stats)
    return l2_normalize(a), l2_normalize(b)


def siglip_loss(a: Tensor, b: Tensor, log_t: Tensor, bias: Tensor) -> Tensor:
    """losses.py:34-52, literally."""
    n = a.shape[0]
    logits = (a @ b.T) * log_t.exp() + bias
    labels = 2 * torch.eye(n) - 1
    return F.binary_cross_entropy_with_logits(logits * labels, (labels + 1) / 2, reduction='mean')


def imu_classifier(sd, imu, mcfg, training=False, update_stats=True, prefix=''):
    """models.py:328-339 with the classifier Sequential (Linear, BN, ReLU, Dropout) × len(hidden) → Linear."""
    cls, _ = imu_encoder(sd, imu, patch_size=mcfg['imu_patch_size'], stride=mcfg['imu_stride'],
                         nhead=mcfg['imu_nhead'], num_layers=mcfg['imu_num_layers'], dropout=0.0,
                         training=False, prefix=prefix + 'imu_encoder.')
    h = cls
    idx = 0
    for _ in mcfg['classifier_hidden_dims']:
        h = F.linear(h, sd[f'{prefix}classifier.{idx}.weight'], sd[f'{prefix}classifier.{idx}.bias'])
        h = F.relu(batch_norm(h, sd, f'{prefix}classifier.{idx + 1}.', training, update_stats=update_stats))
        idx += 4
    return F.linear(h, sd[f'{prefix}classifier.{idx}.weight'], sd[f'{prefix}classifier.{idx}.bias'])


# ----------------------------------------------------------------------------------------------------------
# Optimiser pieces (torch.optim.AdamW defaults + clip_grad_norm_, trainer.py:74-78,138-141)
# ----------------------------------------------------------------------------------------------------------
def clip_grad_norm(grads, max_norm: float = 1.0, eps: float = 1e-6):
    total = torch.sqrt(sum((g.double() ** 2).sum() for g in grads if g is not None)).float()
    coef = max_norm / (total + eps)
    if coef < 1.0:
        for g in grads:
            if g is not None:
                g.mul_(coef)
    return total


def adamw_step(params, grads, exp_avg, exp_avg_sq, step: int, lr: float, betas=(0.9, 0.999), eps=1e-8,
               weight_decay=0.01):
    """One torch.optim.AdamW step (non-amsgrad); params with grad None are skipped."""
    b1, b2 = betas
    for p, g, m, v in zip(params, grads, exp_avg, exp_avg_sq):
        if g is None:
            continue
        p.mul_(1 - lr * weight_decay)
        m.lerp_(g, 1 - b1)
        v.mul_(b2).addcmul_(g, g, value=1 - b2)
        bc1 = 1 - b1 ** step
        bc2 = 1 - b2 ** step
        denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
        p.addcdiv_(m, denom, value=-lr / bc1)


# ----------------------------------------------------------------------------------------------------------
# Cross-entropy family (losses.py:57-150; nn.CrossEntropyLoss of ClassificationTrainer, trainer.py:249,300)
# ----------------------------------------------------------------------------------------------------------
def _log_softmax(z: Tensor) -> Tensor:
    m = z.max(dim=1, keepdim=True).values
    return z - (m + (z - m).exp().sum(dim=1, keepdim=True).log())


def _reduce(v: Tensor, reduction: str) -> Tensor:
    return v.mean() if reduction == 'mean' else v.sum() if reduction == 'sum' else v


def cross_entropy(z: Tensor, y: Tensor, reduction: str = 'mean', label_smoothing: float = 0.0) -> Tensor:
    """F.cross_entropy with class-index targets (mean over rows) and optional label smoothing
    (q = (1-eps)·onehot + eps/C), restated from log-softmax."""
    lp = _log_softmax(z)
    C = z.shape[1]
    nll = -lp.gather(1, y.view(-1, 1)).squeeze(1)
    v = (1 - label_smoothing) * nll + label_smoothing * (-lp.sum(dim=1) / C)
    return _reduce(v, reduction)


def focal_loss(z: Tensor, y: Tensor, alpha: float = 1.0, gamma: float = 2.0, reduction: str = 'mean') -> Tensor:
    """losses.py:101-116: alpha·(1 - exp(-ce))^gamma·ce."""
    ce = cross_entropy(z, y, 'none')
    return _reduce(alpha * (1 - torch.exp(-ce)) ** gamma * ce, reduction)


def label_smoothing_ce(z: Tensor, y: Tensor, epsilon: float = 0.1, reduction: str = 'mean') -> Tensor:
    """losses.py:129-150."""
    return cross_entropy(z, y, reduction, label_smoothing=epsilon)


def info_nce(a: Tensor, b: Tensor, temperature: float = 0.07) -> Tensor:
    """losses.py:67-87: symmetric CE over a·bᵀ/τ with diagonal targets."""
    s = a @ b.T / temperature
    y = torch.arange(a.shape[0])
    return (cross_entropy(s, y) + cross_entropy(s.T, y)) / 2
