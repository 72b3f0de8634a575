"""ORACLE — test infrastructure only.  CPU fp32 restatement of the cross-attention fusion (north_star extension).

Only `tests/` may import this module, as the checker.  Parity unpinned w.r.t. the reference: the reference has no
fusion module (its encoders only meet in the SigLIP loss, `src/models/models.py:239-291`), so this restates the
build's own definition (`cmhar/fusion.py`) with plain torch ops on a state_dict of that module:
q = Wq·imu, [k|v] = Wkv·video, h = LayerNorm(Wr·imu + Wo·MHA(q, k, v)) (eps 1e-5), fused = mean over IMU tokens,
logits = Wc·fused.

`bf16=True` restates the bf16 path's STORAGE (not a reference behaviour): the video tokens and the K|V weights as the
bf16 GEMM operands, q / [k|v] / the attention output stored in bf16 (and the gradients stored into them), the flash
kernel's bf16 P / dS operands (`cpu_model._FlashBF16`); the IMU-side GEMMs, LayerNorm, mean and classifier stay fp32.
Its distance to the fp32 run bounds the bf16 path's error (tests/test_fusion_gpu.py).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from .cpu_model import _FlashBF16, _rq


def fusion_forward(sd, imu_tokens, video_tokens, num_heads, eps=1e-5, prefix='', bf16=False):
    p = prefix
    rq = _rq if bf16 else (lambda t, *a: t)                        # stored bf16: value and incoming gradient
    rf = (lambda t: _rq(t, True, False)) if bf16 else (lambda t: t)  # bf16 GEMM operand over an fp32 tensor
    B, Lq, _ = imu_tokens.shape
    Lk = video_tokens.shape[1]
    d = sd[p + 'q_proj.weight'].shape[0]
    D = d // num_heads
    q = rq(F.linear(imu_tokens, sd[p + 'q_proj.weight'], sd[p + 'q_proj.bias']))
    kv = rq(F.linear(rf(video_tokens), rf(sd[p + 'kv_proj.weight']), sd[p + 'kv_proj.bias']))
    k, v = kv[..., :d], kv[..., d:]
    q = q.view(B, Lq, num_heads, D).transpose(1, 2)
    k = k.reshape(B, Lk, num_heads, D).transpose(1, 2)
    v = v.reshape(B, Lk, num_heads, D).transpose(1, 2)
    if bf16:
        a = _FlashBF16.apply(q, k, v, 1.0 / math.sqrt(D))
    else:
        a = torch.softmax(q @ k.transpose(-1, -2) / math.sqrt(D), dim=-1) @ v
    a = rq(a.transpose(1, 2).reshape(B, Lq, d))
    h = F.linear(imu_tokens, sd[p + 'res_proj.weight'], sd[p + 'res_proj.bias']) + \
        F.linear(a, sd[p + 'out_proj.weight'], sd[p + 'out_proj.bias'])
    y = F.layer_norm(h, (d,), sd[p + 'norm.weight'], sd[p + 'norm.bias'], eps)
    fused = y.mean(dim=1)
    return F.linear(fused, sd[p + 'classifier.weight'], sd[p + 'classifier.bias']), fused
