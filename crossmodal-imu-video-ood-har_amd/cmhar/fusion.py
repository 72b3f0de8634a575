"""Cross-attention IMU↔video fusion (north_star extension "CrossAttentionFusion"; BASELINE config 4).

The reference has no fusion module — its two encoders only meet in the SigLIP loss (`src/models/models.py:239-291`,
`src/models/losses.py:9-54`) — so this defines one on top of the drop-in encoders' outputs (parity
unpinned w.r.t. the reference, checked against the CPU restatement `oracle/fusion_cpu.py`):

    q = Wq·imu_tokens,  k = Wk·video_tokens,  v = Wv·video_tokens            (IMU tokens query the video tokens)
    h = LayerNorm(Wr·imu_tokens + Wo·MHA(q, k, v))                           (post-LN residual, eps 1e-5)
    fused = mean over the IMU tokens of h;   logits = Wc·fused

`CrossModalFusionClassifier(config)` wires IMUEncoder tokens (B, 1+N, 128) and the VideoMAE backbone's
last_hidden_state (B, L, 768) through it.  Execution: the video-side K/V projection (M = B·L rows) is one bf16 MFMA
GEMM with the K and V weights concatenated; attention is the flash kernel (head dim 64, Lq = IMU tokens, Lk = video
tokens); the residual add rides in the output-projection GEMM's epilogue; LayerNorm, token mean and the small
IMU-side GEMMs (M = B·Lq) are cmhar kernels in fp32.  compute_dtype 'fp32' runs every piece in exact fp32 (parity mode).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from . import _lib as L
from . import kernels as K
from ._lib import call, ptr


def _cast(x, dt):
    x = x.contiguous()
    if x.dtype == dt:
        return x
    return K.copy2d(x, torch.empty(x.shape, dtype=dt, device=x.device))


class _LinearFn(torch.autograd.Function):
    """y[M,N] (out_dt) = x·Wᵀ + b (+ residual) with the GEMM operands in `dt` (bf16: MFMA; fp32: exact)."""

    @staticmethod
    def forward(ctx, x, weight, bias, residual, dt, out_dt):
        xc = _cast(x, dt)
        wc = _cast(weight.detach(), dt)
        # the exact-fp32 GEMM writes fp32 / bf16; an fp16 result of it (fp16 inference path) is cast afterwards
        gemm_dt = torch.float32 if (dt == torch.float32 and out_dt == torch.float16) else out_dt
        y = torch.empty(xc.shape[0], wc.shape[0], dtype=gemm_dt, device=x.device)
        K.gemm(0, xc, wc, y, bias=None if bias is None else bias.detach(),
               residual=None if residual is None else _cast(residual, gemm_dt))
        y = _cast(y, out_dt)
        ctx.save_for_backward(xc, wc)
        ctx.dt, ctx.x_dtype, ctx.has_bias, ctx.has_res = dt, x.dtype, bias is not None, residual is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, wc = ctx.saved_tensors
        dyc = _cast(dy, ctx.dt)
        dx = dw = db = dres = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(xc.shape, dtype=ctx.x_dtype, device=dy.device)
            K.gemm(1, dyc, wc, dx)
        if ctx.needs_input_grad[1]:
            dw = torch.empty(wc.shape, dtype=torch.float32, device=dy.device)
            K.gemm(2, dyc, xc, dw)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = K.colsum(dy.contiguous())
        if ctx.has_res and ctx.needs_input_grad[3]:
            dres = dy
        return dx, dw, db, dres, None, None


class _AttnFn(torch.autograd.Function):
    """Multi-head attention of [B·Lq, H·D] queries over packed [B·Lk, 2·H·D] keys | values; the backward writes
    dK and dV straight into the two column halves of one packed gradient."""

    @staticmethod
    def forward(ctx, q, kv, B, H, Lq, Lk, D):
        k, v = kv[:, :H * D], kv[:, H * D:]
        o = torch.empty(B * Lq, H * D, dtype=q.dtype, device=q.device)
        lse = torch.empty(B * H * Lq, dtype=torch.float32, device=q.device)
        scale = 1.0 / math.sqrt(D)
        K.attention_fwd(q, k, v, o, lse, B=B, H=H, Lq=Lq, Lk=Lk, D=D, scale=scale)
        ctx.save_for_backward(q, kv, o, lse)
        ctx.geom = (B, H, Lq, Lk, D, scale)
        return o

    @staticmethod
    def backward(ctx, do):
        q, kv, o, lse = ctx.saved_tensors
        B, H, Lq, Lk, D, scale = ctx.geom
        do = _cast(do, q.dtype)
        dq = torch.empty(B * Lq, H * D, dtype=q.dtype, device=q.device)
        dkv = torch.empty(B * Lk, 2 * H * D, dtype=q.dtype, device=q.device)
        K.attention_bwd(q, kv[:, :H * D], kv[:, H * D:], o, do, lse, dq, dkv[:, :H * D], dkv[:, H * D:], B=B, H=H,
                        Lq=Lq, Lk=Lk, D=D, scale=scale)
        return dq, dkv, None, None, None, None, None


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, gamma, beta, eps):
        h = h.contiguous()
        y, mean, rstd = K.layernorm_fwd(h, gamma.detach(), beta.detach(), eps)
        ctx.save_for_backward(h, gamma, mean, rstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        h, gamma, mean, rstd = ctx.saved_tensors
        dg = torch.empty_like(gamma)
        db = torch.empty_like(gamma)
        dh = K.layernorm_bwd(dy.contiguous(), h, gamma.detach(), mean, rstd, dg, db)
        return dh, dg, db, None


class _TokenMeanFn(torch.autograd.Function):
    """[B·S, C] fp32 → [B, C] mean over each sample's S tokens (cmhar_avgpool_cl)."""

    @staticmethod
    def forward(ctx, x, B, S):
        x = x.contiguous()
        C = x.shape[1]
        out = torch.empty(B, C, dtype=torch.float32, device=x.device)
        call('cmhar_avgpool_cl', L.dtype_code(x.dtype), B, S, C, ptr(x), ptr(out), L.stream(x.device))
        ctx.geom = (B, S, C, x.dtype)
        return out

    @staticmethod
    def backward(ctx, dout):
        B, S, C, dt = ctx.geom
        dx = torch.empty(B * S, C, dtype=dt, device=dout.device)
        call('cmhar_avgpool_cl_bwd', L.dtype_code(dt), B, S, C, ptr(dout.contiguous()), ptr(dx),
             L.stream(dout.device))
        return dx, None, None


class CrossAttentionFusion(L.NoReplicate, nn.Module):
    def __init__(self, imu_dim=128, video_dim=768, d_model=256, num_heads=4, num_classes=32, eps=1e-5,
                 compute_dtype='bf16'):
        super().__init__()
        if d_model % num_heads or d_model // num_heads not in (8, 16, 32, 64):
            raise ValueError('head dim must be 8/16/32/64')
        if compute_dtype in ('bf16', 'fp16') and d_model // num_heads != 64:
            raise ValueError(f'{compute_dtype} (MFMA flash) attention needs head dim 64')
        self.d_model, self.num_heads, self.eps, self.compute_dtype = d_model, num_heads, eps, compute_dtype
        self.q_proj = nn.Linear(imu_dim, d_model)
        self.kv_proj = nn.Linear(video_dim, 2 * d_model)      # rows [0, d): K, [d, 2d): V
        self.out_proj = nn.Linear(d_model, d_model)
        self.res_proj = nn.Linear(imu_dim, d_model)
        self.norm = nn.LayerNorm(d_model, eps=eps)
        self.classifier = nn.Linear(d_model, num_classes)

    def forward(self, imu_tokens, video_tokens):
        """imu_tokens (B, Lq, imu_dim), video_tokens (B, Lk, video_dim) → (logits (B, classes), fused (B, d))."""
        if not imu_tokens.is_cuda:
            raise RuntimeError('CrossAttentionFusion runs on the cmhar HIP library: move it to the GPU')
        B, Lq, _ = imu_tokens.shape
        Lk = video_tokens.shape[1]
        d, H = self.d_model, self.num_heads
        dt = {'bf16': torch.bfloat16, 'fp16': torch.float16}.get(self.compute_dtype, torch.float32)
        xi = imu_tokens.reshape(B * Lq, -1).float()
        xv = video_tokens.reshape(B * Lk, -1)
        f32 = torch.float32
        # IMU-side GEMMs (M = B·Lq rows, a few MFLOP) stay exact fp32; the video-side K|V projection (M = B·Lk)
        # runs in the compute dtype on the MFMA GEMM
        q = _LinearFn.apply(xi, self.q_proj.weight, self.q_proj.bias, None, f32, dt)
        kv = _LinearFn.apply(xv, self.kv_proj.weight, self.kv_proj.bias, None, dt, dt)
        a = _AttnFn.apply(q, kv, B, H, Lq, Lk, d // H)
        r = _LinearFn.apply(xi, self.res_proj.weight, self.res_proj.bias, None, f32, f32)
        h = _LinearFn.apply(a, self.out_proj.weight, self.out_proj.bias, r, f32, f32)
        y = _LayerNormFn.apply(h, self.norm.weight, self.norm.bias, self.eps)
        fused = _TokenMeanFn.apply(y, B, Lq)
        logits = _LinearFn.apply(fused, self.classifier.weight, self.classifier.bias, None, torch.float32,
                                 torch.float32)
        return logits, fused


class CrossModalFusionClassifier(nn.Module):
    """IMU encoder tokens × VideoMAE tokens → CrossAttentionFusion → class logits (BASELINE config 4's model)."""

    def __init__(self, config, d_model=256, num_heads=4):
        super().__init__()
        from .models import IMUEncoder, VideoEncoder
        m = config.model
        self.imu_encoder = IMUEncoder(config)
        self.video_encoder = VideoEncoder(config)
        if not self.video_encoder.is_videomae:
            raise ValueError('CrossModalFusionClassifier needs a token-producing (VideoMAE) video backbone')
        self.fusion = CrossAttentionFusion(m.imu_d_model, self.video_encoder.feature_dim, d_model, num_heads,
                                           m.num_classes, compute_dtype=getattr(m, 'compute_dtype', 'bf16'))

    def forward(self, imu, video):
        from .videomae import run_backbone
        _, imu_tokens = self.imu_encoder(imu)
        video_tokens = run_backbone(self.video_encoder.backbone, video, token0_only=False)
        logits, _ = self.fusion(imu_tokens, video_tokens)
        return logits
