"""VideoMAE backbone on the cmhar HIP kernels — drop-in for `transformers.VideoMAEModel` as used by the reference
VideoEncoder (`src/models/models.py:154-158,197-203`).

Module tree and parameter names follow the third-party HF implementation exactly
(`embeddings.patch_embeddings.projection`, `encoder.layer.{i}.attention.attention.{query,key,value}`,
`.attention.output.dense`, `.intermediate.dense`, `.output.dense`, `.layernorm_before/after`, optional final
`layernorm`), so reference checkpoints load with `strict=True`.  The whole backbone forward/backward is ONE
autograd node whose body is a sequence of HIP launches:

  im2col(tubelet) → GEMM(+bias +sin-cos pos) → 12 × [LN → QKV GEMM(+bias) → flash attention
  → out-proj GEMM(+bias +residual) → LN → FC1 GEMM(+bias, GELU, pre-act saved) → FC2 GEMM(+bias +residual)]

and the mirrored backward (dgrad GEMMs with fused GELU'/residual epilogues, split-K fp32 wgrad GEMMs that also
emit the bias gradients, flash attention backward, fused LN backward with the residual gradient).  Compute dtype: bf16 (MFMA, fp32 accumulate),
fp32 (exact parity mode), or fp16 (MFMA, fp32 accumulate; forward only — the inference path of BASELINE config 5);
master weights and their gradients stay fp32.
"""
from __future__ import annotations

import json
import math
import os
import types
import warnings
from typing import List, Optional

import numpy as np
import torch
import torch.nn as nn

from . import _lib as L
from . import kernels as K
from .grads import AutogradSink
from .weights import PackedWeights


def sinusoid_table(n_position: int, d_hid: int) -> torch.Tensor:
    """modeling_videomae.py:80-91 (angle = pos / 10000^(2*(j//2)/d), f64 then f32)."""
    pos = np.arange(n_position, dtype=np.float64)[:, None]
    j = np.arange(d_hid)[None, :]
    ang = pos / np.power(10000, 2 * (j // 2) / d_hid)
    tab = np.empty_like(ang)
    tab[:, 0::2] = np.sin(ang[:, 0::2])
    tab[:, 1::2] = np.cos(ang[:, 1::2])
    return torch.from_numpy(tab.astype(np.float32))


class _SelfAttention(nn.Module):
    def __init__(self, hd, qkv_bias):
        super().__init__()
        self.query = nn.Linear(hd, hd, bias=qkv_bias)
        self.key = nn.Linear(hd, hd, bias=qkv_bias)
        self.value = nn.Linear(hd, hd, bias=qkv_bias)


class _Dense(nn.Module):
    def __init__(self, i, o):
        super().__init__()
        self.dense = nn.Linear(i, o)


class _Attention(nn.Module):
    def __init__(self, hd, qkv_bias):
        super().__init__()
        self.attention = _SelfAttention(hd, qkv_bias)
        self.output = _Dense(hd, hd)


class VideoMAELayer(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.attention = _Attention(cfg.hidden_size, cfg.qkv_bias)
        self.intermediate = _Dense(cfg.hidden_size, cfg.intermediate_size)
        self.output = _Dense(cfg.intermediate_size, cfg.hidden_size)
        self.layernorm_before = nn.LayerNorm(cfg.hidden_size, eps=cfg.layer_norm_eps)
        self.layernorm_after = nn.LayerNorm(cfg.hidden_size, eps=cfg.layer_norm_eps)


class _PatchEmbeddings(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        p, t = cfg.patch_size, cfg.tubelet_size
        self.projection = nn.Conv3d(cfg.num_channels, cfg.hidden_size, kernel_size=(t, p, p), stride=(t, p, p))


class _Embeddings(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.patch_embeddings = _PatchEmbeddings(cfg)
        n = (cfg.image_size // cfg.patch_size) ** 2 * (cfg.num_frames // cfg.tubelet_size)
        self.register_buffer('position_embeddings', sinusoid_table(n, cfg.hidden_size), persistent=False)


class _Encoder(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.layer = nn.ModuleList([VideoMAELayer(cfg) for _ in range(cfg.num_hidden_layers)])


def default_videomae_config(**kw):
    cfg = dict(image_size=224, patch_size=16, num_channels=3, num_frames=16, tubelet_size=2, hidden_size=768,
               num_hidden_layers=12, num_attention_heads=12, intermediate_size=3072, hidden_act='gelu',
               layer_norm_eps=1e-12, qkv_bias=True, use_mean_pooling=True)
    cfg.update({k: v for k, v in kw.items() if v is not None})
    return types.SimpleNamespace(**cfg)


_DTYPES = {'bf16': torch.bfloat16, 'fp16': torch.float16, 'fp32': torch.float32}


class VideoMAEOutput:
    def __init__(self, last_hidden_state):
        self.last_hidden_state = last_hidden_state

    def __getitem__(self, i):
        return (self.last_hidden_state,)[i]


class VideoMAEBackbone(L.NoReplicate, nn.Module):
    """HF-compatible VideoMAEModel whose forward/backward run on the cmhar HIP library."""

    def __init__(self, cfg, compute_dtype: str = 'bf16'):
        super().__init__()
        self.config = cfg
        self.compute_dtype = compute_dtype
        self.embeddings = _Embeddings(cfg)
        self.encoder = _Encoder(cfg)
        self.layernorm = None if cfg.use_mean_pooling else nn.LayerNorm(cfg.hidden_size, eps=cfg.layer_norm_eps)
        self._init_weights()
        self._packs = None

    # HF VideoMAEPreTrainedModel._init_weights: normal(0, 0.02) Linear/Conv3d, zero bias, LN (1, 0)
    @torch.no_grad()
    def _init_weights(self):
        for m in self.modules():
            if isinstance(m, (nn.Linear, nn.Conv3d)):
                m.weight.normal_(0.0, 0.02)
                if m.bias is not None:
                    m.bias.zero_()
            elif isinstance(m, nn.LayerNorm):
                m.weight.fill_(1.0)
                m.bias.zero_()

    @classmethod
    def from_pretrained(cls, path: str, compute_dtype='bf16', **overrides):
        """Load a local HF-format VideoMAE directory (config.json + model.safetensors / pytorch_model.bin).
        Hub names cannot be fetched offline: the caller decides what to do when this raises."""
        with open(os.path.join(path, 'config.json')) as f:
            c = json.load(f)
        keys = ['image_size', 'patch_size', 'num_channels', 'num_frames', 'tubelet_size', 'hidden_size',
                'num_hidden_layers', 'num_attention_heads', 'intermediate_size', 'hidden_act', 'layer_norm_eps',
                'qkv_bias', 'use_mean_pooling']
        cfg = default_videomae_config(**{k: c[k] for k in keys if k in c})
        for k, v in overrides.items():
            setattr(cfg, k, v)
        m = cls(cfg, compute_dtype)
        sd = None
        st = os.path.join(path, 'model.safetensors')
        if os.path.exists(st):
            from safetensors.torch import load_file
            sd = load_file(st)
        else:
            bn = os.path.join(path, 'pytorch_model.bin')
            if os.path.exists(bn):
                sd = torch.load(bn, map_location='cpu', weights_only=True)
        if sd is not None:
            sd = {k[len('videomae.'):] if k.startswith('videomae.') else k: v for k, v in sd.items()}
            m.load_state_dict(sd, strict=False)
        return m

    # ------------------------------------------------------------------------------------------------------
    def _weights(self):
        """Packed compute-dtype weights (QKV concatenated), refreshed when the fp32 masters change."""
        dt = _DTYPES.get(self.compute_dtype, torch.float32)
        dev = self.embeddings.patch_embeddings.projection.weight.device
        if self._packs is None or self._packs.device != dev or self._packs.dtype != dt:
            self._packs = PackedWeights(dev, dt)
            pe = self.embeddings.patch_embeddings.projection
            self._packs.add_weight('patch', [pe.weight])
            for i, layer in enumerate(self.encoder.layer):
                a = layer.attention.attention
                self._packs.add_weight(f'qkv{i}', [a.query.weight, a.key.weight, a.value.weight])
                if a.query.bias is not None:
                    self._packs.add_bias(f'bqkv{i}', [a.query.bias, a.key.bias, a.value.bias])
                self._packs.add_weight(f'o{i}', [layer.attention.output.dense.weight])
                self._packs.add_weight(f'fc1_{i}', [layer.intermediate.dense.weight])
                self._packs.add_weight(f'fc2_{i}', [layer.output.dense.weight])
            self._packs.build()
        self._packs.refresh()
        return self._packs

    def forward(self, pixel_values, bool_masked_pos=None, **kwargs):
        if bool_masked_pos is not None:
            raise NotImplementedError('masked-token pretraining is not on the accelerated path')
        out = run_backbone(self, pixel_values, token0_only=False)
        return VideoMAEOutput(out)


# ----------------------------------------------------------------------------------------------------------
# the backbone as one autograd node
# ----------------------------------------------------------------------------------------------------------
class _Ctx:
    pass


def _layer_params(layer):
    a = layer.attention.attention
    return dict(ln1w=layer.layernorm_before.weight, ln1b=layer.layernorm_before.bias,
                qw=a.query.weight, kw=a.key.weight, vw=a.value.weight,
                qb=a.query.bias, kb=a.key.bias, vb=a.value.bias,
                ow=layer.attention.output.dense.weight, ob=layer.attention.output.dense.bias,
                ln2w=layer.layernorm_after.weight, ln2b=layer.layernorm_after.bias,
                f1w=layer.intermediate.dense.weight, f1b=layer.intermediate.dense.bias,
                f2w=layer.output.dense.weight, f2b=layer.output.dense.bias)


def _forward_impl(m: VideoMAEBackbone, video: torch.Tensor, save: bool):
    cfg = m.config
    W = m._weights()
    dt = W.dtype
    B, T, Cc, Hh, Ww = video.shape
    if Cc != cfg.num_channels or Hh != cfg.image_size or Ww != cfg.image_size:
        raise ValueError(f'Input video {tuple(video.shape)} does not match model geometry')
    Hd, nh, P, tub = cfg.hidden_size, cfg.num_attention_heads, cfg.patch_size, cfg.tubelet_size
    D = Hd // nh
    Lt = (T // tub) * (Hh // P) * (Ww // P)
    pos = m.embeddings.position_embeddings
    if pos.shape[0] != Lt:
        raise ValueError(f'{Lt} tokens but the position table has {pos.shape[0]} rows (num_frames mismatch)')
    M = B * Lt
    scale = D ** -0.5
    video = video.contiguous().float()
    patches = K.tubelet_im2col(video, tub, P, dt)
    pe = m.embeddings.patch_embeddings.projection
    x = K.linear(patches, W['patch'], pe.bias, rowadd=pos, rowadd_mod=Lt)
    st = _Ctx()
    st.geom = (B, Lt, M, Hd, nh, D, scale)
    st.patches = patches if save else None
    st.layers = []
    # bf16 training path: the QKV epilogue writes the keys pre-scaled by scale·log2(e) (one rounding of the fp32
    # product, as before), the forward runs with scale = 1/log2(e) — scores land in the exp2 domain — and the
    # backward (cmhar_attention_bwd_prescaled) drops its per-score multiply (−6 % attention backward time)
    st.prescaled = dt == torch.bfloat16 and D == 64
    colscale = (Hd, 2 * Hd, scale * K.LOG2E) if st.prescaled else None
    fscale = 1.0 / K.LOG2E if st.prescaled else scale
    for layer in m.encoder.layer:
        p = _layer_params(layer)
        eps = layer.layernorm_before.eps
        h1, mu1, rs1 = K.layernorm_fwd(x, p['ln1w'], p['ln1b'], eps)
        qkv = K.linear(h1, W[f'qkv{len(st.layers)}'], W.get(f'bqkv{len(st.layers)}'), colscale=colscale)
        o = torch.empty(M, Hd, dtype=dt, device=x.device)
        lse = torch.empty(B * nh * Lt, dtype=torch.float32, device=x.device)
        K.attention_fwd(qkv[:, :Hd], qkv[:, Hd:2 * Hd], qkv[:, 2 * Hd:], o, lse, B=B, H=nh, Lq=Lt, Lk=Lt, D=D,
                        scale=fscale)
        x1 = K.linear(o, W[f'o{len(st.layers)}'], p['ob'], residual=x)
        h2, mu2, rs2 = K.layernorm_fwd(x1, p['ln2w'], p['ln2b'], layer.layernorm_after.eps)
        # the FC1 epilogue writes gelu(a) and gelu'(a) (shared transcendentals); the backward only multiplies
        pre = torch.empty(M, cfg.intermediate_size, dtype=dt, device=x.device) if save else None
        g = K.linear(h2, W[f'fc1_{len(st.layers)}'], p['f1b'], act=L.ACT_GELU_SAVEGRAD if save else L.ACT_GELU,
                     aux_out=pre)
        x2 = K.linear(g, W[f'fc2_{len(st.layers)}'], p['f2b'], residual=x1)
        st.layers.append((x, h1, mu1, rs1, qkv, o, lse, x1, h2, mu2, rs2, pre, g) if save else None)
        x = x2
    if m.layernorm is not None:
        xf, muf, rsf = K.layernorm_fwd(x, m.layernorm.weight, m.layernorm.bias, m.layernorm.eps)
        st.final = (x, muf, rsf) if save else None
        x = xf
    st.out = x
    return x, st


_WGRAD_STREAMS = {}


def _wgrad_stream(dev):
    s = _WGRAD_STREAMS.get(dev)
    if s is None:
        s = _WGRAD_STREAMS[dev] = torch.cuda.Stream(dev)
    return s


def _backward_impl(m: VideoMAEBackbone, st, dx, sink, overlap_wgrad=True):
    """dx: [M, Hd] gradient of the backbone output (compute dtype).  Parameter gradients go to `sink`
    (cmhar.grads): fp32, written by the wgrad GEMM / colsum / LN-backward epilogues with β = 0 or 1."""
    W = m._weights()
    B, Lt, M, Hd, nh, D, scale = st.geom
    dev = dx.device

    # Optionally (module attribute `overlap_wgrad`) the weight gradients (dW = dYᵀX, split-K), which do not feed the
    # rest of the backward, run on their own stream so their workgroups can fill CUs the critical-path kernels leave
    # idle; parameter groups are then declared final (gradient bucket all-reduce) from that stream, after it has
    # caught up with the main stream's LayerNorm gradients.  Measured on MI355X at B=32: no gain (the two GEMMs
    # slow each other through shared L2), so it is off by default.
    cur = torch.cuda.current_stream(dev)
    side = _wgrad_stream(dev) if overlap_wgrad else cur

    def wgrad(params, dy, x, shape, bias=None):
        """Weight gradient GEMM; the bias gradient (Σ_tokens dy) rides on the same GEMM's MFMA operand tiles."""
        out, beta = sink.dest(params, shape, dev)
        bout, bbeta = (None, 0.0)
        if bias:
            bout, bbeta = sink.dest(bias, (sum(q.numel() for q in bias),), dev)
        if side is cur:
            K.linear_wgrad(dy, x, out=out, beta=beta, bias_out=bout, bias_beta=bbeta)
            return
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            K.linear_wgrad(dy, x, out=out, beta=beta, bias_out=bout, bias_beta=bbeta)
        dy.record_stream(side)
        x.record_stream(side)

    def done(params):
        if side is cur:
            sink.done(params)
            return
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            sink.done(params)

    def ln_grads(wp, bp):
        gw, bw = sink.dest([wp], wp.shape, dev)
        gb, bb = sink.dest([bp], bp.shape, dev)
        if bw != bb:
            raise RuntimeError('LayerNorm weight/bias gradient state differs')
        return gw, gb, bw

    if m.layernorm is not None:
        x, muf, rsf = st.final
        gw, gb, beta = ln_grads(m.layernorm.weight, m.layernorm.bias)
        dx = K.layernorm_bwd(dx, x, m.layernorm.weight, muf, rsf, gw, gb, beta_acc=beta)
        sink.done([m.layernorm.weight, m.layernorm.bias])
    for li in reversed(range(len(m.encoder.layer))):
        layer = m.encoder.layer[li]
        p = _layer_params(layer)
        x, h1, mu1, rs1, qkv, o, lse, x1, h2, mu2, rs2, pre, g = st.layers[li]
        st.layers[li] = None
        # x2 = x1 + FC2(gelu(FC1(LN2(x1))))
        dpre = K.linear_dgrad(dx, W[f'fc2_{li}'], act=L.ACT_MULAUX, aux_in=pre)     # pre holds gelu'(a)
        wgrad([p['f2w']], dx, g, p['f2w'].shape, [p['f2b']])
        del g
        dh2 = K.linear_dgrad(dpre, W[f'fc1_{li}'])
        wgrad([p['f1w']], dpre, h2, p['f1w'].shape, [p['f1b']])
        del dpre, pre
        gw2, gb2, beta = ln_grads(p['ln2w'], p['ln2b'])
        dx1 = K.layernorm_bwd(dh2, x1, p['ln2w'], mu2, rs2, gw2, gb2, dres=dx, beta_acc=beta)
        del dh2, dx
        # x1 = x + O·Woᵀ + bo
        do = K.linear_dgrad(dx1, W[f'o{li}'])
        wgrad([p['ow']], dx1, o, p['ow'].shape, [p['ob']])
        dqkv = torch.empty(M, 3 * Hd, dtype=dx1.dtype, device=dev)
        attn_bwd = K.attention_bwd_prescaled if st.prescaled else K.attention_bwd
        attn_bwd(qkv[:, :Hd], qkv[:, Hd:2 * Hd], qkv[:, 2 * Hd:], o, do, lse, dqkv[:, :Hd], dqkv[:, Hd:2 * Hd],
                 dqkv[:, 2 * Hd:], B=B, H=nh, Lq=Lt, Lk=Lt, D=D, scale=scale)
        del do, o, qkv
        dh1 = K.linear_dgrad(dqkv, W[f'qkv{li}'])
        wgrad([p['qw'], p['kw'], p['vw']], dqkv, h1, (3 * Hd, Hd),
              [p['qb'], p['kb'], p['vb']] if p['qb'] is not None else None)
        del dqkv
        gw1, gb1, beta = ln_grads(p['ln1w'], p['ln1b'])
        dx = K.layernorm_bwd(dh1, x, p['ln1w'], mu1, rs1, gw1, gb1, dres=dx1, beta_acc=beta)
        del dh1, dx1
        done([q for q in p.values() if q is not None])
    pe = m.embeddings.patch_embeddings.projection
    wgrad([pe.weight], dx, st.patches, (pe.weight.shape[0], pe.weight[0].numel()), [pe.bias])
    done([pe.weight, pe.bias])
    if side is not cur:
        cur.wait_stream(side)
    st.patches = None


class _BackboneFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, video, module, token0_only, *params):
        x, st = _forward_impl(module, video, save=True)
        ctx.module, ctx.st, ctx.token0_only = module, st, token0_only
        ctx.params = params
        B, Lt, M, Hd = st.geom[:4]
        if token0_only:
            out = torch.empty(B, Hd, dtype=torch.float32, device=x.device)
            K.copy2d(x.view(B, Lt * Hd)[:, :Hd], out)
        else:
            out = torch.empty(B, Lt, Hd, dtype=torch.float32, device=x.device)
            K.copy2d(x, out.view(M, Hd))
        st.out = None
        return out

    @staticmethod
    def backward(ctx, gout):
        m, st = ctx.module, ctx.st
        B, Lt, M, Hd = st.geom[:4]
        dt = m._weights().dtype
        gout = gout.contiguous()
        if ctx.token0_only:
            dx = torch.zeros(M, Hd, dtype=dt, device=gout.device)
            K.copy2d(gout, dx.view(B, Lt * Hd)[:, :Hd])
        else:
            dx = torch.empty(M, Hd, dtype=dt, device=gout.device)
            K.copy2d(gout.view(M, Hd), dx)
        sink = getattr(m, '_grad_sink', None) or AutogradSink()
        _backward_impl(m, st, dx, sink, overlap_wgrad=getattr(m, "overlap_wgrad", False))
        ctx.st = None
        out = [None, None, None]
        for p in ctx.params:
            out.append(sink.result(p) if p.requires_grad else None)
        return tuple(out)


def run_backbone(m: VideoMAEBackbone, video: torch.Tensor, token0_only: bool) -> torch.Tensor:
    """Backbone forward (+ autograd node when gradients are needed).  Returns fp32 (B,Hd) token-0 features
    (`last_hidden_state[:, 0]`, models.py:201) or the full fp32 last_hidden_state (B, L, Hd)."""
    params = list(m.parameters())
    if torch.is_grad_enabled() and any(p.requires_grad for p in params):
        if m.compute_dtype == 'fp16':
            raise RuntimeError("compute_dtype 'fp16' is the inference-only path (BASELINE config 5): run it under "
                               "torch.no_grad() / with frozen parameters, or use 'bf16' / 'fp32' for training")
        return _BackboneFn.apply(video, m, token0_only, *params)
    with torch.no_grad():
        x, st = _forward_impl(m, video, save=False)
        B, Lt, M, Hd = st.geom[:4]
        if token0_only:
            out = torch.empty(B, Hd, dtype=torch.float32, device=x.device)
            K.copy2d(x.view(B, Lt * Hd)[:, :Hd], out)
        else:
            out = torch.empty(B, Lt, Hd, dtype=torch.float32, device=x.device)
            K.copy2d(x, out.view(M, Hd))
        return out
