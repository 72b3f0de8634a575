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
emit the bias gradients, flash attention backward, fused LN backward with the residual gradient).  When only
`last_hidden_state[:, 0]` is consumed (VideoEncoder, models.py:201) the LAST layer runs its query side, attention
output, MLP and LayerNorm 2 on the token-0 rows only (_last_layer_token0_fwd / _bwd): the same outputs and gradients,
none of the rows the reference computes and drops.  Compute dtype: bf16 (MFMA, fp32 accumulate),
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
                self._packs.add_weight(f'qkv{i}', [a.query.weight, a.key.weight, a.value.weight], transpose=_DGRAD_WT)
                if a.query.bias is not None:
                    self._packs.add_bias(f'bqkv{i}', [a.query.bias, a.key.bias, a.value.bias])
                self._packs.add_weight(f'o{i}', [layer.attention.output.dense.weight], transpose=_DGRAD_WT)
                self._packs.add_weight(f'fc1_{i}', [layer.intermediate.dense.weight], transpose=_DGRAD_WT)
                self._packs.add_weight(f'fc2_{i}', [layer.output.dense.weight], transpose=_DGRAD_WT)
            self._packs.build()
        self._packs.refresh()
        return self._packs

    def forward(self, pixel_values, bool_masked_pos=None, **kwargs):
        if bool_masked_pos is not None:
            raise NotImplementedError('masked-token pretraining is not on the accelerated path')
        out = run_backbone(self, pixel_values, token0_only=False)
        return VideoMAEOutput(out)


# Input-gradient GEMMs dX = dY·W on the transposed bf16 weight copy Wᵀ [K, N] in the FORWARD layout (K-contiguous B
# reads, the 8-phase / tail-split forward kernels) instead of the dgrad layout's transposed LDS reads of W [N, K]
# (cmhar.weights.PackedWeights.transposed: one multi-matrix transpose launch per step after AdamW).  Same fp32 products
# and epilogues; CMHAR_DGRAD_WT=0 restores the dgrad layout (A/B knob).
_DGRAD_WT = os.environ.get('CMHAR_DGRAD_WT', '1') != '0'


def _dgrad(W, name, dy, rows=None, act=L.ACT_NONE, aux_in=None, residual=None, out=None):
    """dX = dY · W[name][rows] (+ epilogue) — on Wᵀ in the forward layout when the pack keeps a transposed copy."""
    wt = W.transposed(name) if hasattr(W, 'transposed') else None
    if wt is None:
        w = W[name] if rows is None else W[name][rows]
        return K.linear_dgrad(dy, w, act=act, aux_in=aux_in, residual=residual, out=out)
    b = wt if rows is None else wt[:, rows]
    if out is None:
        out = torch.empty(dy.shape[0], b.shape[0], dtype=dy.dtype, device=dy.device)
    return K.gemm(0, dy, b, out, act=act, aux_in=aux_in, residual=residual)


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


def _token0_last_ok(m, B, dt):
    """Whether the last layer may run on the token-0 rows only (see _last_layer_token0_fwd): the bf16 weight-gradient
    GEMMs contract over the B token-0 rows, which the bf16 kernels need in multiples of 8; CMHAR_TOKEN0_LAST=0 turns
    it off (A/B knob)."""
    if os.environ.get('CMHAR_TOKEN0_LAST', '1') == '0' or len(m.encoder.layer) == 0:
        return False
    return dt == torch.float32 or B % 8 == 0


def _last_layer_token0_fwd(m, layer, li, x, W, geom, colscale, fscale, save):
    """The LAST encoder layer when only `last_hidden_state[:, 0]` is consumed (VideoEncoder, models.py:201).

    Row t of the layer output depends on row t of the attention output and MLP only, so for token 0 of each clip
    only these rows are needed: LN1 (all rows, for the keys / values), K|V projection (all rows), Q projection of
    the token-0 rows, attention with ONE query per (clip, head) over all 1568 keys, out-projection, LN2, FC1 and FC2
    on the B token-0 rows.  The values computed — and, through _last_layer_token0_bwd, every parameter gradient —
    are those of the full layer: the rows skipped feed nothing the model returns (the reference computes them and
    drops them at models.py:201).  Returns the token-0 output rows [B, Hd] and the saved state."""
    B, Lt, M, Hd, nh, D, scale = geom
    p = _layer_params(layer)
    h1, mu1, rs1 = K.layernorm_fwd(x, p['ln1w'], p['ln1b'], layer.layernorm_before.eps)
    wqkv, bqkv = W[f'qkv{li}'], W.get(f'bqkv{li}')
    wq, wkv = wqkv[:Hd], wqkv[Hd:]
    bq = bqkv[:Hd] if bqkv is not None else None
    bkv = bqkv[Hd:] if bqkv is not None else None
    kv = K.linear(h1, wkv, bkv, colscale=None if colscale is None else (0, Hd, colscale[2]))
    h1_0 = h1.view(B, Lt, Hd)[:, 0]
    q0 = K.linear(h1_0, wq, bq)
    o0 = torch.empty(B, Hd, dtype=x.dtype, device=x.device)
    lse0 = torch.empty(B * nh, dtype=torch.float32, device=x.device)
    K.attention_fwd(q0, kv[:, :Hd], kv[:, Hd:], o0, lse0, B=B, H=nh, Lq=1, Lk=Lt, D=D, scale=fscale)
    x_0 = x.view(B, Lt, Hd)[:, 0]
    x1_0 = K.linear(o0, W[f'o{li}'], p['ob'], residual=x_0)
    h2_0, mu2, rs2 = K.layernorm_fwd(x1_0, p['ln2w'], p['ln2b'], layer.layernorm_after.eps)
    pre0 = torch.empty(B, m_inter(layer), dtype=x.dtype, device=x.device) if save else None
    g0 = K.linear(h2_0, W[f'fc1_{li}'], p['f1b'], act=L.ACT_GELU_SAVEGRAD if save else L.ACT_GELU, aux_out=pre0)
    x2_0 = K.linear(g0, W[f'fc2_{li}'], p['f2b'], residual=x1_0)
    saved = ('token0', x, h1, mu1, rs1, q0, kv, o0, lse0, x1_0, h2_0, mu2, rs2, pre0, g0) if save else None
    return x2_0, saved


def m_inter(layer):
    return layer.intermediate.dense.weight.shape[0]


def _forward_impl(m: VideoMAEBackbone, video: torch.Tensor, save: bool, token0_only: bool = False):
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
    st.token0 = token0_only and _token0_last_ok(m, B, dt)
    nlayer = len(m.encoder.layer)
    for layer in m.encoder.layer:
        if st.token0 and len(st.layers) == nlayer - 1:
            x, saved = _last_layer_token0_fwd(m, layer, len(st.layers), x, W, st.geom, colscale, fscale, save)
            st.layers.append(saved)
            break
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
# backward's weight-gradient stream use (module attribute `overlap_wgrad` overrides): '0' (default) = all on the main
# stream, '1' = the weight-gradient GEMMs (+ their split-K reduces) on the side stream, 'reduce' = only the split-K
# reduces on the side stream.  Measured at B = 32, alternated runs on one box: with the 8-phase weight-gradient kernel
# 682.5 / 681.4 clips/s side stream vs 675.0 / 675.2 all-main (+1 %); 'reduce' 679.5 / 678.6 vs 683.1 / 682.3
# all-main on another box.  Off by default: with two streams every backward kernel's measured duration is a share of
# a chip it splits with the other stream (the bench's HIP events and rocprofv3 then disagree by ~15 % on the dominant
# kernel), which the per-kernel roofline accounting of bench.py cannot attribute; DESIGN.md §Round 3.
_OVERLAP_WGRAD = {'1': True, 'reduce': 'reduce'}.get(os.environ.get('CMHAR_OVERLAP_WGRAD', '0'), False)


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
    # caught up with the main stream's LayerNorm gradients (default: see _OVERLAP_WGRAD for the measurements).
    # overlap_wgrad = 'reduce': the weight-gradient GEMMs stay on the main stream and only their split-K
    # reduces (memory-bound, off the critical path: nothing in the backward reads dW) go to the side stream, from
    # partial slabs of their own; parameter groups are declared final from the side stream as above.
    cur = torch.cuda.current_stream(dev)
    side = _wgrad_stream(dev) if overlap_wgrad else cur
    reduce_only = overlap_wgrad == 'reduce'

    def wgrad(params, dy, x, shape, bias=None):
        """Weight gradient GEMM; the bias gradient (Σ_tokens dy) rides on the same GEMM's MFMA operand tiles."""
        out, beta = sink.dest(params, shape, dev)
        bout, bbeta = (None, 0.0)
        if bias:
            bout, bbeta = sink.dest(bias, (sum(q.numel() for q in bias),), dev)
        if side is cur or reduce_only:
            K.linear_wgrad(dy, x, out=out, beta=beta, bias_out=bout, bias_beta=bbeta,
                           reduce_stream=side if reduce_only else None)
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
        if isinstance(st.layers[li][0], str):           # 'token0': the pruned last layer
            dx = _last_layer_token0_bwd(st, li, p, W, dx, wgrad, ln_grads, sink, dev)
            done([q for q in p.values() if q is not None])
            continue
        x, h1, mu1, rs1, qkv, o, lse, x1, h2, mu2, rs2, pre, g = st.layers[li]
        st.layers[li] = None
        # x2 = x1 + FC2(gelu(FC1(LN2(x1))))
        dpre = _dgrad(W, f'fc2_{li}', dx, act=L.ACT_MULAUX, aux_in=pre)     # pre holds gelu'(a)
        wgrad([p['f2w']], dx, g, p['f2w'].shape, [p['f2b']])
        del g
        dh2 = _dgrad(W, f'fc1_{li}', dpre)
        wgrad([p['f1w']], dpre, h2, p['f1w'].shape, [p['f1b']])
        del dpre, pre
        gw2, gb2, beta = ln_grads(p['ln2w'], p['ln2b'])
        dx1 = K.layernorm_bwd(dh2, x1, p['ln2w'], mu2, rs2, gw2, gb2, dres=dx, beta_acc=beta)
        del dh2, dx
        # x1 = x + O·Woᵀ + bo
        do = _dgrad(W, f'o{li}', dx1)
        wgrad([p['ow']], dx1, o, p['ow'].shape, [p['ob']])
        dqkv = torch.empty(M, 3 * Hd, dtype=dx1.dtype, device=dev)
        attn_bwd = K.attention_bwd_prescaled if st.prescaled else K.attention_bwd
        attn_bwd(qkv[:, :Hd], qkv[:, Hd:2 * Hd], qkv[:, 2 * Hd:], o, do, lse, dqkv[:, :Hd], dqkv[:, Hd:2 * Hd],
                 dqkv[:, 2 * Hd:], B=B, H=nh, Lq=Lt, Lk=Lt, D=D, scale=scale)
        del do, o, qkv
        dh1 = _dgrad(W, f'qkv{li}', dqkv)
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


def _last_layer_token0_bwd(st, li, p, W, dx0, wgrad, ln_grads, sink, dev):
    """Backward of _last_layer_token0_fwd.  dx0: [B, Hd] gradient of the token-0 output rows (the only rows the model
    returns, so the gradient of every other row of the layer output is zero).  The MLP, LN2, out-projection and the
    attention's query side run on the B token-0 rows; the keys / values receive their (dense) gradients from the one
    query per (clip, head); LN1's backward and the QKV weight gradients cover every row.  Returns dx [M, Hd]."""
    B, Lt, M, Hd, nh, D, scale = st.geom
    _, x, h1, mu1, rs1, q0, kv, o0, lse0, x1_0, h2_0, mu2, rs2, pre0, g0 = st.layers[li]
    st.layers[li] = None
    dpre0 = _dgrad(W, f'fc2_{li}', dx0, act=L.ACT_MULAUX, aux_in=pre0)
    wgrad([p['f2w']], dx0, g0, p['f2w'].shape, [p['f2b']])
    dh2_0 = _dgrad(W, f'fc1_{li}', dpre0)
    wgrad([p['f1w']], dpre0, h2_0, p['f1w'].shape, [p['f1b']])
    del dpre0, pre0, g0
    gw2, gb2, beta = ln_grads(p['ln2w'], p['ln2b'])
    dx1_0 = K.layernorm_bwd(dh2_0, x1_0, p['ln2w'], mu2, rs2, gw2, gb2, dres=dx0, beta_acc=beta)
    do0 = _dgrad(W, f'o{li}', dx1_0)
    wgrad([p['ow']], dx1_0, o0, p['ow'].shape, [p['ob']])
    dq0 = torch.empty(B, Hd, dtype=dx0.dtype, device=dev)
    dkv = torch.empty(M, 2 * Hd, dtype=dx0.dtype, device=dev)
    attn_bwd = K.attention_bwd_prescaled if st.prescaled else K.attention_bwd
    attn_bwd(q0, kv[:, :Hd], kv[:, Hd:], o0, do0, lse0, dq0, dkv[:, :Hd], dkv[:, Hd:], B=B, H=nh, Lq=1, Lk=Lt, D=D,
             scale=scale)
    del do0, o0
    dh1 = _dgrad(W, f'qkv{li}', dkv, rows=slice(Hd, None))     # K|V rows: every token
    dh1_0 = dh1.view(B, Lt, Hd)[:, 0]
    _dgrad(W, f'qkv{li}', dq0, rows=slice(None, Hd), residual=dh1_0, out=dh1_0)   # + Q rows: token-0 rows (one rounding)
    # QKV weight / bias gradients into the packed [3Hd, Hd] destination: Q rows from the token-0 rows, K|V rows
    # from every row
    out, wbeta = sink.dest([p['qw'], p['kw'], p['vw']], (3 * Hd, Hd), dev)
    bout, bbeta = (None, 0.0)
    if p['qb'] is not None:
        bout, bbeta = sink.dest([p['qb'], p['kb'], p['vb']], (3 * Hd,), dev)
    h1_0 = h1.view(B, Lt, Hd)[:, 0]
    K.linear_wgrad(dq0, h1_0, out=out[:Hd], beta=wbeta, bias_out=None if bout is None else bout[:Hd],
                   bias_beta=bbeta)
    K.linear_wgrad(dkv, h1, out=out[Hd:], beta=wbeta, bias_out=None if bout is None else bout[Hd:], bias_beta=bbeta)
    del dkv, kv, q0
    gw1, gb1, beta = ln_grads(p['ln1w'], p['ln1b'])
    dx = K.layernorm_bwd(dh1, x, p['ln1w'], mu1, rs1, gw1, gb1, beta_acc=beta)
    # the residual path's gradient is nonzero on the token-0 rows only: those B rows' LN backward again, with dx1_0 in
    # its dres epilogue, so each is ONE bf16 rounding of LN'(dh1) + dx1_0 as in the full layer's fused backward (a
    # copy-add after the first pass rounded them twice); that pass's dγ / dβ of the B rows are discarded
    mu0 = K.copy2d(mu1.view(B, Lt)[:, :1], torch.empty(B, 1, dtype=torch.float32, device=dev)).view(B)
    rs0 = K.copy2d(rs1.view(B, Lt)[:, :1], torch.empty(B, 1, dtype=torch.float32, device=dev)).view(B)
    scratch = torch.empty(2, Hd, dtype=torch.float32, device=dev)
    K.layernorm_bwd(dh1.view(B, Lt, Hd)[:, 0], x.view(B, Lt, Hd)[:, 0], p['ln1w'], mu0, rs0, scratch[0], scratch[1],
                    dres=dx1_0, dh=dx.view(B, Lt, Hd)[:, 0])
    return dx


class _BackboneFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, video, module, token0_only, *params):
        x, st = _forward_impl(module, video, save=True, token0_only=token0_only)
        ctx.module, ctx.st, ctx.token0_only = module, st, token0_only
        ctx.params = params
        B, Lt, M, Hd = st.geom[:4]
        if token0_only:
            out = torch.empty(B, Hd, dtype=torch.float32, device=x.device)
            K.copy2d(x if st.token0 else x.view(B, Lt * Hd)[:, :Hd], out)
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
        if ctx.token0_only and st.token0:
            dx = torch.empty(B, Hd, dtype=dt, device=gout.device)        # the token-0 rows' gradient only
            K.copy2d(gout, dx)
        elif ctx.token0_only:
            dx = torch.zeros(M, Hd, dtype=dt, device=gout.device)
            K.copy2d(gout, dx.view(B, Lt * Hd)[:, :Hd])
        else:
            dx = torch.empty(M, Hd, dtype=dt, device=gout.device)
            K.copy2d(gout.view(M, Hd), dx)
        sink = getattr(m, '_grad_sink', None) or AutogradSink()
        _backward_impl(m, st, dx, sink, overlap_wgrad=getattr(m, "overlap_wgrad", _OVERLAP_WGRAD))
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
        x, st = _forward_impl(m, video, save=False, token0_only=token0_only)
        B, Lt, M, Hd = st.geom[:4]
        if token0_only:
            out = torch.empty(B, Hd, dtype=torch.float32, device=x.device)
            K.copy2d(x if st.token0 else x.view(B, Lt * Hd)[:, :Hd], out)
        else:
            out = torch.empty(B, Lt, Hd, dtype=torch.float32, device=x.device)
            K.copy2d(x, out.view(M, Hd))
        return out
