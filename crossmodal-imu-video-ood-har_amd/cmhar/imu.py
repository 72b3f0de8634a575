"""IMU encoder (PatchTST-style transformer) on the cmhar HIP library — drop-in for the reference
`PatchEmbedding` / `IMUEncoder` (`src/models/models.py:16-132`).

Same constructor signature, same module tree (`patch_embed.projections.{c}`, `cls_token`, `pos_encoding`,
`transformer.layers.{i}` = torch `nn.TransformerEncoderLayer` parameter containers, `norm`), same construction
order (so `torch.manual_seed` gives the reference's initial weights), same outputs `(cls (B,D), tokens (B,T,D))`
including the reference's positional-table truncation (`models.py:122-123`: only CLS + the first
`max_patches` patch tokens — i.e. channel 0 at the default geometry — reach the transformer; the other
channels' projections still receive exact-zero gradients).

Computation is exact fp32 (the encoder is ~21 MFLOP per window, latency-bound): fused embed kernel, then per
post-LN layer: QKV GEMM, attention (+prob dropout), out-proj GEMM, add+dropout+LayerNorm, FC1 GEMM with fused
ReLU+dropout, FC2 GEMM, add+dropout+LayerNorm; final LayerNorm.  Dropout masks come from a counter hash and are
regenerated, not stored, in backward.
"""
from __future__ import annotations

import ctypes
import math
import os

import torch
import torch.nn as nn

from . import _lib as L
from . import kernels as K


class PatchEmbedding(nn.Module):
    """models.py:16-50: unfold(L, patch, stride) then one Linear(patch → d_model) per channel."""

    def __init__(self, in_channels, patch_size, stride, d_model):
        super().__init__()
        self.patch_size = patch_size
        self.stride = stride
        self.d_model = d_model
        self.projections = nn.ModuleList([nn.Linear(patch_size, d_model) for _ in range(in_channels)])

    def forward(self, x):
        """(B, C, L) → (B, C, N, D)  (standalone use; IMUEncoder uses the fused embed kernel)."""
        B, Cc, Lx = x.shape
        x = x.contiguous()
        N = (Lx - self.patch_size) // self.stride + 1
        out = torch.empty(B, Cc, N, self.d_model, dtype=torch.float32, device=x.device)
        for c in range(Cc):
            lin = self.projections[c]
            epi = L.epilogue(bias=lin.bias)
            L.call('cmhar_gemm_generic', L.F32, L.F32, N, self.d_model, self.patch_size, B,
                   x.data_ptr() + c * Lx * 4, self.stride, 1, Cc * Lx, lin.weight.data_ptr(), 1, self.patch_size, 0,
                   out.data_ptr() + c * N * self.d_model * 4, self.d_model, Cc * N * self.d_model,
                   ctypes.byref(epi), L.stream(x.device))
        return out


class IMUEncoder(L.NoReplicate, nn.Module):
    """models.py:53-132."""

    def __init__(self, config):
        super().__init__()
        self.config = config
        model_cfg = config.model
        self.in_channels = config.data.imu_channels
        self.patch_size = model_cfg.imu_patch_size
        self.stride = model_cfg.imu_stride
        self.d_model = model_cfg.imu_d_model
        self.patch_embed = PatchEmbedding(self.in_channels, self.patch_size, self.stride, self.d_model)
        self.cls_token = nn.Parameter(torch.randn(1, 1, self.d_model))
        max_patches = (config.data.imu_window_size - self.patch_size) // self.stride + 1
        self.pos_encoding = nn.Parameter(torch.randn(1, max_patches + 1, self.d_model))
        encoder_layer = nn.TransformerEncoderLayer(d_model=self.d_model, nhead=model_cfg.imu_nhead,
                                                   dim_feedforward=self.d_model * 4, dropout=model_cfg.imu_dropout,
                                                   batch_first=True)
        self.transformer = nn.TransformerEncoder(encoder_layer, num_layers=model_cfg.imu_num_layers,
                                                 enable_nested_tensor=False)
        self.norm = nn.LayerNorm(self.d_model)
        self.nhead = model_cfg.imu_nhead
        self.dropout_p = float(model_cfg.imu_dropout)
        self._seed_base = int(getattr(config.training, 'seed', 42))
        self._calls = 0

    def forward(self, x):
        """x (B, C, L) → cls (B, D), encoded (B, 1+N', D)."""
        if x.dim() != 3 or x.shape[1] != self.in_channels:
            raise ValueError(f'expected (B, {self.in_channels}, L) IMU windows, got {tuple(x.shape)}')
        p = self.dropout_p if self.training else 0.0
        seed = 0
        if p > 0:   # fresh dropout stream per call, reproducible, no device sync
            self._calls += 1
            seed = (self._seed_base * 0x9E3779B1 + self._calls * 0x85EBCA77) & ((1 << 62) - 1)
        params = list(self.parameters())
        x = x.contiguous().float()
        if torch.is_grad_enabled() and any(q.requires_grad for q in params):
            return _IMUFn.apply(x, self, p, seed, *params)
        with torch.no_grad():
            enc, _ = _imu_forward(self, x, p, seed, save=False)
            B, T, D = enc.shape
            return enc[:, 0].contiguous(), enc


def _layer(m, i):
    return m.transformer.layers[i]


def _imu_forward(m: IMUEncoder, x, p, seed, save):
    B, Cc, Lx = x.shape
    P, S, D = m.patch_size, m.stride, m.d_model
    N = (Lx - P) // S + 1
    T = min(1 + Cc * N, m.pos_encoding.shape[1])
    M = B * T
    dev = x.device
    emb = torch.empty(M, D, dtype=torch.float32, device=dev)
    ws = K.ptr_array([lin.weight for lin in m.patch_embed.projections])
    bs = K.ptr_array([lin.bias for lin in m.patch_embed.projections])
    L.call('cmhar_imu_embed_fwd', B, Cc, Lx, N, P, S, D, T, x.data_ptr(), ws, bs, m.cls_token.data_ptr(),
           m.pos_encoding.data_ptr(), emb.data_ptr(), L.stream(dev))
    nh = m.nhead
    dh = D // nh
    scale = 1.0 / math.sqrt(dh)
    if _fused_ok(m, T):
        return _imu_forward_fused(m, emb, p, seed, (B, Cc, Lx, N, T, M, D, nh, dh, scale))
    h = emb
    saved = []
    for i in range(len(m.transformer.layers)):
        lay = _layer(m, i)
        sd = seed + 7919 * (i + 1)
        qkv = K.linear(h, lay.self_attn.in_proj_weight, lay.self_attn.in_proj_bias)
        o = torch.empty(M, D, dtype=torch.float32, device=dev)
        lse = torch.empty(B * nh * T, dtype=torch.float32, device=dev)
        K.attention_fwd(qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], o, lse, B=B, H=nh, Lq=T, Lk=T, D=dh,
                        scale=scale, pdrop=p, seed=sd + 1)
        a = K.linear(o, lay.self_attn.out_proj.weight, lay.self_attn.out_proj.bias)
        s1 = torch.empty(M, D, dtype=torch.float32, device=dev)
        h1, mu1, rs1 = K.layernorm_fwd(h, lay.norm1.weight, lay.norm1.bias, lay.norm1.eps, b=a, pdrop=p, seed=sd + 2,
                                       h_out=s1)
        fd = K.linear(h1, lay.linear1.weight, lay.linear1.bias, act=L.ACT_RELU, pdrop=p, seed=sd + 3)
        f2 = K.linear(fd, lay.linear2.weight, lay.linear2.bias)
        s2 = torch.empty(M, D, dtype=torch.float32, device=dev)
        h2, mu2, rs2 = K.layernorm_fwd(h1, lay.norm2.weight, lay.norm2.bias, lay.norm2.eps, b=f2, pdrop=p,
                                       seed=sd + 4, h_out=s2)
        if save:
            saved.append((h, qkv, o, lse, s1, mu1, rs1, h1, fd, s2, mu2, rs2))
        h = h2
    enc, muf, rsf = K.layernorm_fwd(h, m.norm.weight, m.norm.bias, m.norm.eps)
    st = dict(geom=(B, Cc, Lx, N, T, M, D, nh, dh, scale), saved=saved, final=(h, muf, rsf), p=p, seed=seed)
    return enc.view(B, T, D), st


# The whole transformer stack + final norm as ONE launch (cmhar_imu_encoder_fwd, bit-identical to the per-op chain
# above) at the reference geometry: d_model 128, 8 heads, FF 512, T <= 32 tokens.  CMHAR_IMU_FUSED=0 keeps the
# per-op launches (A/B tests).
_FUSED = os.environ.get('CMHAR_IMU_FUSED', '1') != '0'


def _fused_ok(m, T):
    if not _FUSED or m.d_model != 128 or m.nhead != 8 or not 1 <= T <= 32:
        return False
    layers = m.transformer.layers
    if not 1 <= len(layers) <= L.IMU_MAX_LAYERS:
        return False
    for lay in layers:
        if lay.linear1.out_features != 512 or lay.norm_first or lay.activation_relu_or_gelu != 1:
            return False
    return all(q.dtype == torch.float32 and q.is_contiguous() for q in m.parameters())


def _imu_forward_fused(m, emb, p, seed, geom):
    B, Cc, Lx, N, T, M, D, nh, dh, scale = geom
    nl = len(m.transformer.layers)
    # one arena per call: per layer qkv | o | s1 | h1 | fd | s2 | h2 (M rows each) | lse | mu1 | rs1 | mu2 | rs2
    per = M * 12 * D + B * nh * T + 4 * M
    arena = torch.empty(nl * per + 2 * M, dtype=torch.float32, device=emb.device)
    arr = (L.IMULayer * nl)()
    saved = []
    h = emb
    for i in range(nl):
        lay = _layer(m, i)
        base = i * per
        views = {}
        off = base
        for name, w in (('qkv', 3 * D), ('o', D), ('s1', D), ('h1', D), ('fd', 4 * D), ('s2', D), ('h2', D)):
            views[name] = arena[off:off + M * w].view(M, w)
            off += M * w
        views['lse'] = arena[off:off + B * nh * T]
        off += B * nh * T
        for name in ('mu1', 'rs1', 'mu2', 'rs2'):
            views[name] = arena[off:off + M]
            off += M
        e = arr[i]
        sa = lay.self_attn
        for f, t in (('w_qkv', sa.in_proj_weight), ('b_qkv', sa.in_proj_bias), ('w_out', sa.out_proj.weight),
                     ('b_out', sa.out_proj.bias), ('ln1_g', lay.norm1.weight), ('ln1_b', lay.norm1.bias),
                     ('w_ff1', lay.linear1.weight), ('b_ff1', lay.linear1.bias), ('w_ff2', lay.linear2.weight),
                     ('b_ff2', lay.linear2.bias), ('ln2_g', lay.norm2.weight), ('ln2_b', lay.norm2.bias)):
            setattr(e, f, t.data_ptr())
        e.eps1, e.eps2 = lay.norm1.eps, lay.norm2.eps
        for name, t in views.items():
            setattr(e, name, t.data_ptr())
        saved.append((h, views['qkv'], views['o'], views['lse'], views['s1'], views['mu1'], views['rs1'], views['h1'],
                      views['fd'], views['s2'], views['mu2'], views['rs2']))
        h = views['h2']
    muf = arena[nl * per:nl * per + M]
    rsf = arena[nl * per + M:]
    enc = torch.empty(M, D, dtype=torch.float32, device=emb.device)   # the module output: not an arena view
    L.call('cmhar_imu_encoder_fwd', B, T, D, nh, 4 * D, nl, emb.data_ptr(), arr, m.norm.weight.data_ptr(),
           m.norm.bias.data_ptr(), m.norm.eps, enc.data_ptr(), muf.data_ptr(), rsf.data_ptr(), scale, p, seed,
           L.stream(emb.device))
    st = dict(geom=geom, saved=saved, final=(h, muf, rsf), p=p, seed=seed, fused=(arr, emb))
    return enc.view(B, T, D), st


def _imu_backward_fused(m, x, st, d_enc):
    """Two launches for the whole stack (cmhar_imu_encoder_bwd), then the embedding backward."""
    B, Cc, Lx, N, T, M, D, nh, dh, scale = st['geom']
    arr, emb = st['fused']
    nl = len(m.transformer.layers)
    dev = d_enc.device
    layers = [_layer(m, i) for i in range(nl)]
    # one arena: per layer the token-gradient scratch, then every parameter gradient, then dx
    tok = M * (3 * D + D + 4 * D + D + D + D)
    pshapes = []
    for lay in layers:
        sa = lay.self_attn
        pshapes.append([(f, t) for f, t in (('dw_qkv', sa.in_proj_weight), ('db_qkv', sa.in_proj_bias),
                                            ('dw_out', sa.out_proj.weight), ('db_out', sa.out_proj.bias),
                                            ('dln1_g', lay.norm1.weight), ('dln1_b', lay.norm1.bias),
                                            ('dw_ff1', lay.linear1.weight), ('db_ff1', lay.linear1.bias),
                                            ('dw_ff2', lay.linear2.weight), ('db_ff2', lay.linear2.bias),
                                            ('dln2_g', lay.norm2.weight), ('dln2_b', lay.norm2.bias))])
    # parameter gradients start on 16-B boundaries (4 floats) so every view is vector-aligned
    psize = sum(((t.numel() + 3) // 4) * 4 for ps in pshapes for _, t in ps)
    arena = torch.empty(nl * tok + psize + 2 * D + M * D, dtype=torch.float32, device=dev)
    garr = (L.IMULayerGrad * nl)()
    grads = {}
    off = 0
    for i in range(nl):
        g = garr[i]
        for name, w in (('dqkv', 3 * D), ('da', D), ('dpre', 4 * D), ('df2', D), ('gln1', D), ('gln2', D)):
            setattr(g, name, arena[off:off + M * w].data_ptr())
            off += M * w
    for i in range(nl):
        for name, t in pshapes[i]:
            v = arena[off:off + t.numel()].view(t.shape)
            off += ((t.numel() + 3) // 4) * 4
            setattr(garr[i], name, v.data_ptr())
            grads[t] = v
    dgf, dbf = arena[off:off + D], arena[off + D:off + 2 * D]
    off += 2 * D
    dx = arena[off:off + M * D].view(M, D)
    h, muf, rsf = st['final']
    L.call('cmhar_imu_encoder_bwd', B, T, D, nh, 4 * D, nl, emb.data_ptr(), arr, garr, m.norm.weight.data_ptr(),
           muf.data_ptr(), rsf.data_ptr(), d_enc.data_ptr(), dgf.data_ptr(), dbf.data_ptr(), dx.data_ptr(), scale,
           st['p'], st['seed'], L.stream(dev))
    grads[m.norm.weight], grads[m.norm.bias] = dgf, dbf
    _embed_backward(m, x, st, dx, grads)
    return grads


def _imu_backward(m: IMUEncoder, x, st, d_enc):
    if 'fused' in st:
        return _imu_backward_fused(m, x, st, d_enc)
    B, Cc, Lx, N, T, M, D, nh, dh, scale = st['geom']
    p, seed = st['p'], st['seed']
    dev = d_enc.device
    grads = {}

    def g32(t):
        return torch.empty(t.shape, dtype=torch.float32, device=dev)

    h, muf, rsf = st['final']
    gw, gb = g32(m.norm.weight), g32(m.norm.bias)
    dh_ = K.layernorm_bwd(d_enc, h, m.norm.weight, muf, rsf, gw, gb)
    grads[m.norm.weight], grads[m.norm.bias] = gw, gb
    for i in reversed(range(len(m.transformer.layers))):
        lay = _layer(m, i)
        sd = seed + 7919 * (i + 1)
        hin, qkv, o, lse, s1, mu1, rs1, h1, fd, s2, mu2, rs2 = st['saved'][i]
        # h2 = LN2(h1 + drop(f2))
        gw2, gb2 = g32(lay.norm2.weight), g32(lay.norm2.bias)
        df2 = torch.empty(M, D, dtype=torch.float32, device=dev)
        ds2 = K.layernorm_bwd(dh_, s2, lay.norm2.weight, mu2, rs2, gw2, gb2, db_out=df2, pdrop=p, seed=sd + 4)
        grads[lay.norm2.weight], grads[lay.norm2.bias] = gw2, gb2
        # f2 = fd·W2ᵀ + b2 ; fd = drop(relu(h1·W1ᵀ + b1))
        dpre = K.linear_dgrad(df2, lay.linear2.weight, act=L.ACT_DRELU, aux_in=fd, pdrop=p, seed=sd + 3)
        grads[lay.linear2.weight] = K.linear_wgrad(df2, fd)
        grads[lay.linear2.bias] = K.colsum(df2)
        dh1 = K.linear_dgrad(dpre, lay.linear1.weight, residual=ds2)
        grads[lay.linear1.weight] = K.linear_wgrad(dpre, h1)
        grads[lay.linear1.bias] = K.colsum(dpre)
        # h1 = LN1(hin + drop(a)) ; a = o·Woᵀ + bo
        gw1, gb1 = g32(lay.norm1.weight), g32(lay.norm1.bias)
        da = torch.empty(M, D, dtype=torch.float32, device=dev)
        ds1 = K.layernorm_bwd(dh1, s1, lay.norm1.weight, mu1, rs1, gw1, gb1, db_out=da, pdrop=p, seed=sd + 2)
        grads[lay.norm1.weight], grads[lay.norm1.bias] = gw1, gb1
        do = K.linear_dgrad(da, lay.self_attn.out_proj.weight)
        grads[lay.self_attn.out_proj.weight] = K.linear_wgrad(da, o)
        grads[lay.self_attn.out_proj.bias] = K.colsum(da)
        dqkv = torch.empty(M, 3 * D, dtype=torch.float32, device=dev)
        K.attention_bwd(qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], o, do, lse, dqkv[:, :D], dqkv[:, D:2 * D],
                        dqkv[:, 2 * D:], B=B, H=nh, Lq=T, Lk=T, D=dh, scale=scale, pdrop=p, seed=sd + 1)
        dh_ = K.linear_dgrad(dqkv, lay.self_attn.in_proj_weight, residual=ds1)
        grads[lay.self_attn.in_proj_weight] = K.linear_wgrad(dqkv, hin)
        grads[lay.self_attn.in_proj_bias] = K.colsum(dqkv)
    _embed_backward(m, x, st, dh_, grads)
    return grads


def _embed_backward(m, x, st, dh_, grads):
    B, Cc, Lx, N, T, M, D, nh, dh, scale = st['geom']
    dev = dh_.device

    def g32(t):
        return torch.empty(t.shape, dtype=torch.float32, device=dev)

    dcls = g32(m.cls_token)
    dpos = g32(m.pos_encoding)
    dws = [g32(lin.weight) for lin in m.patch_embed.projections]
    dbs = [g32(lin.bias) for lin in m.patch_embed.projections]
    L.call('cmhar_imu_embed_bwd', B, Cc, Lx, N, m.patch_size, m.stride, D, T, m.pos_encoding.shape[1], x.data_ptr(),
           dh_.data_ptr(), dcls.data_ptr(), dpos.data_ptr(), K.ptr_array(dws), K.ptr_array(dbs), L.stream(dev))
    grads[m.cls_token], grads[m.pos_encoding] = dcls, dpos
    for lin, dw, db in zip(m.patch_embed.projections, dws, dbs):
        grads[lin.weight], grads[lin.bias] = dw, db


class _IMUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, module, p, seed, *params):
        enc, st = _imu_forward(module, x, p, seed, save=True)
        ctx.module, ctx.st, ctx.params = module, st, params
        ctx.save_for_backward(x)
        B, T, D = enc.shape
        cls = torch.empty(B, D, dtype=torch.float32, device=x.device)
        K.copy2d(enc.view(B, T * D)[:, :D], cls)
        return cls, enc

    @staticmethod
    def backward(ctx, dcls, denc):
        (x,) = ctx.saved_tensors
        st = ctx.st
        B, Cc, Lx, N, T, M, D = st['geom'][:7]
        d = torch.zeros(M, D, dtype=torch.float32, device=x.device)
        if denc is not None:
            K.copy2d(denc.reshape(M, D).contiguous(), d)   # (an expanded gradient, e.g. of enc.sum(), has stride 0)
        if dcls is not None:
            K.copy2d(dcls.contiguous(), d.view(B, T * D)[:, :D], beta=1.0)
        grads = _imu_backward(ctx.module, x, st, d)
        ctx.st = None
        return (None, None, None, None) + tuple(grads.get(q) if q.requires_grad else None for q in ctx.params)
