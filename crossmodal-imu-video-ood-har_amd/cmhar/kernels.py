"""Tensor-level wrappers over the cmhar C ABI.

Every wrapper validates shapes, strides, dtypes and alignment on the host BEFORE launching (a malformed launch
of a hand-written kernel can fault the GPU), passes raw device pointers + the caller's current HIP stream, and
raises on any non-zero return code.  No wrapper has a torch fallback.
"""
from __future__ import annotations

import ctypes as C
import math
import os

import torch

from . import _lib as L
from ._lib import call, ptr

# ------------------------------------------------------------------------------------------------------------
# optional launch tracer: HIP events recorded on the launching stream around selected kernels (bench.py uses it
# to measure the dominant kernel's average duration live over the timed region)
# ------------------------------------------------------------------------------------------------------------
class Tracer:
    def __init__(self):
        self.active = False
        self.only = None       # optional set of kernel symbols to time (None = all)
        self.records = []      # (kernel symbol, flops, bytes, start_event, end_event)

    def begin(self, name=None):
        if not self.active or (self.only is not None and name not in self.only):
            return None
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        return ev

    def end(self, ev0, name, flops, nbytes):
        if ev0 is None:
            return
        ev1 = torch.cuda.Event(enable_timing=True)
        ev1.record()
        self.records.append((name, flops, nbytes, ev0, ev1))

    def summary(self):
        """{symbol: (launches, total_ms, total_flops, total_bytes)} — call after synchronising."""
        out = {}
        for name, fl, nb, e0, e1 in self.records:
            n, ms, f, b = out.get(name, (0, 0.0, 0, 0))
            out[name] = (n + 1, ms + e0.elapsed_time(e1), f + fl, b + nb)
        return out


TRACE = Tracer()

_GEMM_SYMBOL = {0: 'gemm_bf16_kernel<true,true,{o}>', 1: 'gemm_bf16_kernel<true,false,{o}>',
                2: 'gemm_bf16_kernel<false,false,{o}>'}
_PLAN = {}


def _gemm_trace_name(layout, M, N, K, s, has_ws, rowsum, out_dtype, reads=False):
    """Trace label of a bf16 GEMM call: the GEMM kernel (template name as rocprofv3 lists it, without the trailing
    integer parameters) that the library's own plan (cmhar_gemm_bf16_plan2; reads: an epilogue the persistent forward
    kernel does not take) launches; a split-K / tail reduce that follows it is launched outside the traced interval."""
    key = (layout, M, N, K, s, has_ws, rowsum)
    plan = L.lib().cmhar_gemm_bf16_plan2(layout, M, N, K, s, int(has_ws), int(rowsum), int(reads))
    _PLAN[key] = plan
    o = 'float' if (plan in (3, 5, 6) or out_dtype == torch.float32) else 'bf16'
    if plan == 7:
        return f'gemm8p_persist_kernel<{o}>'
    if plan in (4, 6):
        ak, bk = layout != 2, layout == 0
        return f'gemm8p_kernel<{str(ak).lower()},{str(bk).lower()},{o}>'
    name = _GEMM_SYMBOL[layout].format(o=o)
    if plan in (1, 2, 3):
        name = name.replace('gemm_bf16_kernel', 'gemm256_kernel')
    return name


def _gemm_has_reduce(layout, M, N, K, s, has_ws, rowsum):
    """Whether the call's plan ends with a split-K / tail reduce launch (plans 2, 3, 5, 6)."""
    return _PLAN[(layout, M, N, K, s, has_ws, rowsum)] in (2, 3, 5, 6)

# ------------------------------------------------------------------------------------------------------------
# workspaces (one growing fp32 buffer per (device, stream))
# ------------------------------------------------------------------------------------------------------------
_WS = {}


def workspace(nfloats: int, device) -> torch.Tensor:
    st = torch.cuda.current_stream(device)
    key = (str(device), st.cuda_stream)
    buf = _WS.get(key)
    if buf is None or buf.numel() < nfloats:
        buf = torch.empty(max(int(nfloats), 1 << 16), dtype=torch.float32, device=device)
        _WS[key] = buf
    return buf


def _check_2d(t, name):
    if t.dim() != 2:
        raise ValueError(f'{name}: expected a 2-D matrix, got {tuple(t.shape)}')
    if t.stride(1) != 1:
        raise ValueError(f'{name}: inner dimension must be contiguous (stride {t.stride()})')
    if not t.is_cuda:
        raise ValueError(f'{name}: must be a device tensor')


def _check_bf16_operand(t, name):
    if t.data_ptr() % 16 or t.stride(0) % 8:
        raise ValueError(f'{name}: bf16 MFMA operands need 16-B aligned rows (ptr {t.data_ptr() % 16}, '
                         f'ld {t.stride(0)})')


def _splits_for(M, N, K):
    """Split-K factor so that small-output / long-K GEMMs (the weight gradients: K = B·L tokens) fill the 256 CUs.
    Mirrors the library's kernel choice: 256² tiles (one 512-thread workgroup per CU) when M, N % 256 == 0 and
    K % 64 == 0, else 128² tiles (two per CU)."""
    big = M % 256 == 0 and N % 256 == 0 and K % 64 == 0
    if big:
        tiles, slots = (M // 256) * (N // 256), 256
    else:
        tiles, slots = math.ceil(M / 128) * math.ceil(N / 128), 512
    if tiles * 3 >= slots * 2 or K < 1024:
        return 1
    return max(1, min(32, round(slots / tiles), K // 512))


_TAIL_WS = {}


_NO_GENERIC_SPLIT = os.environ.get('CMHAR_GENERIC_SPLIT', '1') == '0'    # A/B knob (debug)


def _generic_splits(M, N, K):
    """Split-K factor for the fp32 LDS-tiled GEMM: one row of 64² tiles (M <= 64: the video projection and the
    projection heads at M = batch rows) over K >= 512 leaves most CUs idle and the K loop latency-bound; aim at ~128
    workgroups with >= 64 k per slice.  The IMU encoder's token GEMMs (M = 13·batch) keep the single-pass order:
    their backward through post-LN layers amplifies summation-order differences (measured: split-K moved g1's
    bias gradients by up to 9e-4 relative, deterministically, vs 1e-6 single-pass)."""
    if _NO_GENERIC_SPLIT:
        return 1
    if M >= 256 and N >= 256 and K >= 4096:
        # fp32 weight gradients of the VideoMAE Linears (M, N = 768..3072, K = tokens): 36-144 tiles of 128² on the
        # f32 MFMA kernel (3 workgroups per CU = 768 slots); split K into slices of >= 512 so that the grid fills
        # the slots once (not 1.05 times: a second, nearly empty round)
        tiles = math.ceil(M / 128) * math.ceil(N / 128)
        return 1 if tiles >= 384 else max(1, min(32, 768 // tiles, K // 512))
    tiles = math.ceil(M / 64) * math.ceil(N / 64)
    if M > 64 or N < 256 or tiles >= 64 or K < 512:
        return 1
    return max(1, min(32, math.ceil(128 / tiles), K // 64))


# Plain library GEMMs on hipBLASLt (`cmhar_blaslt_linear`): the forward-layout bf16 / fp16 shapes listed in CMHAR_BLASLT
# ("N,K" pairs separated by ';'; empty = none), with at most a bias and a residual in the epilogue and at least 4096
# rows.  Default: the N = 768 launches of the VideoMAE step — attention output projection forward and input gradient
# (768,768), FC2 forward and FC1 input gradient (768,3072), QKV input gradient (768,2304), the token-0 layer's K|V
# input gradient (768,1536).  There 588 tiles of 256² fall on 256 CUs as 2.3 rounds; the hand-written kernels split
# the last round along K (+ a reduce launch) or run it a third full, the vendor's stream-K kernel balances 196
# workgroups of exactly 3 tiles.  Measured (round 6, tools/debug/blaslt_ab.sh, one box, alternated): bench step
# 735.2 / 727.2 clips/s hand-written, 754.4 / 757.4 with this list (profiles/r06_blaslt_ab.log).  The hand-written
# plans stay for every other shape and caller (and for these with CMHAR_BLASLT="").
_BLASLT = {tuple(int(v) for v in t.split(',')) for t in
           os.environ.get('CMHAR_BLASLT', '768,768;768,3072;768,2304;768,1536').split(';') if t.strip()}


_BLASLT_OK = {}


def _blaslt_route(layout, M, N, K, a, b, out, bias, residual, aux_in, aux_out, rowadd, act, alpha, beta, splits,
                  pdrop, rowsum, colscale, reduce_stream):
    if not _BLASLT or layout != 0 or (N, K) not in _BLASLT or M < 4096 or out.dtype != a.dtype:
        return False
    if (aux_in is not None or aux_out is not None or rowadd is not None or act != L.ACT_NONE or alpha != 1.0 or
            beta != 0.0 or splits is not None or pdrop > 0.0 or rowsum is not None or colscale is not None or
            reduce_stream is not None):
        return False
    if residual is not None and residual.stride(1) != 1:
        return False
    # the library must have an algorithm for this exact call (planned once per shape / strides / epilogue); where it
    # has none the hand-written kernels take the call
    key = (L.dtype_code(a.dtype), M, N, K, a.stride(0), b.stride(0), out.stride(0), bias is not None,
           residual is not None, residual.stride(0) if residual is not None else 0)
    ok = _BLASLT_OK.get(key)
    if ok is None:
        ok = _BLASLT_OK[key] = bool(L.lib().cmhar_blaslt_linear_ok(*key[:7], int(key[7]), int(key[8]), key[9]))
    return ok


def _tail_ws(M, N, K):
    key = (M, N, K)
    v = _TAIL_WS.get(key)
    if v is None:
        v = _TAIL_WS[key] = int(L.lib().cmhar_gemm_bf16_ws(M, N, K))
    return v


# ------------------------------------------------------------------------------------------------------------
# GEMM: C = A·B in one of three layouts (see include/cmhar.h)
# ------------------------------------------------------------------------------------------------------------
def gemm(layout: int, a: torch.Tensor, b: torch.Tensor, out: torch.Tensor, *, bias=None, residual=None,
         aux_in=None, aux_out=None, rowadd=None, rowadd_mod=1, act=L.ACT_NONE, alpha=1.0, beta=0.0, splits=None,
         pdrop=0.0, seed=0, rowsum=None, rowsum_beta=0.0, colscale=None, reduce_stream=None):
    """layout 0: out[M,N] = a[M,K]·b[N,K]ᵀ;  1: a[M,K]·b[K,N];  2: a[K,M]ᵀ·b[K,N].
    rowsum (layout 2, bf16, 256-tile shapes): rowsum[m] = Σ_k a[k,m] + rowsum_beta·rowsum[m] (bias gradient).
    colscale (lo, hi, s): columns [lo, hi) (multiples of 8) of the product + bias scaled by s before the activation.
    reduce_stream (bf16 split-K plans): the split-K reduce (which writes `out` / `rowsum`) runs on that stream, after
    the GEMM kernel, from a partial-slab buffer of its own; the caller orders its readers of `out` after that stream."""
    for t, n in ((a, 'A'), (b, 'B'), (out, 'C')):
        _check_2d(t, n)
    if layout == 0:
        M, K = a.shape
        N = b.shape[0]
        ok = b.shape[1] == K
    elif layout == 1:
        M, K = a.shape
        N = b.shape[1]
        ok = b.shape[0] == K
    elif layout == 2:
        K, M = a.shape
        N = b.shape[1]
        ok = b.shape[0] == K
    else:
        raise ValueError(layout)
    if not ok or tuple(out.shape) != (M, N):
        raise ValueError(f'gemm layout {layout}: shapes A{tuple(a.shape)} B{tuple(b.shape)} C{tuple(out.shape)}')
    if a.dtype != b.dtype:
        raise TypeError('A and B must share a dtype')
    for t, n in ((bias, 'bias'), (rowadd, 'rowadd')):
        if t is not None and (t.dtype != torch.float32 or not t.is_contiguous() and t.dim() == 1):
            raise TypeError(f'{n} must be fp32')
    if bias is not None and bias.numel() != N:
        raise ValueError('bias length')
    for t, n in ((residual, 'residual'), (aux_in, 'aux_in'), (aux_out, 'aux_out')):
        if t is not None:
            _check_2d(t, n)
            if tuple(t.shape) != (M, N) or t.dtype != out.dtype:
                raise ValueError(f'{n} must be [{M},{N}] {out.dtype}')
    if rowadd is not None and (rowadd.dim() != 2 or rowadd.shape[1] != N or rowadd.stride(1) != 1):
        raise ValueError('rowadd must be [mod, N]')
    if beta != 0.0 and out.dtype != torch.float32:
        raise ValueError('beta accumulation only for fp32 outputs')
    if rowsum is not None:
        if not rowsum_supported(layout, a.dtype, M, N, K):
            raise ValueError('rowsum needs the bf16 256-tile weight-gradient path')
        if rowsum.dtype != torch.float32 or rowsum.numel() != M or not rowsum.is_contiguous():
            raise ValueError(f'rowsum must be a contiguous fp32 [{M}] tensor')
    if colscale is not None and (colscale[0] % 8 or colscale[1] % 8 or not 0 <= colscale[0] <= colscale[1] <= N):
        raise ValueError('colscale columns must be a multiple-of-8 range inside [0, N]')
    epi = L.epilogue(bias, residual, aux_in, aux_out, rowadd, rowadd_mod, act, alpha, beta, pdrop, seed, rowsum,
                     rowsum_beta, colscale)
    st = L.stream(out.device)
    if a.dtype in (torch.bfloat16, torch.float16) and _blaslt_route(layout, M, N, K, a, b, out, bias, residual, aux_in,
                                                                     aux_out, rowadd, act, alpha, beta, splits, pdrop,
                                                                     rowsum, colscale, reduce_stream):
        ev = TRACE.begin('hipblaslt_linear') if TRACE.active else None
        call('cmhar_blaslt_linear', L.dtype_code(a.dtype), M, N, K, ptr(a), a.stride(0), ptr(b), b.stride(0), ptr(out),
             out.stride(0), ptr(bias), ptr(residual), residual.stride(0) if residual is not None else 0, st)
        extra = out.element_size() * M * N if residual is not None else 0
        TRACE.end(ev, 'hipblaslt_linear', 2 * M * N * K, 2 * (M * K + N * K) + out.element_size() * M * N + extra)
        return out
    if a.dtype == torch.float16:
        # fp16 inference path (BASELINE config 5): the bf16 kernels on the fp16 MFMA, forward layout only
        if layout != 0 or rowsum is not None:
            raise ValueError('fp16 GEMM: forward layout 0 only (inference path)')
        _check_bf16_operand(a, 'A')
        _check_bf16_operand(b, 'B')
        if K % 8:
            raise ValueError('fp16 GEMM needs K to be a multiple of 8')
        if out.dtype not in (torch.float16, torch.float32):
            raise TypeError('fp16 GEMM output must be fp16 or fp32')
        s = 1 if splits is None else splits
        ws = workspace(s * M * N, out.device) if s > 1 else None
        if s == 1 and splits is None:
            n = _tail_ws(M, N, K)
            if n:
                ws = workspace(n, out.device)
        call('cmhar_gemm_f16', layout, L.dtype_code(out.dtype), M, N, K, ptr(a), a.stride(0), ptr(b), b.stride(0),
             ptr(out), out.stride(0), C.byref(epi), s, ptr(ws), st)
        return out
    if a.dtype == torch.bfloat16:
        _check_bf16_operand(a, 'A')
        _check_bf16_operand(b, 'B')
        if K % 8 or (layout >= 1 and N % 8) or (layout == 2 and M % 8):
            raise ValueError('bf16 GEMM needs K (and the row-contraction operand widths) to be multiples of 8')
        if out.dtype not in (torch.bfloat16, torch.float32):
            raise TypeError('out dtype')
        s = _splits_for(M, N, K) if splits is None else splits
        ws = None
        if s > 1 and reduce_stream is not None:
            # slabs of their own (the stream-ordered caching allocator keeps them until the reduce stream is done)
            ws = torch.empty(s * M * N + (s * M if rowsum is not None else 0), dtype=torch.float32, device=out.device)
        elif s > 1:
            ws = workspace(s * M * N + (s * M if rowsum is not None else 0), out.device)
        elif splits is None and rowsum is None:
            n = _tail_ws(M, N, K)
            if n:
                ws = workspace(n, out.device)
        ev = name = None
        if TRACE.active:
            # an epilogue the persistent forward kernel does not take (the library's epi_persist_ok)
            pok = (alpha == 1.0 and pdrop <= 0.0 and rowadd is None and beta == 0.0 and
                   ((act == L.ACT_NONE and aux_in is None) or
                    (act == L.ACT_GELU_SAVEGRAD and aux_out is not None and residual is None and aux_in is None) or
                    (act == L.ACT_MULAUX and aux_in is not None and residual is None)))
            name = _gemm_trace_name(layout, M, N, K, s, ws is not None, rowsum is not None, out.dtype, not pok)
            ev = TRACE.begin(name)
        if ev is None and reduce_stream is not None and s > 1:
            args = (layout, L.dtype_code(out.dtype), M, N, K, ptr(a), a.stride(0), ptr(b), b.stride(0), ptr(out),
                    out.stride(0), C.byref(epi), s, ptr(ws))
            call('cmhar_gemm_bf16_phased', *args, st, 1)
            reduce_stream.wait_stream(torch.cuda.current_stream(out.device))
            call('cmhar_gemm_bf16_phased', *args, reduce_stream.cuda_stream, 2)
            ws.record_stream(reduce_stream)
        elif ev is None:
            call('cmhar_gemm_bf16', layout, L.dtype_code(out.dtype), M, N, K, ptr(a), a.stride(0), ptr(b),
                 b.stride(0), ptr(out), out.stride(0), C.byref(epi), s, ptr(ws), st)
        else:
            # traced: the GEMM kernel alone between the events (phase 1), then its split-K / tail reduce (phase 2)
            args = (layout, L.dtype_code(out.dtype), M, N, K, ptr(a), a.stride(0), ptr(b), b.stride(0), ptr(out),
                    out.stride(0), C.byref(epi), s, ptr(ws), st)
            call('cmhar_gemm_bf16_phased', *args, 1)
            # algorithmic bytes: operands once + output once + every epilogue tensor (residual / aux in / aux out)
            extra = sum(t.element_size() * M * N for t in (residual, aux_in, aux_out) if t is not None)
            TRACE.end(ev, name, 2 * M * N * K, 2 * (M * K + N * K) + out.element_size() * M * N + extra)
            if _gemm_has_reduce(layout, M, N, K, s, ws is not None, rowsum is not None):
                call('cmhar_gemm_bf16_phased', *args, 2)
    else:
        if layout == 0:
            sam, sak, sbk, sbn = a.stride(0), 1, 1, b.stride(0)
        elif layout == 1:
            sam, sak, sbk, sbn = a.stride(0), 1, b.stride(0), 1
        else:
            sam, sak, sbk, sbn = 1, a.stride(0), b.stride(0), 1
        s = _generic_splits(M, N, K) if splits is None else splits
        if s > 1:
            ws = workspace(s * M * N, out.device)
            call('cmhar_gemm_generic_splitk', L.dtype_code(a.dtype), L.dtype_code(out.dtype), M, N, K, s, ptr(a), sam,
                 sak, ptr(b), sbk, sbn, ptr(out), out.stride(0), C.byref(epi), ptr(ws), st)
        else:
            call('cmhar_gemm_generic', L.dtype_code(a.dtype), L.dtype_code(out.dtype), M, N, K, 1, ptr(a), sam, sak,
                 0, ptr(b), sbk, sbn, 0, ptr(out), out.stride(0), 0, C.byref(epi), st)
    return out


def linear(x, w, bias=None, *, residual=None, act=L.ACT_NONE, aux_out=None, rowadd=None, rowadd_mod=1,
           out=None, out_dtype=None, pdrop=0.0, seed=0, colscale=None):
    """y = dropout(act(x·wᵀ + bias [+ rowadd])) [+ residual]  — nn.Linear forward (+ fused activation)."""
    M, N = x.shape[0], w.shape[0]
    if out is None:
        out = torch.empty(M, N, dtype=out_dtype or x.dtype, device=x.device)
    return gemm(0, x, w, out, bias=bias, residual=residual, act=act, aux_out=aux_out, rowadd=rowadd,
                rowadd_mod=rowadd_mod, pdrop=pdrop, seed=seed, colscale=colscale)


def linear_dgrad(dy, w, *, act=L.ACT_NONE, aux_in=None, residual=None, out=None, beta=0.0, pdrop=0.0, seed=0):
    """dx = (dy·w) [* dropmask] [* act'(aux_in)] [+ residual]."""
    M, K = dy.shape[0], w.shape[1]
    if out is None:
        out = torch.empty(M, K, dtype=dy.dtype, device=dy.device)
    return gemm(1, dy, w, out, act=act, aux_in=aux_in, residual=residual, beta=beta, pdrop=pdrop, seed=seed)


def rowsum_supported(layout, dtype, M, N, K):
    return layout == 2 and dtype == torch.bfloat16 and M % 256 == 0 and N % 256 == 0 and K % 64 == 0


def linear_wgrad(dy, x, *, out=None, beta=0.0, bias_out=None, bias_beta=0.0, reduce_stream=None):
    """dW[N,K] (fp32) = dyᵀ·x;  bias_out[N] (fp32, optional) = Σ_m dy[m, :] (+ bias_beta·bias_out).
    The bias gradient rides on the wgrad GEMM's own MFMA operand tiles when the shape allows it, else it is a
    separate column-sum launch.  reduce_stream: see gemm()."""
    N, K = dy.shape[1], x.shape[1]
    if out is None:
        out = torch.empty(N, K, dtype=torch.float32, device=dy.device)
    if bias_out is not None and not rowsum_supported(2, dy.dtype, N, K, dy.shape[0]):
        colsum(dy, bias_out, beta=bias_beta)
        bias_out = None
    return gemm(2, dy, x, out, beta=beta, rowsum=bias_out, rowsum_beta=bias_beta, reduce_stream=reduce_stream)


def colsum(x, out=None, *, alpha=1.0, beta=0.0):
    """out[n] (fp32) = alpha Σ_m x[m, n] + beta out[n]  — bias gradients."""
    _check_2d(x, 'x')
    M, N = x.shape
    if out is None:
        out = torch.empty(N, dtype=torch.float32, device=x.device)
    n = L.lib().cmhar_colsum_ws(M, N)
    ws = workspace(n, x.device)
    call('cmhar_colsum', L.dtype_code(x.dtype), M, N, ptr(x), x.stride(0), ptr(out), alpha, beta, ptr(ws), ws.numel(),
         L.stream(x.device))
    return out


# ------------------------------------------------------------------------------------------------------------
# attention
# ------------------------------------------------------------------------------------------------------------
def _head_view_ok(t, B, L_, H, D, name):
    _check_2d(t, name)
    if t.shape[0] != B * L_ or t.shape[1] < H * D:
        raise ValueError(f'{name}: expected [{B * L_}, >={H * D}] got {tuple(t.shape)}')


def attention_fwd(q, k, v, out, lse, *, B, H, Lq, Lk, D, scale, pdrop=0.0, seed=0):
    for t, n, Lx in ((q, 'q', Lq), (k, 'k', Lk), (v, 'v', Lk), (out, 'o', Lq)):
        _head_view_ok(t, B, Lx, H, D, n)
    if lse.numel() < B * H * Lq or lse.dtype != torch.float32:
        raise ValueError('lse workspace')
    dt = L.dtype_code(q.dtype)
    if D not in (8, 16, 32, 64):
        raise ValueError(f'head dim {D} not supported')
    if dt in (L.BF16, L.F16) and D == 64 and pdrop == 0.0:     # flash (MFMA) path: 16-B aligned rows
        for t, n in ((q, 'q'), (k, 'k'), (v, 'v'), (out, 'o')):
            _check_bf16_operand(t, n)
    ev = TRACE.begin('attn_fwd_bf16') if (dt == L.BF16 and D == 64 and pdrop == 0.0) else None
    call('cmhar_attention_fwd', dt, B, H, Lq, Lk, D, ptr(q), q.stride(0), ptr(k), k.stride(0), ptr(v), v.stride(0),
         ptr(out), out.stride(0), ptr(lse), scale, pdrop, seed, L.stream(q.device))
    TRACE.end(ev, 'attn_fwd_bf16', 4 * B * H * Lq * Lk * D, 2 * (B * Lq + 2 * B * Lk + B * Lq) * H * D)
    return out


def attention_fwd_opt(mode=-1):
    """The bf16 / fp16 flash forward's bulk launch mode: 1 = optimistic running max + exact rerun of the workgroups
    whose rows left its range (default), 0 = one exact lazy-rescale launch; mode < 0 only queries.  Returns the
    previous mode (`cmhar_attention_fwd_opt`)."""
    return L.lib().cmhar_attention_fwd_opt(int(mode))


def attention_bwd(q, k, v, o, do, lse, dq, dk, dv, *, B, H, Lq, Lk, D, scale, pdrop=0.0, seed=0):
    for t, n, Lx in ((q, 'q', Lq), (k, 'k', Lk), (v, 'v', Lk), (o, 'o', Lq), (do, 'do', Lq), (dq, 'dq', Lq),
                     (dk, 'dk', Lk), (dv, 'dv', Lk)):
        _head_view_ok(t, B, Lx, H, D, n)
    dt = L.dtype_code(q.dtype)
    if D not in (8, 16, 32, 64):
        raise ValueError(f'head dim {D} not supported')
    if dt == L.F16:
        raise ValueError('fp16 is the inference-only path: no attention backward')
    flash = dt == L.BF16 and D == 64 and pdrop == 0.0
    if flash:
        for t, n in ((q, 'q'), (k, 'k'), (v, 'v'), (o, 'o'), (do, 'do'), (dq, 'dq'), (dk, 'dk'), (dv, 'dv')):
            _check_bf16_operand(t, n)
    delta = workspace(B * H * Lq, q.device)
    ev = TRACE.begin('attn_bwd_bf16(dq+delta,dkdv)') if flash else None
    call('cmhar_attention_bwd', dt, B, H, Lq, Lk, D, ptr(q), q.stride(0), ptr(k), k.stride(0), ptr(v), v.stride(0),
         ptr(o), o.stride(0), ptr(do), do.stride(0), ptr(lse), ptr(delta), ptr(dq), dq.stride(0), ptr(dk),
         dk.stride(0), ptr(dv), dv.stride(0), scale, pdrop, seed, L.stream(q.device))
    TRACE.end(ev, 'attn_bwd_bf16(dq+delta,dkdv)', 14 * B * H * Lq * Lk * D, 2 * (6 * B * Lq + 4 * B * Lk) * H * D)


LOG2E = 1.4426950408889634


def attention_bwd_prescaled(q, k, v, o, do, lse, dq, dk, dv, *, B, H, Lq, Lk, D, scale):
    """Backward of bf16 flash attention whose keys were written pre-scaled by scale·log2(e) (linear(..., colscale))
    and whose forward ran with scale = 1/log2(e): dq, dv and dk (gradient of the UNSCALED key) for the true `scale`."""
    for t, n, Lx in ((q, 'q', Lq), (k, 'k', Lk), (v, 'v', Lk), (o, 'o', Lq), (do, 'do', Lq), (dq, 'dq', Lq),
                     (dk, 'dk', Lk), (dv, 'dv', Lk)):
        _head_view_ok(t, B, Lx, H, D, n)
        _check_bf16_operand(t, n)
    if q.dtype != torch.bfloat16 or D != 64:
        raise ValueError('pre-scaled attention backward: bf16, head dim 64')
    delta = workspace(B * H * Lq, q.device)
    ev = TRACE.begin('attn_bwd_bf16(dq+delta,dkdv)')
    call('cmhar_attention_bwd_prescaled', B, H, Lq, Lk, ptr(q), q.stride(0), ptr(k), k.stride(0), ptr(v), v.stride(0),
         ptr(o), o.stride(0), ptr(do), do.stride(0), ptr(lse), ptr(delta), ptr(dq), dq.stride(0), ptr(dk),
         dk.stride(0), ptr(dv), dv.stride(0), scale, L.stream(q.device))
    TRACE.end(ev, 'attn_bwd_bf16(dq+delta,dkdv)', 14 * B * H * Lq * Lk * D, 2 * (6 * B * Lq + 4 * B * Lk) * H * D)


# ------------------------------------------------------------------------------------------------------------
# norms
# ------------------------------------------------------------------------------------------------------------
def layernorm_fwd(a, gamma, beta, eps, *, b=None, pdrop=0.0, seed=0, h_out=None, out=None, mean=None, rstd=None):
    _check_2d(a, 'a')
    M, N = a.shape
    if N > 1024:
        raise ValueError('LayerNorm width > 1024')
    if out is None:
        out = torch.empty_like(a, memory_format=torch.contiguous_format)
    if mean is None:
        mean = torch.empty(M, dtype=torch.float32, device=a.device)
    if rstd is None:
        rstd = torch.empty(M, dtype=torch.float32, device=a.device)
    if b is not None and (tuple(b.shape) != (M, N) or b.dtype != a.dtype):
        raise ValueError('b shape')
    call('cmhar_layernorm_fwd', L.dtype_code(a.dtype), M, N, ptr(a), a.stride(0), ptr(b),
         b.stride(0) if b is not None else 0, pdrop, seed, ptr(h_out), h_out.stride(0) if h_out is not None else 0,
         ptr(out), out.stride(0), ptr(gamma), ptr(beta), ptr(mean), ptr(rstd), eps, L.stream(a.device))
    return out, mean, rstd


def layernorm_bwd(dy, h, gamma, mean, rstd, dgamma, dbeta, *, dres=None, dh=None, db_out=None, pdrop=0.0, seed=0,
                  beta_acc=0.0):
    M, N = h.shape
    if dh is None:
        dh = torch.empty_like(h, memory_format=torch.contiguous_format)
    n = L.lib().cmhar_layernorm_bwd_ws(M, N)
    ws = workspace(n, h.device)
    call('cmhar_layernorm_bwd', L.dtype_code(h.dtype), M, N, ptr(dy), dy.stride(0), ptr(h), h.stride(0), ptr(gamma),
         ptr(mean), ptr(rstd), ptr(dres), dres.stride(0) if dres is not None else 0, ptr(dh), dh.stride(0),
         ptr(db_out), db_out.stride(0) if db_out is not None else 0, pdrop, seed, ptr(dgamma), ptr(dbeta), beta_acc,
         ptr(ws), L.stream(h.device))
    return dh


def batchnorm_fwd(x, w, b, rmean, rvar, training, momentum, eps, relu, num_batches_tracked=None):
    B, Cc = x.shape
    y = torch.empty_like(x)
    sm = torch.empty(Cc, dtype=torch.float32, device=x.device)
    sr = torch.empty(Cc, dtype=torch.float32, device=x.device)
    call('cmhar_batchnorm_fwd', B, Cc, ptr(x), ptr(y), ptr(w), ptr(b), ptr(rmean), ptr(rvar), ptr(sm), ptr(sr),
         int(training), momentum, eps, int(relu), ptr(num_batches_tracked), L.stream(x.device))
    return y, sm, sr


def batchnorm_bwd(x, y, dy, w, sm, sr, training, relu):
    B, Cc = x.shape
    dx = torch.empty_like(x)
    dw = torch.empty(Cc, dtype=torch.float32, device=x.device)
    db = torch.empty(Cc, dtype=torch.float32, device=x.device)
    call('cmhar_batchnorm_bwd', B, Cc, ptr(x), ptr(y), ptr(dy.contiguous()), ptr(w), ptr(sm), ptr(sr), ptr(dx),
         ptr(dw), ptr(db), int(training), int(relu), 0.0, L.stream(x.device))
    return dx, dw, db


def l2normalize_fwd(x, eps=1e-12):
    M, N = x.shape
    y = torch.empty_like(x)
    nrm = torch.empty(M, dtype=torch.float32, device=x.device)
    call('cmhar_l2normalize_fwd', M, N, ptr(x), ptr(y), ptr(nrm), eps, L.stream(x.device))
    return y, nrm


def l2normalize_bwd(y, dy, nrm, eps=1e-12):
    M, N = y.shape
    dx = torch.empty_like(y)
    call('cmhar_l2normalize_bwd', M, N, ptr(y), ptr(dy.contiguous()), ptr(nrm), ptr(dx), eps, L.stream(y.device))
    return dx


def copy2d(src, dst, alpha=1.0, beta=0.0, pdrop=0.0, seed=0):
    """dst = alpha * src * dropmask + beta * dst (casts / gathers / adds / dropout)."""
    _check_2d(src, 'src')
    _check_2d(dst, 'dst')
    if src.shape != dst.shape:
        raise ValueError('copy2d shape')
    call('cmhar_copy2d', L.dtype_code(src.dtype), L.dtype_code(dst.dtype), src.shape[0], src.shape[1], ptr(src),
         src.stride(0), ptr(dst), dst.stride(0), alpha, beta, pdrop, seed, L.stream(src.device))
    return dst


_REDUCTIONS = {'none': 0, 'mean': 1, 'sum': 2}


def cross_entropy(logits, labels=None, *, ignore_index=-100, label_smoothing=0.0, gamma=0.0, alpha=1.0,
                  reduction='mean', loss=None, row_loss=None, pred=None, correct=None, status=None, dlogits=None,
                  grad_scale=1.0, grad_beta=0.0, g_up=None):
    """Row-softmax cross-entropy family on a (possibly transposed) fp32 logit view [N, C] — see include/cmhar.h.
    labels: int64 device [N] or None (= arange, InfoNCE).  dlogits may have its own strides (e.g. a transposed
    view accumulated with grad_beta = 1)."""
    if logits.dim() != 2 or logits.dtype != torch.float32 or not logits.is_cuda:
        raise ValueError('logits: fp32 device matrix expected')
    N, Cc = logits.shape
    if labels is not None and (labels.dtype != torch.int64 or labels.shape != (N,) or not labels.is_contiguous()):
        raise ValueError(f'labels: contiguous int64 [{N}] expected')
    for t, n in ((row_loss, 'row_loss'), (pred, 'pred')):
        if t is not None and (t.numel() != N or not t.is_contiguous()):
            raise ValueError(f'{n}: [{N}] expected')
    if dlogits is not None and (tuple(dlogits.shape) != (N, Cc) or dlogits.dtype != torch.float32):
        raise ValueError('dlogits shape')
    red = _REDUCTIONS[reduction]
    if dlogits is not None and red == 0 and (g_up is None or g_up.numel() != N):
        raise ValueError("reduction='none' needs per-row upstream gradients")
    ws = workspace(L.lib().cmhar_cross_entropy_ws(N), logits.device)
    call('cmhar_cross_entropy', N, Cc, ptr(logits), logits.stride(0), logits.stride(1), ptr(labels), ignore_index,
         label_smoothing, gamma, alpha, red, ptr(loss), ptr(row_loss), ptr(pred), ptr(correct), ptr(status),
         ptr(dlogits), dlogits.stride(0) if dlogits is not None else 0,
         dlogits.stride(1) if dlogits is not None else 0, grad_scale, grad_beta, ptr(g_up), ptr(ws),
         L.stream(logits.device))


def tubelet_im2col(video, tub, P, out_dtype):
    if video.dtype != torch.float32 or video.dim() != 5 or not video.is_contiguous():
        raise ValueError('video must be a contiguous fp32 (B,T,C,H,W) tensor')
    B, T, Cc, H, W = video.shape
    if T % tub or H % P or W % P or P % 8:
        raise ValueError(f'video {tuple(video.shape)} incompatible with tubelet {tub} patch {P}')
    Lt = (T // tub) * (H // P) * (W // P)
    out = torch.empty(B * Lt, Cc * tub * P * P, dtype=out_dtype, device=video.device)
    call('cmhar_tubelet_im2col', L.dtype_code(out_dtype), B, T, Cc, H, W, tub, P, ptr(video), ptr(out),
         L.stream(video.device))
    return out


def ptr_array(tensors):
    arr = (C.c_void_p * len(tensors))(*[t.data_ptr() for t in tensors])
    return arr
