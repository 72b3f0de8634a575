"""Kernel-level parity on the MI355X: every HIP kernel against a plain torch fp32 reference of the same op.

Tolerances are written per test: exact-fp32 kernels ≤ 1e-5 relative; bf16-operand kernels are compared with the
fp32 reference evaluated ON THE SAME bf16-ROUNDED INPUTS, so the only differences are accumulation order
(fp32) and the final bf16 rounding of outputs (≤ 2^-8 relative)."""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = 'cuda'


def K():
    from cmhar import kernels
    return kernels


def L():
    from cmhar import _lib
    return _lib


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _ints(shape, lo=-3, hi=4, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(lo, hi, shape, generator=g).float()


# ---------------------------------------------------------------------------------------------------------------
# GEMM
# ---------------------------------------------------------------------------------------------------------------
def _ref_gemm(layout, a, b):
    a, b = a.float(), b.float()
    if layout == 0:
        return a @ b.T
    if layout == 1:
        return a @ b
    return a.T @ b


def _operands(layout, M, N, Kd, maker, dt):
    if layout == 0:
        a, b = maker((M, Kd), 1), maker((N, Kd), 2)
    elif layout == 1:
        a, b = maker((M, Kd), 1), maker((Kd, N), 2)
    else:
        a, b = maker((Kd, M), 1), maker((Kd, N), 2)
    return a.to(DEV, dt), b.to(DEV, dt)


@pytest.mark.parametrize('layout', [0, 1, 2])
@pytest.mark.parametrize('shape', [(128, 128, 64), (256, 384, 192), (200, 136, 72), (64, 8, 8), (1000, 768, 520),
                                   (256, 256, 64), (512, 768, 256), (1024, 512, 3072)])   # last 3: 256² DMA kernel
def test_gemm_bf16_exact_integers(layout, shape):
    """Small integers are exact in bf16 and their dot products exact in fp32: output must match bit-for-bit.
    Asymmetric operands catch any row/column swap of the C/D layout."""
    M, N, Kd = shape
    a, b = _operands(layout, M, N, Kd, lambda s, sd: _ints(s, seed=sd), torch.bfloat16)
    out = torch.empty(M, N, dtype=torch.float32, device=DEV)
    K().gemm(layout, a, b, out, splits=1)
    torch.cuda.synchronize()
    assert torch.equal(out, _ref_gemm(layout, a, b))


@pytest.mark.parametrize('layout', [0, 1, 2])
def test_gemm_bf16_splitk_exact(layout):
    M, N, Kd = 256, 256, 4096
    a, b = _operands(layout, M, N, Kd, lambda s, sd: _ints(s, -2, 3, seed=sd), torch.bfloat16)
    out = torch.empty(M, N, dtype=torch.float32, device=DEV)
    K().gemm(layout, a, b, out, splits=7)
    assert torch.equal(out, _ref_gemm(layout, a, b))


@pytest.mark.parametrize('layout', [0, 1])
@pytest.mark.parametrize('Kd', [1024, 2048])
def test_gemm_bf16_tail_split_exact(layout, Kd):
    """260 output tiles of 256²: two full chip rounds run whole-K; the last tile rows are split along K and reduced
    with the epilogue (K = 2048; K = 1024 stays one whole-K launch) — bias + residual must land on
    the right rows.  Integer operands: bit-exact."""
    from cmhar import _lib
    M, N = 256 * 130, 512
    assert (_lib.lib().cmhar_gemm_bf16_ws(M, N, Kd) > 0) == (Kd >= 2048)   # K = 1024: plain whole-K launch
    a, b = _operands(layout, M, N, Kd, lambda s, sd: _ints(s, -2, 3, seed=sd), torch.bfloat16)
    bias = _ints((N,), seed=7).to(DEV)
    res = _ints((M, N), seed=8).to(DEV)
    out = torch.empty(M, N, dtype=torch.float32, device=DEV)
    K().gemm(layout, a, b, out, bias=bias, residual=res)
    torch.cuda.synchronize()
    assert torch.equal(out, _ref_gemm(layout, a, b) + bias + res)


def test_gemm_bf16_epilogues():
    torch.manual_seed(0)
    M, N, Kd = 384, 512, 256
    a = torch.randn(M, Kd, device=DEV).bfloat16()
    w = (torch.randn(N, Kd, device=DEV) / 16).bfloat16()
    bias = torch.randn(N, device=DEV)
    res = torch.randn(M, N, device=DEV).bfloat16()
    ref_pre = a.float() @ w.float().T + bias
    # GELU with pre-activation saved
    pre = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    y = K().linear(a, w, bias, act=L().ACT_GELU, aux_out=pre)
    assert rel(pre, ref_pre) < 4e-3
    assert rel(y, torch.nn.functional.gelu(ref_pre)) < 4e-3
    # residual
    y2 = K().linear(a, w, bias, residual=res)
    assert rel(y2, ref_pre + res.float()) < 4e-3
    # rowadd (position table) with modulus
    tab = torch.randn(7, N, device=DEV)
    y3 = K().linear(a, w, bias, rowadd=tab, rowadd_mod=7)
    idx = torch.arange(M, device=DEV) % 7
    assert rel(y3, ref_pre + tab[idx]) < 4e-3
    # dgelu backward epilogue: (dy·W) * gelu'(pre)
    dy = torch.randn(M, N, device=DEV).bfloat16()
    w2 = (torch.randn(N, Kd, device=DEV) / 16).bfloat16()   # [N, K] weight; dgrad output [M, K]
    g_in = torch.randn(M, Kd, device=DEV).bfloat16()
    dx = K().linear_dgrad(dy, w2, act=L().ACT_DGELU, aux_in=g_in)
    xg = g_in.float().requires_grad_(True)
    gl = torch.autograd.grad(torch.nn.functional.gelu(xg), xg, torch.ones_like(xg))[0]
    assert rel(dx, (dy.float() @ w2.float()) * gl) < 4e-3
    # fp32 accumulate (beta = 1)
    acc = torch.randn(N, Kd, device=DEV)
    ref = acc + dy.float().T @ a.float()
    K().linear_wgrad(dy, a, out=acc, beta=1.0)
    assert rel(acc, ref) < 1e-5


def _gelu_ref(x):
    """float64 GELU(erf) and its derivative through erfc (1 + erf(x/√2) cancels to 0 below x ≈ -8.3 even in
    float64, erfc keeps full relative precision)."""
    x64 = x.double()
    cdf = 0.5 * torch.erfc(-x64 / math.sqrt(2))
    return x64 * cdf, cdf + x64 * torch.exp(-0.5 * x64 * x64) / math.sqrt(2 * math.pi)


@pytest.mark.parametrize('shape', [(512, 512, 256), (384, 520, 136)])     # 256-tile DMA kernel and the 128² kernel
def test_gemm_gelu_savegrad_and_mulaux(shape):
    """act 5: out = gelu(a), aux = gelu'(a) from shared transcendentals; act 6: out = acc · aux (the backward).
    Compared against float64 erf-GELU on the same bf16 operands: only bf16 output rounding may differ."""
    torch.manual_seed(3)
    M, N, Kd = shape
    a = torch.randn(M, Kd, device=DEV).bfloat16()
    w = (torch.randn(N, Kd, device=DEV) / 8).bfloat16()
    bias = torch.randn(N, device=DEV)
    pre = a.double() @ w.double().T + bias.double()
    gp = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    y = K().linear(a, w, bias, act=L().ACT_GELU_SAVEGRAD, aux_out=gp)
    g_ref, gp_ref = _gelu_ref(pre)
    assert rel(y, g_ref) < 4e-3 and rel(gp, gp_ref) < 4e-3
    # fp32 output: the formula itself (relative error of erfc < 1.2e-7) — tight
    y32 = torch.empty(M, N, device=DEV)
    gp32 = torch.empty(M, N, device=DEV)
    K().gemm(0, a, w, y32, bias=bias, act=L().ACT_GELU_SAVEGRAD, aux_out=gp32)
    assert rel(y32, g_ref) < 2e-6 and rel(gp32, gp_ref) < 2e-6
    # tail precision on EXACT pre-activations (one-hot rows pick bf16 weights, so the GEMM adds no rounding):
    # the erfc form keeps ~2e-6 relative accuracy down to x = -9, where 1 + erf(x/√2) (torch's fp32 GELU) has
    # already cancelled to percent-level error at x ≈ -5
    Kx = 64
    onehot = torch.zeros(Kx, Kx, device=DEV)
    onehot[torch.arange(Kx), torch.arange(Kx)] = 1.0
    xs = torch.linspace(-9.0, 3.0, 256 * Kx, device=DEV).bfloat16().view(256, Kx)
    yt = torch.empty(Kx, 256, device=DEV)
    gt = torch.empty(Kx, 256, device=DEV)
    K().gemm(0, onehot.bfloat16(), xs, yt, act=L().ACT_GELU_SAVEGRAD, aux_out=gt)
    gx, gpx = _gelu_ref(xs.double().T)
    assert ((yt.double() - gx).abs() <= 2e-5 * gx.abs() + 1e-30).all()
    assert ((gt.double() - gpx).abs() <= 2e-5 * gpx.abs() + 1e-6).all()
    # backward against the saved derivative
    dy = torch.randn(M, N, device=DEV).bfloat16()
    w2 = (torch.randn(N, Kd, device=DEV) / 8).bfloat16()
    aux = torch.randn(M, Kd, device=DEV).bfloat16()
    dx = K().linear_dgrad(dy, w2, act=L().ACT_MULAUX, aux_in=aux)
    assert rel(dx, (dy.float() @ w2.float()) * aux.float()) < 4e-3


@pytest.mark.parametrize('splits', [1, 5])
@pytest.mark.parametrize('beta', [0.0, 1.0])
def test_wgrad_fused_bias_rowsum_exact(splits, beta):
    """The wgrad GEMM's all-ones MFMA row sum (bias gradient) on integer operands: bit-exact, with and without
    split-K, overwrite and accumulate."""
    T, N, Kin = 2048, 768, 512           # dy [T, N], x [T, Kin] → dW [N, Kin], db [N]
    dy = _ints((T, N), seed=4).to(DEV, torch.bfloat16)
    x = _ints((T, Kin), seed=5).to(DEV, torch.bfloat16)
    dw = torch.full((N, Kin), 3.0, device=DEV)
    db = torch.full((N,), 2.0, device=DEV)
    K().gemm(2, dy, x, dw, beta=beta, splits=splits, rowsum=db, rowsum_beta=beta)
    torch.cuda.synchronize()
    assert torch.equal(dw, dy.float().T @ x.float() + 3.0 * beta)
    assert torch.equal(db, dy.float().sum(0) + 2.0 * beta)


def test_wgrad_8phase_bit_identical_to_two_phase(tmp_path):
    """The weight-gradient GEMM on the 8-phase schedule (plans 4 / 6) against the two-phase gemm256_kernel (plans 1 /
    3): same per-output accumulation order, so every dW and fused bias gradient must be bit-identical (worker:
    tests/wgrad8p_worker.py, one process per kernel choice)."""
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

    def run(v):
        out = tmp_path / f'w{v}.pt'
        env = dict(os.environ, CMHAR_GEMM_8P_WGRAD=str(v), CMHAR_AB_OUT=str(out))
        p = subprocess.run([sys.executable, '-u', os.path.join(repo, 'tests', 'wgrad8p_worker.py')], env=env,
                           stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=100)
        assert p.returncode == 0, p.stdout.decode(errors='replace')[-4000:]
        return torch.load(out, weights_only=True)

    a, b = run(1), run(0)
    assert a.keys() == b.keys()
    for k in a:
        if k.startswith('plan'):
            assert a[k].item() in (4, 6) and b[k].item() in (1, 3), (k, a[k].item(), b[k].item())
            continue
        assert torch.isfinite(a[k]).all(), k
        assert torch.equal(a[k], b[k]), (k, (a[k] - b[k]).abs().max().item())


def test_wgrad_bias_fallback_shapes():
    """Shapes off the 256-tile path get the bias gradient from the column-sum kernel instead."""
    torch.manual_seed(5)
    dy = torch.randn(304, 200, device=DEV).bfloat16()
    x = torch.randn(304, 72, device=DEV).bfloat16()
    db = torch.empty(200, device=DEV)
    dw = K().linear_wgrad(dy, x, bias_out=db)
    assert rel(dw, dy.float().T @ x.float()) < 1e-5
    assert rel(db, dy.float().sum(0)) < 1e-5


@pytest.mark.parametrize('layout', [0, 1, 2])
def test_gemm_generic_fp32(layout):
    torch.manual_seed(1)
    M, N, Kd = 173, 91, 67
    a, b = _operands(layout, M, N, Kd, lambda s, sd: torch.randn(s), torch.float32)
    out = torch.empty(M, N, device=DEV)
    K().gemm(layout, a, b, out)
    assert rel(out, _ref_gemm(layout, a, b)) < 1e-6


@pytest.mark.parametrize('layout', [0, 1, 2])
@pytest.mark.parametrize('M,N,Kd', [(32, 768, 768), (32, 512, 768), (7, 300, 1000), (64, 256, 4096)])
def test_gemm_generic_splitk_fp32(layout, M, N, Kd):
    """Skinny fp32 GEMMs take the split-K path (partials + ordered combine with the epilogue): bias, ReLU,
    residual and beta accumulation must land as in the single-pass kernel."""
    from cmhar.kernels import _generic_splits
    assert _generic_splits(M, N, Kd) > 1
    torch.manual_seed(2)
    a, b = _operands(layout, M, N, Kd, lambda s, sd: torch.randn(s), torch.float32)
    bias = torch.randn(N, device=DEV)
    res = torch.randn(M, N, device=DEV)
    out = torch.randn(M, N, device=DEV)
    old = out.clone()
    K().gemm(layout, a, b, out, bias=bias, residual=res, act=L().ACT_RELU, beta=0.5)
    want = torch.relu(_ref_gemm(layout, a, b) + bias) + res + 0.5 * old
    assert rel(out, want) < 3e-6
    out1 = torch.empty(M, N, device=DEV)
    K().gemm(layout, a, b, out1, splits=1)
    assert rel(out1, _ref_gemm(layout, a, b)) < 3e-6


# ---------------------------------------------------------------------------------------------------------------
# attention
# ---------------------------------------------------------------------------------------------------------------
def _attn_ref(q, k, v, B, H, Lq, Lk, D, scale):
    q = q.float().view(B, Lq, H, D).transpose(1, 2)
    k = k.float().view(B, Lk, H, D).transpose(1, 2)
    v = v.float().view(B, Lk, H, D).transpose(1, 2)
    p = torch.softmax(q @ k.transpose(-1, -2) * scale, -1)
    return (p @ v).transpose(1, 2).reshape(B * Lq, H * D)


@pytest.mark.parametrize('L_', [64, 200, 1568])
def test_flash_attention_bf16_fwd_bwd(L_):
    """O, dQ, dK, dV vs torch fp32 autograd, each within 3x the error of the same algorithm with the kernel's bf16
    roundings emulated + 1e-3 (tests/flash_ref.py)."""
    from flash_ref import check_flash
    torch.manual_seed(2)
    B, H, D = 2, 3, 64
    scale = D ** -0.5
    qkv = (torch.randn(B * L_, 3 * H * D, device=DEV) * 1.5).bfloat16()
    q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
    o = torch.empty(B * L_, H * D, dtype=torch.bfloat16, device=DEV)
    lse = torch.empty(B * H * L_, device=DEV)
    K().attention_fwd(q, k, v, o, lse, B=B, H=H, Lq=L_, Lk=L_, D=D, scale=scale)
    do = torch.randn(B * L_, H * D, device=DEV).bfloat16()
    dqkv = torch.empty_like(qkv)
    K().attention_bwd(q, k, v, o, do, lse, dqkv[:, :H * D], dqkv[:, H * D:2 * H * D], dqkv[:, 2 * H * D:],
                      B=B, H=H, Lq=L_, Lk=L_, D=D, scale=scale)
    got = {'o': o, 'dq': dqkv[:, :H * D], 'dk': dqkv[:, H * D:2 * H * D], 'dv': dqkv[:, 2 * H * D:]}
    check_flash(got, q, k, v, do, B=B, H=H, Lq=L_, Lk=L_, D=D, scale=scale)


@pytest.mark.parametrize('Lq,Lk', [(1568, 1568), (129, 257), (32, 200), (1, 64), (300, 33), (26, 3136), (13, 392),
                                   (3136, 3136), (320, 320), (64, 100)])
def test_flash_attention_ragged_tails(Lq, Lk):
    """The split-sequence tail kernels (csrc/attention.hip, tails of <= 64 queries / keys past the last full block, in
    workgroups of 32 rows — 3136 = 12·256 + 64 is the 32-frame geometry):
    forward O, dQ, dK, dV vs torch fp32 autograd within 3x the emulated bf16-rounding error + 1e-3, with the TAIL rows
    checked on their own (a tail bug would hide in a whole-tensor norm), at cross-attention shapes (Lq != Lk)
    including a whole-tail-only sequence (Lq <= 32)."""
    from flash_ref import check_flash
    torch.manual_seed(13)
    B, H, D = 2, 2, 64
    scale = D ** -0.5
    q = (torch.randn(B * Lq, H * D, device=DEV) * 1.5).bfloat16()
    kv = (torch.randn(B * Lk, 2 * H * D, device=DEV) * 1.5).bfloat16()
    k, v = kv[:, :H * D], kv[:, H * D:]
    o = torch.empty(B * Lq, H * D, dtype=torch.bfloat16, device=DEV)
    lse = torch.empty(B * H * Lq, device=DEV)
    K().attention_fwd(q, k, v, o, lse, B=B, H=H, Lq=Lq, Lk=Lk, D=D, scale=scale)
    do = torch.randn(B * Lq, H * D, device=DEV).bfloat16()
    dq = torch.empty_like(q)
    dkv = torch.empty_like(kv)
    K().attention_bwd(q, k, v, o, do, lse, dq, dkv[:, :H * D], dkv[:, H * D:], B=B, H=H, Lq=Lq, Lk=Lk, D=D,
                      scale=scale)
    qt = (Lq // 128) * 128 if Lq % 128 else max(Lq - 128, 0)      # first row of the query tail region
    kt = (Lk // 128) * 128 if Lk % 128 else max(Lk - 128, 0)
    got = {'o': o, 'dq': dq, 'dk': dkv[:, :H * D], 'dv': dkv[:, H * D:]}
    check_flash(got, q, k, v, do, B=B, H=H, Lq=Lq, Lk=Lk, D=D, scale=scale, row_ranges={'q': qt, 'k': kt})


@pytest.mark.parametrize('pattern', ['ramp', 'spikes', 'flat_jump'])
def test_flash_attention_running_max_moves(pattern):
    """The forward's lazy rescale (the running row max moves only when a score exceeds it by 2^8 in p) at inputs that
    make it fire mid-sequence: key norms ramping up along the sequence (the max grows every few tiles), isolated
    large-score spikes late in the sequence, and a tile whose scores all jump by ~4.5 (log2) above the running max
    (many moderate p whose lane sum exceeds 2^8 without any single one doing so).  O, dQ, dK, dV within 3x the
    emulated bf16-rounding error + 1e-3 of fp32 autograd."""
    from flash_ref import check_flash
    torch.manual_seed(21)
    B, H, D, L_ = 2, 2, 64, 700
    scale = D ** -0.5
    q = torch.randn(B * L_, H * D, device=DEV)
    k = torch.randn(B * L_, H * D, device=DEV)
    pos = torch.arange(L_, device=DEV).repeat(B).float()[:, None]
    if pattern == 'ramp':
        k = k * (0.2 + 3.0 * pos / L_)
    elif pattern == 'spikes':
        sel = (pos % 97 == 96) & (pos > 300)
        k = torch.where(sel, q.roll(1, 0) * 4.0, k * 0.5)
    else:
        k = k * 0.1
        q = q.abs() * 0.3
        k = torch.where((pos >= 320) & (pos < 384), k + 2.0, k)     # one whole tile of uniformly higher scores
    q, k = q.bfloat16(), k.bfloat16()
    v = torch.randn(B * L_, H * D, device=DEV).bfloat16()
    o = torch.empty(B * L_, H * D, dtype=torch.bfloat16, device=DEV)
    lse = torch.empty(B * H * L_, device=DEV)
    K().attention_fwd(q, k, v, o, lse, B=B, H=H, Lq=L_, Lk=L_, D=D, scale=scale)
    do = torch.randn(B * L_, H * D, device=DEV).bfloat16()
    dq, dk, dv = (torch.empty_like(q) for _ in range(3))
    K().attention_bwd(q, k, v, o, do, lse, dq, dk, dv, B=B, H=H, Lq=L_, Lk=L_, D=D, scale=scale)
    assert torch.isfinite(o.float()).all()
    check_flash({'o': o, 'dq': dq, 'dk': dk, 'dv': dv}, q, k, v, do, B=B, H=H, Lq=L_, Lk=L_, D=D, scale=scale)


@pytest.mark.parametrize('L_', [200, 1568])
def test_flash_attention_prescaled_keys(L_):
    """The VideoMAE bf16 training form: the QKV GEMM's epilogue writes K pre-scaled by scale·log2(e) (colscale), the
    forward runs with scale = 1/log2(e) and cmhar_attention_bwd_prescaled returns dQ, dV and the gradient of the
    UNSCALED key — vs torch fp32 autograd on the unscaled operands within 3x the emulated bf16-rounding error + 1e-3;
    and the colscale epilogue itself against the unscaled GEMM (same fp32 product, one rounding)."""
    from flash_ref import check_flash
    torch.manual_seed(12)
    B, H, D = 2, 3, 64
    Hd, scale = H * D, D ** -0.5
    c = scale * K().LOG2E
    x = torch.randn(B * L_, 256, device=DEV).bfloat16()
    w = (torch.randn(3 * Hd, 256, device=DEV) * 0.1).bfloat16()
    bias = torch.randn(3 * Hd, device=DEV) * 0.1
    qkv = K().linear(x, w, bias, colscale=(Hd, 2 * Hd, c))
    plain = (x.float() @ w.float().T + bias)
    assert rel(qkv[:, :Hd], plain[:, :Hd]) < 5e-3 and rel(qkv[:, 2 * Hd:], plain[:, 2 * Hd:]) < 5e-3
    assert rel(qkv[:, Hd:2 * Hd], c * plain[:, Hd:2 * Hd]) < 5e-3
    q, kp, v = qkv[:, :Hd], qkv[:, Hd:2 * Hd], qkv[:, 2 * Hd:]
    o = torch.empty(B * L_, Hd, dtype=torch.bfloat16, device=DEV)
    lse = torch.empty(B * H * L_, device=DEV)
    K().attention_fwd(q, kp, v, o, lse, B=B, H=H, Lq=L_, Lk=L_, D=D, scale=1.0 / K().LOG2E)
    do = torch.randn(B * L_, Hd, device=DEV).bfloat16()
    dqkv = torch.empty_like(qkv)
    K().attention_bwd_prescaled(q, kp, v, o, do, lse, dqkv[:, :Hd], dqkv[:, Hd:2 * Hd], dqkv[:, 2 * Hd:],
                                B=B, H=H, Lq=L_, Lk=L_, D=D, scale=scale)
    got = {'o': o, 'dq': dqkv[:, :Hd], 'dk': dqkv[:, Hd:2 * Hd], 'dv': dqkv[:, 2 * Hd:]}
    check_flash(got, q, kp.float() / c, v, do, B=B, H=H, Lq=L_, Lk=L_, D=D, scale=scale)


@pytest.mark.parametrize('D', [16, 64])
def test_attention_fp32_exact(D):
    torch.manual_seed(3)
    B, H, L_ = 3, 2, 13 if D == 16 else 130
    scale = D ** -0.5
    qkv = torch.randn(B * L_, 3 * H * D, device=DEV)
    q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
    o = torch.empty(B * L_, H * D, device=DEV)
    lse = torch.empty(B * H * L_, device=DEV)
    K().attention_fwd(q, k, v, o, lse, B=B, H=H, Lq=L_, Lk=L_, D=D, scale=scale)
    qr, kr, vr = (t.clone().requires_grad_(True) for t in (q, k, v))
    ref = _attn_ref(qr, kr, vr, B, H, L_, L_, D, scale)
    assert rel(o, ref) < 1e-5
    do = torch.randn(B * L_, H * D, device=DEV)
    gq, gk, gv = torch.autograd.grad(ref, (qr, kr, vr), do)
    dq, dk, dv = (torch.empty(B * L_, H * D, device=DEV) for _ in range(3))
    K().attention_bwd(q, k, v, o, do, lse, dq, dk, dv, B=B, H=H, Lq=L_, Lk=L_, D=D, scale=scale)
    assert rel(dq, gq) < 1e-5 and rel(dk, gk) < 1e-5 and rel(dv, gv) < 1e-5


def test_attention_fp32_dropout_consistent():
    """With prob-dropout the kernel computes a fixed (seeded) masked function; its backward must be that
    function's exact gradient: checked against a central finite difference along a random direction."""
    torch.manual_seed(4)
    B, H, L_, D = 2, 2, 13, 16
    p = 0.3
    scale = D ** -0.5
    qkv = torch.randn(B * L_, 3 * H * D, device=DEV)
    q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
    o = torch.empty(B * L_, H * D, device=DEV)
    lse = torch.empty(B * H * L_, device=DEV)
    K().attention_fwd(q, k, v, o, lse, B=B, H=H, Lq=L_, Lk=L_, D=D, scale=scale, pdrop=p, seed=1234)
    # dropout changes the output; without it the kernel is the softmax average
    o0 = torch.empty_like(o)
    K().attention_fwd(q, k, v, o0, lse, B=B, H=H, Lq=L_, Lk=L_, D=D, scale=scale)
    assert rel(o0, _attn_ref(q, k, v, B, H, L_, L_, D, scale)) < 1e-5
    assert rel(o, o0) > 1e-3
    # gradient check by directional finite difference of the (deterministic) masked function
    K().attention_fwd(q, k, v, o, lse, B=B, H=H, Lq=L_, Lk=L_, D=D, scale=scale, pdrop=p, seed=1234)
    do = torch.randn_like(o)
    dq, dk, dv = (torch.empty_like(o) for _ in range(3))
    K().attention_bwd(q, k, v, o, do, lse, dq, dk, dv, B=B, H=H, Lq=L_, Lk=L_, D=D, scale=scale, pdrop=p, seed=1234)
    dirs = [torch.randn_like(o) * 1e-2 for _ in range(3)]
    def f(qq, kk_, vv):
        oo = torch.empty_like(o)
        ll = torch.empty_like(lse)
        K().attention_fwd(qq, kk_, vv, oo, ll, B=B, H=H, Lq=L_, Lk=L_, D=D, scale=scale, pdrop=p, seed=1234)
        return (oo.double() * do.double()).sum().item()
    fd = (f(q + dirs[0], k + dirs[1], v + dirs[2]) - f(q - dirs[0], k - dirs[1], v - dirs[2])) / 2
    an = sum((g.double() * d.double()).sum().item() for g, d in zip((dq, dk, dv), dirs))
    assert abs(fd - an) < 2e-3 * abs(an) + 1e-6


# ---------------------------------------------------------------------------------------------------------------
# norms / small ops
# ---------------------------------------------------------------------------------------------------------------
@pytest.mark.parametrize('dt', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('N', [768, 128, 256, 1024])
def test_layernorm_fwd_bwd(dt, N):
    torch.manual_seed(5)
    M = 333
    x = torch.randn(M, N, device=DEV).to(dt)
    g = 1 + 0.1 * torch.randn(N, device=DEV)
    b = 0.1 * torch.randn(N, device=DEV)
    eps = 1e-12 if N == 768 else 1e-5
    y, mu, rs = K().layernorm_fwd(x, g, b, eps)
    xr = x.float().clone().requires_grad_(True)
    gr, br = g.clone().requires_grad_(True), b.clone().requires_grad_(True)
    ref = torch.nn.functional.layer_norm(xr, (N,), gr, br, eps)
    tol = 1e-5 if dt == torch.float32 else 8e-3
    assert rel(y, ref) < tol
    x64 = x.double()
    assert rel(mu, x64.mean(1)) < 1e-6
    assert rel(rs, 1 / (x64.var(1, unbiased=False) + eps).sqrt()) < 1e-5
    dy = torch.randn(M, N, device=DEV).to(dt)
    dres = torch.randn(M, N, device=DEV).to(dt)
    gx, gg, gb = torch.autograd.grad(ref, (xr, gr, br), dy.float())
    dgam = torch.empty(N, device=DEV)
    dbet = torch.empty(N, device=DEV)
    dx = K().layernorm_bwd(dy, x, g, mu, rs, dgam, dbet, dres=dres)
    assert rel(dx, gx + dres.float()) < (1e-5 if dt == torch.float32 else 1e-2)
    assert rel(dgam, gg) < 1e-4 and rel(dbet, gb) < 1e-5


@pytest.mark.parametrize('shape', [(5000, 300), (20000, 768), (50176, 3072)])
def test_colsum_and_copy(shape):
    torch.manual_seed(6)
    Mr, Nc = shape
    x = torch.randn(Mr, Nc, device=DEV).bfloat16()
    out = torch.full((Nc,), 2.0, device=DEV)
    K().colsum(x, out, beta=1.0)
    assert rel(out, x.float().sum(0) + 2.0) < 1e-5
    y = torch.empty(Mr, Nc, device=DEV)
    K().copy2d(x, y, alpha=0.5)
    assert torch.equal(y, x.float() * 0.5)


def test_batchnorm_relu_l2norm():
    torch.manual_seed(7)
    B, Cc = 32, 512
    x = torch.randn(B, Cc, device=DEV)
    bn = torch.nn.BatchNorm1d(Cc).to(DEV)
    with torch.no_grad():
        bn.weight.normal_(1, 0.1)
        bn.bias.normal_(0, 0.1)
    rm, rv = bn.running_mean.clone(), bn.running_var.clone()
    y, sm, sr = K().batchnorm_fwd(x, bn.weight, bn.bias, rm, rv, True, 0.1, 1e-5, True)
    xr = x.clone().requires_grad_(True)
    ref = torch.relu(bn(xr))
    assert rel(y, ref) < 1e-5
    assert rel(rm, bn.running_mean) < 1e-6 and rel(rv, bn.running_var) < 1e-6
    dy = torch.randn_like(x)
    gx, gw, gb = torch.autograd.grad(ref, (xr, bn.weight, bn.bias), dy)
    dx, dw, db = K().batchnorm_bwd(x, y, dy, bn.weight, sm, sr, True, True)
    assert rel(dx, gx) < 1e-5 and rel(dw, gw) < 1e-5 and rel(db, gb) < 1e-5
    yn, nrm = K().l2normalize_fwd(x)
    xr = x.clone().requires_grad_(True)
    refn = torch.nn.functional.normalize(xr, dim=1)
    assert rel(yn, refn) < 1e-6
    (gn,) = torch.autograd.grad(refn, xr, dy)
    assert rel(K().l2normalize_bwd(yn, dy, nrm), gn) < 1e-5


def test_siglip_loss_matches_reference_formula():
    from cmhar.losses import SigmoidContrastiveLoss
    from fixtures import load
    fx = load('g3_siglip')
    a = torch.tensor(fx['a'], device=DEV, requires_grad=True)
    b = torch.tensor(fx['b'], device=DEV, requires_grad=True)
    lf = SigmoidContrastiveLoss().to(DEV)
    loss = lf(a, b)
    loss.backward()
    assert abs(loss.item() - float(fx['loss'])) < 1e-6
    assert rel(a.grad.cpu(), torch.tensor(fx['grad_a'])) < 1e-5
    assert rel(b.grad.cpu(), torch.tensor(fx['grad_b'])) < 1e-5
    assert abs(lf.temperature.grad.item() - float(fx['grad_temperature'])) < 1e-5 * max(1, abs(float(fx['grad_temperature'])))
    assert abs(lf.bias.grad.item() - float(fx['grad_bias'])) < 1e-6


def test_tubelet_im2col_gemm_equals_conv3d():
    torch.manual_seed(8)
    B, T, Cc, H, W, P, tub, Hd = 2, 4, 3, 32, 48, 16, 2, 64
    video = torch.randn(B, T, Cc, H, W, device=DEV)
    conv = torch.nn.Conv3d(Cc, Hd, (tub, P, P), stride=(tub, P, P)).to(DEV)
    ref = conv(video.permute(0, 2, 1, 3, 4)).flatten(2).transpose(1, 2).reshape(-1, Hd)
    patches = K().tubelet_im2col(video, tub, P, torch.float32)
    out = K().linear(patches, conv.weight.detach().reshape(Hd, -1), conv.bias.detach())
    assert rel(out, ref) < 1e-5


def test_clip_and_fused_adamw_match_torch():
    from cmhar.optim import FusedAdamW, clip_grad_norm_
    torch.manual_seed(9)
    shapes = [(300, 77), (1000,), (3, 5, 7), (65536 + 17,)]
    ps = [torch.randn(s, device=DEV) for s in shapes]
    ours = [torch.nn.Parameter(p.clone()) for p in ps]
    theirs = [torch.nn.Parameter(p.clone()) for p in ps]
    opt_a = FusedAdamW(ours, lr=1e-3, weight_decay=0.01)
    opt_b = torch.optim.AdamW(theirs, lr=1e-3, weight_decay=0.01)
    for step in range(3):
        for a, b in zip(ours, theirs):
            g = torch.randn_like(a) * (10 if step == 0 else 0.01)
            a.grad, b.grad = g.clone(), g.clone()
        na = clip_grad_norm_(ours, 1.0)
        nb = torch.nn.utils.clip_grad_norm_(theirs, 1.0)
        assert abs(na.item() - nb.item()) < 1e-5 * nb.item()
        opt_a.step()
        opt_b.step()
    for a, b in zip(ours, theirs):
        assert (a - b).abs().max().item() < 1e-6
        assert rel(opt_a.state[a]['exp_avg_sq'], opt_b.state[b]['exp_avg_sq']) < 1e-6


@pytest.mark.parametrize('write_grad', [True, False])
def test_fused_adamw_folded_clip_bit_identical(write_grad):
    """FusedAdamW(max_grad_norm=1.0) (the clip coefficient applied inside the AdamW pass) against clip_grad_norm_ +
    FusedAdamW.step: bit-identical parameters, moments and bf16 shadows; `.grad` afterwards is the clipped gradient
    (write_clipped_grad=True) or left unclipped (False).  Covers the vectorised body, ragged tails and parameters
    whose storage is not 16-B aligned (views at odd offsets: the scalar path)."""
    from cmhar.optim import FusedAdamW, clip_grad_norm_
    torch.manual_seed(11)
    flat = torch.randn(4096 + 3, device=DEV)
    base = [torch.randn(s, device=DEV) for s in [(300, 77), (1000,), (3, 5, 7), (65536 + 17,)]] + \
        [flat[1:1 + 999].view(999), flat[1003:1003 + 2048].view(32, 64)]
    ours = [torch.nn.Parameter(p.clone()) for p in base[:4]] + [torch.nn.Parameter(p) for p in base[4:]]
    flat2 = flat.clone()
    theirs = [torch.nn.Parameter(p.clone()) for p in base[:4]] + \
        [torch.nn.Parameter(flat2[1:1 + 999].view(999)), torch.nn.Parameter(flat2[1003:1003 + 2048].view(32, 64))]
    assert ours[4].data_ptr() % 16 != 0
    opt_a = FusedAdamW(ours, lr=1e-3, weight_decay=0.01, max_grad_norm=1.0, write_clipped_grad=write_grad)
    opt_b = FusedAdamW(theirs, lr=1e-3, weight_decay=0.01)
    for step in range(3):
        grads = [torch.randn_like(a) * (10 if step != 1 else 0.01) for a in ours]
        for a, b, g in zip(ours, theirs, grads):
            a.grad, b.grad = g.clone(), g.clone()
        opt_a.step()
        nb = clip_grad_norm_(theirs, 1.0)
        opt_b.step()
        assert opt_a.last_grad_norm.item() == nb.item()
        for a, b, g in zip(ours, theirs, grads):
            assert torch.equal(a.grad, b.grad if write_grad else g)
    for a, b in zip(ours, theirs):
        assert torch.equal(a, b)
        assert torch.equal(opt_a.state[a]['exp_avg'], opt_b.state[b]['exp_avg'])
        assert torch.equal(opt_a.state[a]['exp_avg_sq'], opt_b.state[b]['exp_avg_sq'])


@pytest.mark.parametrize('D', [16, 32])
def test_attention_bf16_storage_small_head(D):
    """bf16 tensors with a head dim the flash kernel does not cover run the exact-math path on bf16 storage."""
    torch.manual_seed(10)
    B, H, L_ = 2, 4, 37
    scale = D ** -0.5
    qkv = torch.randn(B * L_, 3 * H * D, device=DEV).bfloat16()
    q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
    o = torch.empty(B * L_, H * D, dtype=torch.bfloat16, device=DEV)
    lse = torch.empty(B * H * L_, device=DEV)
    K().attention_fwd(q, k, v, o, lse, B=B, H=H, Lq=L_, Lk=L_, D=D, scale=scale)
    qr, kr, vr = (t.float().clone().requires_grad_(True) for t in (q, k, v))
    ref = _attn_ref(qr, kr, vr, B, H, L_, L_, D, scale)
    assert rel(o, ref) < 8e-3
    do = torch.randn(B * L_, H * D, device=DEV).bfloat16()
    gq, gk, gv = torch.autograd.grad(ref, (qr, kr, vr), do.float())
    dq, dk, dv = (torch.empty_like(o) for _ in range(3))
    K().attention_bwd(q, k, v, o, do, lse, dq, dk, dv, B=B, H=H, Lq=L_, Lk=L_, D=D, scale=scale)
    assert rel(dq, gq) < 1e-2 and rel(dk, gk) < 1e-2 and rel(dv, gv) < 1e-2


@pytest.mark.parametrize('write_grad', [True, False])
def test_fused_adamw_clip_params_beyond_owned(write_grad):
    """`clip_params` (the trainers pass model.parameters(), as trainer.py:140/304 clip over them) enter the
    norm even when the optimizer does not own them, and their `.grad` is clipped like clip_grad_norm_ leaves it —
    also with write_clipped_grad=False (another optimizer may step them); the owned parameters' update
    is bit-identical to clip_grad_norm_(all) + step."""
    from cmhar.optim import FusedAdamW, clip_grad_norm_
    torch.manual_seed(12)
    base = [torch.randn(s, device=DEV) for s in [(300, 77), (1000,), (3, 5, 7), (4099,)]]
    ours = [torch.nn.Parameter(p.clone()) for p in base]
    theirs = [torch.nn.Parameter(p.clone()) for p in base]
    opt_a = FusedAdamW(ours[:2], lr=1e-3, weight_decay=0.01, max_grad_norm=1.0, clip_params=ours,
                       write_clipped_grad=write_grad)
    opt_b = FusedAdamW(theirs[:2], lr=1e-3, weight_decay=0.01)
    for step in range(2):
        grads = [torch.randn_like(a) * 10 for a in ours]
        for a, b, g in zip(ours, theirs, grads):
            a.grad, b.grad = g.clone(), g.clone()
        opt_a.step()
        nb = clip_grad_norm_(theirs, 1.0)
        opt_b.step()
        assert opt_a.last_grad_norm.item() == nb.item()
        for a, b in zip(ours if write_grad else ours[2:], theirs if write_grad else theirs[2:]):
            assert torch.equal(a.grad, b.grad)
    for a, b in zip(ours, theirs):
        assert torch.equal(a, b)


def test_mfma_peak_probe():
    """csrc/probe.hip (the on-box MFMA peak bench.py reports as roofline.peak_measured): a plausible dense bf16 rate
    per shape — above 1400 TF/s (the chip lowers its clock under dense MFMA load on random data; the 8-chain probe read
    1480-1832 TF/s on 32x32x16 and 1736-1971 on 16x16x32 across the round-4 boxes, so 1400 is ~0.8x the lowest) and
    below the 2.5 PF vendor peak."""
    import bench
    shapes = {}
    tf = bench.measure_mfma_peak(torch.device(DEV), blocks=1024, iters=4000, reps=2, per_shape=shapes)
    print(f'MFMA peak probe: {tf:.1f} TFLOP/s', shapes)
    assert set(shapes) == {'32x32x16', '16x16x32'} and tf == max(shapes.values())
    for v in shapes.values():       # DVFS: random-data MFMA loops hold ≈1.9 GHz (MICROARCH DVFS give-back)
        assert 1400.0 < v < 2500.0, shapes


def test_packed_weights_transposed_copies():
    """PackedWeights(transpose=True): cmhar_mt_transpose_bf16 builds Wᵀ of every pack in one launch (ragged 64-tile
    edges included), rebuilt only after the shadows change (FusedAdamW.mark_fresh / a version-triggered cast)."""
    from cmhar.weights import PackedWeights
    torch.manual_seed(14)
    ps = [torch.nn.Parameter(torch.randn(s, device=DEV)) for s in [(200, 72), (136, 72), (64, 520), (768, 768)]]
    pk = PackedWeights(DEV, torch.bfloat16)
    pk.add_weight('a', ps[:2], transpose=True)
    pk.add_weight('b', [ps[2]], transpose=True)
    pk.add_weight('c', [ps[3]])
    pk.build()
    pk.refresh(force=True)
    ta, tb = pk.transposed('a'), pk.transposed('b')
    assert pk.transposed('c') is None
    assert torch.equal(ta, pk['a'].t()) and torch.equal(tb, pk['b'].t())
    assert torch.equal(ta, torch.cat([ps[0], ps[1]]).detach().bfloat16().t())
    with torch.no_grad():
        ps[2].mul_(-2.0)
    pk.refresh()
    assert torch.equal(pk.transposed('b'), (ps[2].detach() * 1.0).bfloat16().t())


def test_videomae_dgrad_transposed_weights_match_dgrad_layout(tmp_path):
    """The VideoMAE backward's input-gradient GEMMs on the transposed weight copies (forward layout, default) against
    the dgrad layout (CMHAR_DGRAD_WT=0), two processes on the same seeded bf16 model (full 12-layer backbone at a small
    clip, incl. the token-0 last layer): every parameter gradient within 1e-3 relative of the other (the two layouts
    order the K accumulation differently inside an MFMA step; same fp32 products, one bf16 rounding each)."""
    import subprocess
    import sys
    import os
    script = r'''
import os, sys, torch
sys.path[:0] = [os.environ["REPO"], os.path.join(os.environ["REPO"], "crossmodal-imu-video-ood-har_amd")]
from cmhar.videomae import VideoMAEBackbone, default_videomae_config, run_backbone
cfg = default_videomae_config(image_size=64, num_frames=4)
torch.manual_seed(0)
m = VideoMAEBackbone(cfg, compute_dtype="bf16").cuda().train()
x = torch.randn(8, 4, 3, 64, 64, device="cuda")
out = run_backbone(m, x, token0_only=True)
g = torch.randn_like(out.float())
(out.float() * g).sum().backward()
torch.save({n: p.grad.cpu() for n, p in m.named_parameters()}, sys.argv[1])
'''
    outs = []
    for v in ('1', '0'):
        f = tmp_path / f'g{v}.pt'
        env = dict(os.environ, CMHAR_DGRAD_WT=v, REPO=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        r = subprocess.run([sys.executable, '-c', script, str(f)], env=env, capture_output=True, text=True, timeout=200)
        assert r.returncode == 0, r.stderr[-3000:]
        outs.append(torch.load(f, weights_only=True))
    worst = max(rel(outs[0][n], outs[1][n]) for n in outs[0] if outs[1][n].norm() > 0)
    print('worst rel diff transposed vs dgrad layout:', worst)
    assert worst < 1e-3, worst
