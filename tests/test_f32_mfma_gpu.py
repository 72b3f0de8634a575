"""The exact-fp32 parity mode's GEMMs on the f32 MFMA.

`v_mfma_f32_32x32x2_f32` is bitwise the k-ordered fmaf chain, which is exactly what the VALU kernel computes, so
moving a GEMM between the two kernels must not change one bit: the worker (tests/f32_gemm_worker.py) runs the same
seeded GEMMs — three layouts, ragged M/N/K, every epilogue kind the path uses, split-K slices with a short tail, a
z-batched bf16-output call — once per kernel (CMHAR_F32_MFMA=1 / 0, read once per process), and the outputs are
compared with torch.equal.  A second test holds the MFMA kernel to an fp64 product at the fp32 rounding bound.
"""
import os
import subprocess
import sys

import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(tmp_path, mfma):
    out = tmp_path / f'ab{mfma}.pt'
    env = dict(os.environ, CMHAR_F32_MFMA=str(mfma), CMHAR_AB_OUT=str(out))
    p = subprocess.run([sys.executable, '-u', os.path.join(REPO, 'tests', 'f32_gemm_worker.py')], env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=100)
    assert p.returncode == 0, p.stdout.decode(errors='replace')[-4000:]
    return torch.load(out, weights_only=True)


@pytest.mark.gpu
def test_f32_mfma_gemm_bit_identical_to_valu_chain(tmp_path):
    a, b = _worker(tmp_path, 1), _worker(tmp_path, 0)
    assert a.keys() == b.keys()
    for k in a:
        assert torch.isfinite(a[k].float()).all(), k
        assert torch.equal(a[k], b[k]), (k, (a[k].float() - b[k].float()).abs().max().item())


@pytest.mark.gpu
@pytest.mark.parametrize('layout', [0, 1, 2])
def test_f32_mfma_gemm_vs_fp64(layout):
    from cmhar import kernels as K
    dev = torch.device('cuda')
    g = torch.Generator(device=dev).manual_seed(layout)
    M, N, Kd = 1100, 1300, 6000
    a = torch.randn((M, Kd) if layout < 2 else (Kd, M), device=dev, generator=g)
    b = torch.randn((N, Kd) if layout == 0 else (Kd, N), device=dev, generator=g)
    c = torch.empty(M, N, device=dev)
    K.gemm(layout, a, b, c)
    a64, b64 = a.double(), b.double()
    am = a64 if layout < 2 else a64.t()
    bm = b64.t() if layout == 0 else b64
    ref = am @ bm
    mag = am.abs() @ bm.abs()
    # a k-ordered f32 chain: |err| <= ~K·2^-24·Σ|a·b| worst case; random signs give ~sqrt(K)·2^-24·Σ|a·b|
    err = ((c.double() - ref).abs() / mag).max().item()
    assert err < 4e-6, err


def _attn_ref64(q, k, v, do, B, H, Lq, Lk, D, scale):
    """fp64 softmax(scale·QKᵀ)V, its natural-log LSE and the three input gradients for [B*L, H*D] row layouts."""
    def heads(t, L_):
        return t.double().view(B, L_, H, D).transpose(1, 2)
    Q, K_, V = heads(q, Lq), heads(k, Lk), heads(v, Lk)
    Q.requires_grad_(True)
    K_.requires_grad_(True)
    V.requires_grad_(True)
    S = (Q @ K_.transpose(-1, -2)) * scale
    lse = torch.logsumexp(S, -1)
    O = torch.softmax(S, -1) @ V
    O.backward(heads(do, Lq))
    back = lambda t, L_: t.transpose(1, 2).reshape(B * L_, H * D)  # noqa: E731
    return back(O.detach(), Lq), lse.detach().reshape(-1), back(Q.grad, Lq), back(K_.grad, Lk), back(V.grad, Lk)


@pytest.mark.gpu
@pytest.mark.parametrize('B,H,Lq,Lk', [(2, 3, 1568, 1568), (1, 2, 300, 200), (2, 1, 13, 1568), (1, 2, 1568, 45),
                                       (1, 1, 129, 64)])
def test_f32_mfma_flash_attention_vs_fp64(B, H, Lq, Lk):
    """The f32-MFMA flash kernels (csrc/attention_f32.hip): forward O / LSE and backward dQ dK dV against fp64, on
    the VideoMAE geometry (1568 tokens, head dim 64) and ragged query / key counts (partial 32-row blocks, 64-row
    tiles, 128-row workgroups).  Bound: 2e-5 of each output's max magnitude — the exact-f32 VALU kernels' own error
    is ~1e-6 at these sizes; f32 rounding of the ~L-term sums allows a few e-6."""
    from cmhar import kernels as K
    dev = torch.device('cuda')
    g = torch.Generator(device=dev).manual_seed(Lq * 7 + Lk)
    D = 64
    scale = D ** -0.5
    q = torch.randn(B * Lq, H * D, device=dev, generator=g) * 2
    k = torch.randn(B * Lk, H * D, device=dev, generator=g) * 2
    v = torch.randn(B * Lk, H * D, device=dev, generator=g)
    do = torch.randn(B * Lq, H * D, device=dev, generator=g)
    o = torch.empty_like(q)
    lse = torch.empty(B * H * Lq, device=dev)
    K.attention_fwd(q, k, v, o, lse, B=B, H=H, Lq=Lq, Lk=Lk, D=D, scale=scale)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    K.attention_bwd(q, k, v, o, do, lse, dq, dk, dv, B=B, H=H, Lq=Lq, Lk=Lk, D=D, scale=scale)
    torch.cuda.synchronize()
    ro, rl, rq, rk, rv = _attn_ref64(q, k, v, do, B, H, Lq, Lk, D, scale)
    for name, got, ref in (('O', o, ro), ('lse', lse, rl), ('dQ', dq, rq), ('dK', dk, rk), ('dV', dv, rv)):
        err = ((got.double() - ref).abs().max() / ref.abs().max()).item()
        assert err < 2e-5, (name, err)
