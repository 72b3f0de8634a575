"""`cmhar_blaslt_linear` (csrc/blaslt.hip): the plain library GEMM on hipBLASLt, out = A·Bᵀ (+ fp32 bias) (+ bf16
residual), at the production N = 768 shapes the `CMHAR_BLASLT` routing may send to it (attention output projection
forward with bias + residual, its input gradient on Wᵀ without an epilogue, FC2 forward / FC1 input gradient at
K = 3072) and at a small ragged M.
* integer operands (exact in bf16; products and sums exact in fp32): bit-exact against the fp64 product + epilogue
  rounded to bf16 — the epilogue order does not matter when every partial sum is exact;
* random bf16 operands: ≤ 4e-3 relative against torch fp32 (the output's bf16 rounding), and ≤ 1 bf16 ulp away from
  the hand-written kernel's result on the same operands for ≥ 99.9 % of the elements;
* the `kernels.gemm` routing: with CMHAR_BLASLT naming the shape, the call lands on hipBLASLt (traced label) and
  matches the hand-written plan within the same bound."""
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


def blaslt(a, b, out, bias=None, residual=None):
    L().call('cmhar_blaslt_linear', L().dtype_code(a.dtype), a.shape[0], b.shape[0], a.shape[1], a.data_ptr(),
             a.stride(0), b.data_ptr(), b.stride(0), out.data_ptr(), out.stride(0), L().ptr(bias), L().ptr(residual),
             residual.stride(0) if residual is not None else 0, L().stream())
    return out


def ref64(a, b, bias, residual):
    r = a.double() @ b.double().t()
    if bias is not None:
        r = r + bias.double()
    if residual is not None:
        r = r + residual.double()
    return r


@pytest.mark.parametrize('M,N,Kd,use_bias,use_res', [
    (50176, 768, 768, True, True),      # out-proj forward
    (50176, 768, 768, False, False),    # out-proj input gradient on Wᵀ
    (50176, 768, 3072, True, True),     # FC2 forward
    (50176, 768, 3072, False, False),   # FC1 input gradient on W1ᵀ
    (4100, 768, 768, True, False),      # ragged rows
])
def test_blaslt_linear_integer_exact(M, N, Kd, use_bias, use_res):
    g = torch.Generator(device=DEV).manual_seed(M + Kd)
    a = torch.randint(-4, 5, (M, Kd), generator=g, device=DEV).to(torch.bfloat16)
    b = torch.randint(-4, 5, (N, Kd), generator=g, device=DEV).to(torch.bfloat16)
    bias = torch.randint(-64, 65, (N,), generator=g, device=DEV).float() if use_bias else None
    res = torch.randint(-64, 65, (M, N), generator=g, device=DEV).to(torch.bfloat16) if use_res else None
    out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    blaslt(a, b, out, bias, res)
    torch.cuda.synchronize()
    exp = ref64(a, b, bias, res).to(torch.bfloat16)
    assert torch.equal(out, exp)


@pytest.mark.parametrize('N,Kd', [(768, 768), (768, 3072)])
def test_blaslt_linear_random_vs_fp32_and_hand_kernel(N, Kd):
    M = 50176
    g = torch.Generator(device=DEV).manual_seed(7 + Kd)
    a = (torch.randn(M, Kd, generator=g, device=DEV) * 0.5).to(torch.bfloat16)
    b = (torch.randn(N, Kd, generator=g, device=DEV) / Kd ** 0.5).to(torch.bfloat16)
    bias = torch.randn(N, generator=g, device=DEV) * 0.1
    res = torch.randn(M, N, generator=g, device=DEV).to(torch.bfloat16)
    out = blaslt(a, b, torch.empty(M, N, dtype=torch.bfloat16, device=DEV), bias, res)
    hand = torch.empty_like(out)
    k = K()
    saved = set(k._BLASLT)
    k._BLASLT.clear()
    try:
        k.gemm(0, a, b, hand, bias=bias, residual=res)
    finally:
        k._BLASLT.update(saved)
    torch.cuda.synchronize()
    ref = a.float() @ b.float().t() + bias + res.float()
    err = ((out.float() - ref).norm() / ref.norm()).item()
    assert err <= 4e-3, err
    # ≤ 1 bf16 ulp from the hand-written kernel almost everywhere (two fp32 summation orders, one rounding each)
    ulp = torch.clamp(hand.float().abs(), min=2.0 ** -30) * 2.0 ** -7
    far = ((out.float() - hand.float()).abs() > ulp).float().mean().item()
    assert far <= 1e-3, far


def test_gemm_routes_listed_shape_to_blaslt():
    k = K()
    M, N, Kd = 8192, 768, 768
    g = torch.Generator(device=DEV).manual_seed(3)
    a = torch.randn(M, Kd, generator=g, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, Kd, generator=g, device=DEV) / Kd ** 0.5).to(torch.bfloat16)
    bias = torch.randn(N, generator=g, device=DEV)
    res = torch.randn(M, N, generator=g, device=DEV).to(torch.bfloat16)
    saved = set(k._BLASLT)
    k._BLASLT.clear()
    hand = k.linear(a, w, bias, residual=res)
    k._BLASLT.add((N, Kd))
    k.TRACE.records, k.TRACE.only, k.TRACE.active = [], None, True
    try:
        lt = k.linear(a, w, bias, residual=res)
        torch.cuda.synchronize()
        names = {r[0] for r in k.TRACE.records}
    finally:
        k.TRACE.active = False
        k.TRACE.records = []
        k._BLASLT.clear()
        k._BLASLT.update(saved)
    assert names == {'hipblaslt_linear'}
    ref = a.float() @ w.float().t() + bias + res.float()
    assert ((lt.float() - ref).norm() / ref.norm()).item() <= 4e-3
    assert ((lt.float() - hand.float()).norm() / hand.float().norm()).item() <= 4e-3


def test_default_routing_list():
    """The default routing list is the step's N = 768 launches (cmhar/kernels.py), and a shape with an epilogue the
    library call does not take (GELU, row add) stays on the hand-written kernels."""
    import os
    k = K()
    if 'CMHAR_BLASLT' not in os.environ:
        assert k._BLASLT == {(768, 768), (768, 3072), (768, 2304), (768, 1536)}
    out = torch.empty(8192, 768, dtype=torch.bfloat16, device=DEV)
    args = dict(out=out, bias=None, residual=None, aux_in=None, aux_out=None, rowadd=None, alpha=1.0, beta=0.0,
                splits=None, pdrop=0.0, rowsum=None, colscale=None, reduce_stream=None)
    saved = set(k._BLASLT)
    k._BLASLT.add((768, 768))
    try:
        a = torch.empty(8192, 768, dtype=torch.bfloat16, device=DEV)
        w = torch.empty(768, 768, dtype=torch.bfloat16, device=DEV)
        assert k._blaslt_route(0, 8192, 768, 768, a, w, act=k.L.ACT_NONE, **args)
        assert not k._blaslt_route(0, 8192, 768, 768, a, w, act=k.L.ACT_GELU, **args)
        assert not k._blaslt_route(1, 8192, 768, 768, a, w, act=k.L.ACT_NONE, **args)
        assert not k._blaslt_route(0, 1024, 768, 768, a, w, act=k.L.ACT_NONE, **args)
        # out bf16, A fp16
        assert not k._blaslt_route(0, 8192, 768, 768, a.half(), w.half(), act=k.L.ACT_NONE, **args)
        args['rowadd'] = torch.zeros(1, 768, device=DEV)
        assert not k._blaslt_route(0, 8192, 768, 768, a, w, act=k.L.ACT_NONE, **args)
    finally:
        k._BLASLT.clear()
        k._BLASLT.update(saved)


@pytest.mark.parametrize('use_bias,use_res', [(True, True), (False, False)])
def test_blaslt_linear_fp16(use_bias, use_res):
    """fp16 operands / output (the config-5 inference path's N = 768 launches): integer operands bit-exact vs fp64,
    random operands ≤ 1e-3 relative vs fp32 (fp16 output rounding, 2^-11)."""
    M, N, Kd = 50176, 768, 768
    g = torch.Generator(device=DEV).manual_seed(11)
    a = torch.randint(-4, 5, (M, Kd), generator=g, device=DEV).half()
    b = torch.randint(-4, 5, (N, Kd), generator=g, device=DEV).half()
    bias = torch.randint(-64, 65, (N,), generator=g, device=DEV).float() if use_bias else None
    res = torch.randint(-64, 65, (M, N), generator=g, device=DEV).half() if use_res else None
    out = blaslt(a, b, torch.empty(M, N, dtype=torch.float16, device=DEV), bias, res)
    torch.cuda.synchronize()
    assert torch.equal(out, ref64(a, b, bias, res).half())
    a = (torch.randn(M, Kd, generator=g, device=DEV) * 0.5).half()
    b = (torch.randn(N, Kd, generator=g, device=DEV) / Kd ** 0.5).half()
    if use_res:
        res = torch.randn(M, N, generator=g, device=DEV).half()
    out = blaslt(a, b, torch.empty(M, N, dtype=torch.float16, device=DEV), bias, res)
    torch.cuda.synchronize()
    ref = a.float() @ b.float().t() + (bias if bias is not None else 0) + (res.float() if res is not None else 0)
    assert ((out.float() - ref).norm() / ref.norm()).item() <= 1e-3
