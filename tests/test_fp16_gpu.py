"""fp16 inference path (BASELINE config 5: "fp16 inference-only"; reference hook `Evaluator.predict`,
src/eval/evaluator.py:28-53) on the MI355X.

Kernels: the forward GEMM on the fp16 MFMA is bit-exact on small-integer operands (exact in fp16, dot products exact
in fp32) on every plan it can take (8-phase 256², tail split, 128² ragged), and within fp16 output rounding
(2^-11 relative) with the fused epilogues; flash attention forward vs a torch fp32 softmax(QKᵀ)V on the same
fp16-rounded inputs.  Model: VideoMAE-B at the metric geometry vs the reference's golden vector (g5, fp32 reference)
at a tolerance that reflects fp16's 10-bit mantissa through 12 layers (bf16's 7-bit mantissa: 6e-2); the tiny
CrossModalModel (g2) forward; training in fp16 is refused."""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def rel(a, b):
    a = torch.as_tensor(a).float().cpu()
    b = torch.as_tensor(np.asarray(b) if not torch.is_tensor(b) else b).float().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _ints(shape, lo=-3, hi=4, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(lo, hi, shape, generator=g).float()


@pytest.mark.parametrize('shape,plan', [((512, 768, 768), 4),          # 8-phase 256² forward kernel
                                        ((256 * 130, 512, 2048), 2),   # 256² + tail split + reduce
                                        ((1024, 256, 3072), 4),        # 8-phase, K = 3072 (FC2 shape class)
                                        ((200, 136, 72), 0)])          # 128² ragged (bounds-checked loads)
@pytest.mark.parametrize('out', ['fp32', 'fp16'])
def test_gemm_f16_exact_integers(shape, plan, out):
    from cmhar import _lib, kernels as K
    M, N, Kd = shape
    a = _ints((M, Kd), seed=1).to(DEV, torch.float16)
    b = _ints((N, Kd), seed=2).to(DEV, torch.float16)
    bias = _ints((N,), seed=3).to(DEV)
    has_ws = _lib.lib().cmhar_gemm_bf16_ws(M, N, Kd) > 0
    assert _lib.lib().cmhar_gemm_bf16_plan(0, M, N, Kd, 1, int(has_ws), 0) == plan
    odt = torch.float32 if out == 'fp32' else torch.float16
    y = torch.empty(M, N, dtype=odt, device=DEV)
    K.gemm(0, a, b, y, bias=bias)
    torch.cuda.synchronize()
    ref = a.float() @ b.float().T + bias
    if out == 'fp32':
        assert torch.equal(y, ref)
    else:
        assert torch.equal(y, ref.half())      # |values| < 2048: exact in fp16 too


def test_gemm_f16_epilogues():
    """GELU (+ pre-activation), residual and the sinusoid rowadd of the tubelet embedding, fp16 output."""
    from cmhar import _lib as L, kernels as K
    torch.manual_seed(0)
    M, N, Kd = 512, 768, 256
    a = torch.randn(M, Kd, device=DEV).half()
    w = (torch.randn(N, Kd, device=DEV) / 16).half()
    bias = torch.randn(N, device=DEV)
    res = torch.randn(M, N, device=DEV).half()
    pre_ref = a.float() @ w.float().T + bias
    y = K.linear(a, w, bias, act=L.ACT_GELU)
    assert y.dtype == torch.float16
    assert rel(y, torch.nn.functional.gelu(pre_ref)) < 1e-3
    y2 = K.linear(a, w, bias, residual=res)
    assert rel(y2, pre_ref + res.float()) < 1e-3
    tab = torch.randn(7, N, device=DEV)
    y3 = K.linear(a, w, bias, rowadd=tab, rowadd_mod=7)
    assert rel(y3, pre_ref + tab[torch.arange(M, device=DEV) % 7]) < 1e-3


def test_gemm_f16_rejects_backward_layouts():
    from cmhar import kernels as K
    a = torch.zeros(256, 256, dtype=torch.float16, device=DEV)
    with pytest.raises(ValueError):
        K.gemm(1, a, a, torch.empty(256, 256, device=DEV))
    with pytest.raises(ValueError):
        K.gemm(2, a, a, torch.empty(256, 256, device=DEV))


@pytest.mark.parametrize('Lq,Lk', [(1568, 1568), (392, 392), (13, 1568), (300, 200)])
def test_flash_attention_f16_forward(Lq, Lk):
    from cmhar import kernels as K
    torch.manual_seed(0)
    B, H, D = 2, 3, 64
    q = torch.randn(B * Lq, H * D, device=DEV).half()
    k = torch.randn(B * Lk, H * D, device=DEV).half()
    v = torch.randn(B * Lk, H * D, device=DEV).half()
    o = torch.empty(B * Lq, H * D, dtype=torch.float16, device=DEV)
    lse = torch.empty(B * H * Lq, device=DEV)
    scale = D ** -0.5
    K.attention_fwd(q, k, v, o, lse, B=B, H=H, Lq=Lq, Lk=Lk, D=D, scale=scale)
    qh = q.float().view(B, Lq, H, D).transpose(1, 2)
    kh = k.float().view(B, Lk, H, D).transpose(1, 2)
    vh = v.float().view(B, Lk, H, D).transpose(1, 2)
    s = qh @ kh.transpose(-1, -2) * scale
    ref = (torch.softmax(s, -1) @ vh).transpose(1, 2).reshape(B * Lq, H * D)
    assert rel(o, ref) < 2e-3                 # P and O rounded to fp16 (2^-11), fp32 accumulation
    lse_ref = torch.logsumexp(s, -1).reshape(-1) / math.log(2) + 0.0
    # kernel LSE is log2-domain of (scale·log2e)·s: log2(Σ exp2(c·s)) = logsumexp(s·scale)/ln 2
    assert torch.allclose(lse, lse_ref, atol=1e-3, rtol=1e-4)


def test_videomae_base_full_geometry_f16():
    """g5 (reference VideoMAE-B fp32, 16×224², 1568 tokens, 12 layers) through the fp16 inference path."""
    from fixtures import fixture_state_dict, load
    from seeded import seeded_input
    from cmhar.config import Config
    from cmhar.models import VideoEncoder
    fx = load('g5_videomae_base_16x224')
    cfg = Config()
    cfg.model.video_backbone = '/nonexistent/videomae-local'
    cfg.model.compute_dtype = 'fp16'
    torch.manual_seed(0)
    with pytest.warns(UserWarning):
        venc = VideoEncoder(cfg)
    venc.load_state_dict(fixture_state_dict(fx), strict=True)
    venc = venc.to(DEV).eval()
    video = seeded_input(int(fx['video_seed']), tuple(int(s) for s in fx['video_shape'])).to(DEV)
    with torch.no_grad():
        feat = venc(video)
        hs = venc.backbone(video).last_hidden_state
    errs = (rel(hs[:, 0], fx['token0']), rel(hs[:, -1], fx['last_row']), rel(feat, fx['feat']))
    print('fp16 g5 rel errors (token0, last row, feat):', errs)
    assert max(errs) < 3e-3, errs            # measured 1.1e-3 on MI355X (bf16 path: 6e-2 bound)


def test_crossmodal_tiny_forward_f16_and_no_training():
    from fixtures import fixture_config, fixture_state_dict, load
    from cmhar.models import CrossModalModel
    fx = load('g2_crossmodal_tiny')
    cfg = fixture_config(fx)
    cfg.model.compute_dtype = 'fp16'
    torch.manual_seed(0)
    m = CrossModalModel(cfg)
    m.load_state_dict(fixture_state_dict(fx), strict=True)
    m = m.to(DEV).train()        # train-mode BN batch statistics, as the fixture
    imu = torch.tensor(fx['imu'], device=DEV)
    video = torch.tensor(fx['video'], device=DEV)
    with torch.no_grad():
        a, b = m(imu, video)
    assert rel(a, fx['imu_proj']) < 1e-5      # IMU branch is fp32
    assert rel(b, fx['video_proj']) < 5e-3
    with pytest.raises(RuntimeError, match='inference-only'):
        m(imu, video)
