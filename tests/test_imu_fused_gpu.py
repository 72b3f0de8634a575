"""The one-launch IMU encoder forward (cmhar_imu_encoder_fwd) against the per-op launch chain it replaces
(cmhar_gemm_generic / cmhar_attention_fwd / cmhar_layernorm_fwd, the path g1 / g4 / g6 pin to the reference):
every output and every tensor saved for the backward must be BIT-identical, with and without dropout, at the
reference window (W = 250: T = 16), the bench window (200: T = 13), config 4's (400: T = 26, the 32-row kernel)
and a tiny one (64: T = 5).  Through the module, forward + backward of the fused path equal the per-op path's."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _encoder(W, p):
    from cmhar.config import Config
    from cmhar.imu import IMUEncoder
    cfg = Config()
    cfg.data.imu_window_size = W
    cfg.model.imu_dropout = p
    torch.manual_seed(0)
    return IMUEncoder(cfg).to(DEV)


@pytest.mark.parametrize('W,B,p', [(200, 32, 0.0), (200, 32, 0.1), (250, 8, 0.1), (400, 8, 0.1), (400, 3, 0.0),
                                   (64, 3, 0.1)])
def test_imu_fused_forward_bit_identical(W, B, p, monkeypatch):
    from cmhar import imu
    m = _encoder(W, p)
    g = torch.Generator(device=DEV).manual_seed(W + B)
    x = torch.randn(B, 6, W, device=DEV, generator=g)
    out = {}
    for fused in (True, False):
        monkeypatch.setattr(imu, '_FUSED', fused)
        assert imu._fused_ok(m, min(1 + 6 * ((W - 16) // 16 + 1), m.pos_encoding.shape[1])) == fused
        with torch.no_grad():
            enc, st = imu._imu_forward(m, x, p, 0x5EED1234 if p > 0 else 0, save=True)
        torch.cuda.synchronize()
        out[fused] = (enc, st)
    (e1, s1), (e0, s0) = out[True], out[False]
    assert torch.equal(e1, e0)
    names = ('h', 'qkv', 'o', 'lse', 's1', 'mu1', 'rs1', 'h1', 'fd', 's2', 'mu2', 'rs2')
    for li, (a, b) in enumerate(zip(s1['saved'], s0['saved'])):
        for n, ta, tb in zip(names, a, b):
            assert ta.shape == tb.shape, (li, n)
            assert torch.equal(ta, tb), (li, n, (ta - tb).abs().max().item())
    for ta, tb in zip(s1['final'], s0['final']):
        assert torch.equal(ta, tb)
    if p > 0:   # the dropout masks are live
        assert (s1['saved'][0][8] == 0).float().mean().item() > 0.5   # relu zeros + dropped


@pytest.mark.parametrize('W,B', [(200, 16), (400, 5)])
def test_imu_fused_module_fwd_bwd_identical(W, B, monkeypatch):
    """Whole module, train mode with dropout: outputs, weight gradients and the embedding's gradients bit-identical
    to the per-op path; bias / LayerNorm-affine gradients (summed over tokens in one sequential pass instead of the
    per-op path's two-level reduction) within 1e-5 relative."""
    from cmhar import imu
    p = 0.1
    res = {}
    for fused in (True, False):
        monkeypatch.setattr(imu, '_FUSED', fused)
        m = _encoder(W, p).train()
        m._calls = 0
        x = torch.randn(B, 6, W, device=DEV, generator=torch.Generator(device=DEV).manual_seed(3))
        cls, enc = m(x)
        (cls.square().sum() + 0.5 * enc.sum()).backward()
        torch.cuda.synchronize()
        res[fused] = (cls.detach(), enc.detach(), [(n, q.grad.clone()) for n, q in m.named_parameters()])
    assert torch.equal(res[True][0], res[False][0])
    assert torch.equal(res[True][1], res[False][1])
    for (n, a), (_, b) in zip(res[True][2], res[False][2]):
        summed = n.endswith('bias') or '.norm' in n or n.startswith('norm.')
        if n.startswith('patch_embed') or n in ('cls_token', 'pos_encoding') or not summed:
            assert torch.equal(a, b), (n, (a - b).abs().max().item())
        else:
            err = ((a - b).norm() / b.norm().clamp_min(1e-30)).item()
            assert err <= 1e-5, (n, err)


def test_imu_fused_rejects_other_geometries():
    """d_model != 128 (e.g. the tiny g2 encoder) keeps the per-op launches; the C entry refuses it."""
    from cmhar import _lib as L
    from cmhar import imu
    from cmhar.config import Config
    from cmhar.imu import IMUEncoder
    cfg = Config()
    cfg.model.imu_d_model = 32
    cfg.model.imu_nhead = 4
    m = IMUEncoder(cfg).to(DEV)
    assert not imu._fused_ok(m, 13)
    arr = (L.IMULayer * 1)()
    rc = L.lib().cmhar_imu_encoder_fwd(2, 13, 32, 4, 128, 1, 1, arr, 1, 1, 1e-5, 1, 1, 1, 0.25, 0.0, 0,
                                       L.stream(torch.device(DEV)))
    assert rc == -1
