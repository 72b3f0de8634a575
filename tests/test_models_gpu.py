"""Model-level parity on the MI355X against golden vectors captured from the REFERENCE implementation
(tests/golden/*.npz, produced by tests/golden/make_golden.py).

fp32 mode must match the reference to ≤1e-4 relative (outputs) — the north-star gate is 1e-3 on fp32 logits;
bf16 mode (the throughput mode) is checked at the tolerance its 8-bit mantissa allows, written per test."""
import json

import numpy as np
import pytest
import torch

from fixtures import fixture_config, fixture_state_dict, load
from seeded import seeded_input

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def rel(a, b):
    a = torch.as_tensor(a).float().cpu()
    b = torch.as_tensor(np.asarray(b)).float()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _grad_errors(model, fx, prefix='', zero_tol=1e-4):
    errs = {}
    gscale = max(float(np.abs(fx[k]).max()) for k in fx.files if k.startswith('grad.'))
    for key in fx.files:
        if key.startswith('grad.'):
            name = prefix + key[5:]
            p = dict(model.named_parameters())[name]
            ref = np.asarray(fx[key])
            if np.abs(ref).max() < 1e-5 * gscale:      # mathematically-zero gradient (noise in the reference)
                assert p.grad is None or p.grad.abs().max().item() < zero_tol * gscale, name
                continue
            errs[name] = rel(p.grad, ref)
        elif key.startswith('gnorm.'):
            name = prefix + key[6:]
            p = dict(model.named_parameters())[name]
            errs[name] = abs(p.grad.double().norm().item() - float(fx[key])) / float(fx[key])
    return errs


def _build(cls_name, fx, dtype='fp32'):
    from cmhar import models
    cfg = fixture_config(fx)
    cfg.model.compute_dtype = dtype
    torch.manual_seed(0)
    if cls_name == 'CrossModalModel':
        m = models.CrossModalModel(cfg)
    elif cls_name == 'IMUEncoder':
        m = models.IMUEncoder(cfg)
    elif cls_name == 'IMUClassifier':
        m = models.IMUClassifier(models.IMUEncoder(cfg), cfg)
    sd = fixture_state_dict(fx)
    m.load_state_dict(sd, strict=True)
    return m.to(DEV), cfg


def test_g1_imu_encoder_fp32():
    fx = load('g1_imu_encoder')
    m, _ = _build('IMUEncoder', fx)
    m.train()
    x = torch.tensor(fx['x'], device=DEV)
    cls, tok = m(x)
    assert rel(cls, fx['cls']) < 1e-5
    assert rel(tok, fx['tokens']) < 1e-5
    r = torch.tensor(fx['r'], device=DEV)
    ((cls * r).sum() + 0.1 * tok.pow(2).sum()).backward()
    errs = _grad_errors(m, fx)
    assert max(errs.values()) < 1e-4, sorted(errs.items(), key=lambda kv: -kv[1])[:5]
    for c in range(1, 6):
        assert m.patch_embed.projections[c].weight.grad.abs().max().item() == 0.0


@pytest.mark.parametrize('dtype,tol_out,tol_grad', [('fp32', 1e-4, 1e-3), ('bf16', 2e-2, 6e-2)])
def test_g2_crossmodal_forward_backward(dtype, tol_out, tol_grad):
    from cmhar.losses import SigmoidContrastiveLoss
    fx = load('g2_crossmodal_tiny')
    m, _ = _build('CrossModalModel', fx, dtype)
    m.train()
    imu = torch.tensor(fx['imu'], device=DEV)
    video = torch.tensor(fx['video'], device=DEV)
    lf = SigmoidContrastiveLoss().to(DEV)
    a, b = m(imu, video)
    assert rel(a, fx['imu_proj']) < tol_out
    assert rel(b, fx['video_proj']) < tol_out
    loss = lf(a, b)
    assert abs(loss.item() - float(fx['loss'])) < tol_out * abs(float(fx['loss']))
    loss.backward()
    errs = _grad_errors(m, fx, zero_tol=1e-4 if dtype == 'fp32' else 2e-3)   # bf16 rounding noise on zero grads
    worst = sorted(errs.items(), key=lambda kv: -kv[1])[:5]
    assert max(errs.values()) < tol_grad, worst
    for key in fx.files:
        if key.startswith('bn.') and 'running' in key:
            assert rel(m.state_dict()[key[3:]], fx[key]) < max(tol_out, 1e-5), key


def test_g2_two_trainer_steps_fused_optimizer():
    """trainer.py:130-144 with cmhar's clip_grad_norm_ + FusedAdamW (lr 1e-5 = LinearLR start factor 0.1)."""
    from cmhar.losses import SigmoidContrastiveLoss
    from cmhar.optim import FusedAdamW, clip_grad_norm_
    fx = load('g2_crossmodal_tiny')
    m, _ = _build('CrossModalModel', fx, 'fp32')
    m.train()
    lf = SigmoidContrastiveLoss().to(DEV)
    opt = FusedAdamW(m.parameters(), lr=1e-5, weight_decay=0.01, shadow_sources=[m.video_encoder.backbone])
    losses = []
    for imu, video in [(fx['imu'], fx['video']), (fx['step_imu2'], fx['step_video2'])]:
        a, b = m(torch.tensor(imu, device=DEV), torch.tensor(video, device=DEV))
        loss = lf(a, b)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        clip_grad_norm_(m.parameters(), 1.0)
        opt.step()
        losses.append(loss.item())
    assert abs(np.mean(losses) - float(fx['step_mean_loss'])) < 1e-4
    gscale = max(float(np.abs(fx[k]).max()) for k in fx.files if k.startswith('grad.'))
    sd = m.state_dict()
    tight = 0
    for key in fx.files:
        if not key.startswith('after.'):
            continue
        name = key[6:]
        got, want = sd[name].detach().cpu().numpy(), fx[key]
        if 'grad.' + name in fx.files:
            ok = np.abs(fx['grad.' + name]) > 1e-3 * gscale     # well-conditioned Adam steps (see oracle test)
            np.testing.assert_allclose(got[ok], want[ok], rtol=1e-5, atol=3e-7, err_msg=name)
            np.testing.assert_allclose(got[~ok], want[~ok], rtol=0, atol=3.1e-5, err_msg=name)   # ≤ 3 Adam steps of lr
            tight += int(ok.sum())
        elif got.dtype.kind == 'f':
            np.testing.assert_allclose(got, want, rtol=1e-4, atol=2e-5, err_msg=name)
        else:
            assert (got == want).all(), name
    assert tight > 20_000


def test_g4_classifier_train_eval():
    fx = load('g4_classifier')
    m, _ = _build('IMUClassifier', fx)
    x = torch.tensor(fx['x'], device=DEV)
    m.train()
    lt = m(x)
    assert rel(lt, fx['logits_train']) < 1e-5
    lt.pow(2).mean().backward()
    errs = _grad_errors(m, fx)
    assert max(errs.values()) < 1e-3, sorted(errs.items(), key=lambda kv: -kv[1])[:5]
    m.eval()
    with torch.no_grad():
        le = m(x)
    assert rel(le, fx['logits_eval']) < 1e-5


@pytest.mark.parametrize('dtype,tol', [('fp32', 1e-3), ('bf16', 6e-2)])
def test_g5_videomae_base_full_geometry(dtype, tol):
    """VideoMAE-B at the metric's clip geometry (16×224², 1568 tokens, 12 layers): token-0 features and the
    VideoEncoder output vs the reference.  fp32 mode: ≤1e-3 relative (north-star logits gate)."""
    from cmhar.config import Config
    from cmhar.models import VideoEncoder
    fx = load('g5_videomae_base_16x224')
    cfg = Config()
    cfg.model.video_backbone = '/nonexistent/videomae-local'
    cfg.model.compute_dtype = dtype
    torch.manual_seed(0)
    with pytest.warns(UserWarning):
        venc = VideoEncoder(cfg)
    venc.load_state_dict(fixture_state_dict(fx), strict=True)
    venc = venc.to(DEV).eval()
    video = seeded_input(int(fx['video_seed']), tuple(int(s) for s in fx['video_shape'])).to(DEV)
    with torch.no_grad():
        feat = venc(video)
        hs = venc.backbone(video).last_hidden_state
    assert rel(hs[:, 0], fx['token0']) < tol
    assert rel(hs[:, -1], fx['last_row']) < tol
    assert rel(feat, fx['feat']) < tol
