"""Trainer and loss drop-ins on the MI355X against golden vectors captured from the reference:

* `cmhar.trainer.CrossModalTrainer.train_epoch`    vs g2 (two reference CrossModalTrainer steps, trainer.py:124-146)
* `cmhar.trainer.ClassificationTrainer` (both modes) vs g6 (reference ClassificationTrainer, trainer.py:236-353)
* `cmhar.losses` InfoNCE / Focal / LabelSmoothing / CrossEntropy vs g7 (reference losses.py:57-167)
* the fused `cmhar_cross_entropy` kernel vs torch fp32 (ignore_index, transposed views, gradient accumulation)

Tolerances are written per check; parameters whose reference update is driven by rounding noise (mathematically
zero gradients) are compared within the Adam steps that noise can produce, as in the oracle tests."""
import numpy as np
import pytest
import torch

from fixtures import fixture_config, fixture_state_dict, load

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _close(a, b, rtol, atol, msg=''):
    a = a.detach().float().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
    np.testing.assert_allclose(a, np.asarray(b), rtol=rtol, atol=atol, err_msg=msg)


# ---------------------------------------------------------------------------------------------------------------
# cross-entropy kernel
# ---------------------------------------------------------------------------------------------------------------
@pytest.mark.parametrize('N,C', [(1, 2), (37, 11), (256, 32), (1000, 300)])
def test_cross_entropy_kernel_matches_torch(N, C):
    from cmhar import kernels as K
    g = torch.Generator().manual_seed(N + C)
    z = (4 * torch.randn(N, C, generator=g)).to(DEV)
    y = torch.randint(0, C, (N,), generator=g)
    y[::7] = -100
    y = y.to(DEV)
    loss = torch.empty((), device=DEV)
    pred = torch.empty(N, dtype=torch.int64, device=DEV)
    corr = torch.empty(1, dtype=torch.int32, device=DEV)
    status = torch.empty(1, dtype=torch.int32, device=DEV)
    dz = torch.empty_like(z)
    gup = torch.tensor([0.7], device=DEV)
    K.cross_entropy(z, y, loss=loss, pred=pred, correct=corr, status=status, dlogits=dz, g_up=gup)
    zr = z.clone().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(zr, y)
    (0.7 * ref).backward()
    if (y != -100).any():
        assert loss.item() == pytest.approx(ref.item(), rel=1e-5, abs=1e-6)
    assert torch.equal(pred, z.argmax(1))
    assert int(corr.item()) == int(((z.argmax(1) == y) & (y != -100)).sum())
    assert int(status.item()) == 0
    _close(dz, zr.grad.cpu(), 1e-4, 1e-7)


def test_cross_entropy_kernel_transposed_view_and_accumulate():
    """InfoNCE's second CE reads Sᵀ through a (1, B) stride view and accumulates into the same dS."""
    from cmhar import kernels as K
    g = torch.Generator().manual_seed(5)
    S = (3 * torch.randn(48, 48, generator=g)).to(DEV)
    dS = torch.empty_like(S)
    l1, l2 = torch.empty((), device=DEV), torch.empty((), device=DEV)
    K.cross_entropy(S, None, loss=l1, dlogits=dS, grad_scale=0.5)
    K.cross_entropy(S.t(), None, loss=l2, dlogits=dS.t(), grad_scale=0.5, grad_beta=1.0)
    Sr = S.clone().requires_grad_(True)
    ar = torch.arange(48, device=DEV)
    ref = (torch.nn.functional.cross_entropy(Sr, ar) + torch.nn.functional.cross_entropy(Sr.t(), ar)) / 2
    ref.backward()
    assert (l1.item() + l2.item()) / 2 == pytest.approx(ref.item(), rel=1e-5)
    _close(dS, Sr.grad.cpu(), 1e-4, 1e-7)


def test_cross_entropy_invalid_label_raises_or_flags():
    from cmhar import kernels as K
    from cmhar.losses import CrossEntropyLoss
    z = torch.randn(4, 5, device=DEV)
    with pytest.raises(IndexError):                       # host labels: checked before the copy, like torch
        CrossEntropyLoss()(z, torch.tensor([0, 1, 5, 2]))
    status = torch.empty(1, dtype=torch.int32, device=DEV)
    loss = torch.empty((), device=DEV)
    K.cross_entropy(z, torch.tensor([0, 1, 5, 2], device=DEV), loss=loss, status=status)
    assert int(status.item()) == 1 and not np.isfinite(loss.item())


# ---------------------------------------------------------------------------------------------------------------
# alternative losses vs the reference (g7)
# ---------------------------------------------------------------------------------------------------------------
def test_g7_losses_match_reference():
    from cmhar.losses import get_loss_function
    fx = load('g7_losses')
    a = torch.tensor(fx['nce_a'], device=DEV).requires_grad_(True)
    b = torch.tensor(fx['nce_b'], device=DEV).requires_grad_(True)
    loss = get_loss_function('infonce', temperature=0.07)(a, b)
    loss.backward()
    assert loss.item() == pytest.approx(float(fx['nce_loss']), rel=1e-5)
    _close(a.grad, fx['nce_grad_a'], 1e-4, 1e-6)
    _close(b.grad, fx['nce_grad_b'], 1e-4, 1e-6)
    y = torch.tensor(fx['cls_labels'], device=DEV)
    kws = {'focal': {'alpha': 0.5, 'gamma': 2.0}, 'label_smoothing': {'epsilon': 0.1}, 'cross_entropy': {}}
    for name, kw in kws.items():
        for red in ('mean', 'sum', 'none'):
            z = torch.tensor(fx['cls_logits'], device=DEV).requires_grad_(True)
            lv = get_loss_function(name, **dict(kw, reduction=red))(z, y)
            w = torch.tensor(fx[f'{name}.{red}.w'], device=DEV) if red == 'none' else torch.tensor(1.0, device=DEV)
            (lv * w).sum().backward()
            _close(lv, fx[f'{name}.{red}.loss'], 1e-5, 1e-6, f'{name}/{red}')
            _close(z.grad, fx[f'{name}.{red}.grad'], 1e-4, 1e-6, f'{name}/{red}')


# ---------------------------------------------------------------------------------------------------------------
# trainers
# ---------------------------------------------------------------------------------------------------------------
def test_g2_crossmodal_trainer_train_epoch():
    """cmhar.trainer.CrossModalTrainer over the two reference batches: mean loss and post-AdamW parameters."""
    from cmhar import models
    from cmhar.losses import SigmoidContrastiveLoss
    from cmhar.trainer import CrossModalTrainer
    fx = load('g2_crossmodal_tiny')
    cfg = fixture_config(fx)
    cfg.model.compute_dtype = 'fp32'
    torch.manual_seed(0)
    m = models.CrossModalModel(cfg)
    m.load_state_dict(fixture_state_dict(fx), strict=True)
    tr = CrossModalTrainer(m, SigmoidContrastiveLoss().to(DEV), cfg, device=DEV)
    assert tr.optimizer.param_groups[0]['lr'] == pytest.approx(1e-5)          # LinearLR start factor 0.1
    batches = [{'imu': torch.tensor(fx['imu']), 'video': torch.tensor(fx['video'])},
               {'imu': torch.tensor(fx['step_imu2']), 'video': torch.tensor(fx['step_video2'])}]
    mean_loss = tr.train_epoch(batches)
    assert mean_loss == pytest.approx(float(fx['step_mean_loss']), abs=1e-4)
    gscale = max(float(np.abs(fx[k]).max()) for k in fx.files if k.startswith('grad.'))
    sd = m.state_dict()
    for key in fx.files:
        if not key.startswith('after.'):
            continue
        name = key[6:]
        got, want = sd[name].detach().cpu().numpy(), fx[key]
        if 'grad.' + name in fx.files:
            ok = np.abs(fx['grad.' + name]) > 1e-3 * gscale
            np.testing.assert_allclose(got[ok], want[ok], rtol=1e-5, atol=3e-7, err_msg=name)
            np.testing.assert_allclose(got[~ok], want[~ok], rtol=0, atol=3.1e-5, err_msg=name)
        elif got.dtype.kind == 'f':
            np.testing.assert_allclose(got, want, rtol=1e-4, atol=2e-5, err_msg=name)
        else:
            assert (got == want).all(), name


@pytest.mark.parametrize('mode', ['linear_probe', 'finetune'])
def test_g6_classification_trainer(mode):
    from cmhar.models import IMUClassifier, IMUEncoder
    from cmhar.trainer import ClassificationTrainer
    fx = load('g6_classification_trainer')
    cfg = fixture_config(fx)
    torch.manual_seed(0)
    clf = IMUClassifier(IMUEncoder(cfg), cfg, freeze_encoder=False)
    clf.load_state_dict(fixture_state_dict(fx), strict=True)
    tr = ClassificationTrainer(clf, cfg, device=DEV, mode=mode)
    batches = [{'imu': torch.tensor(fx[f'imu{i}']), 'label': torch.tensor(fx[f'label{i}'])} for i in range(2)]
    m = tr.train_epoch(batches)
    assert m['loss'] == pytest.approx(float(fx[f'{mode}.train_loss']), rel=1e-5)
    assert m['accuracy'] == pytest.approx(float(fx[f'{mode}.train_acc']))
    v = tr.validate([{'imu': torch.tensor(fx['val_imu']), 'label': torch.tensor(fx['val_label'])}])
    assert v['loss'] == pytest.approx(float(fx[f'{mode}.val_loss']), rel=5e-4)   # noise-driven BN means (below)
    for k in ('accuracy', 'balanced_accuracy', 'f1_macro'):
        assert v[k] == pytest.approx(float(fx[f'{mode}.val_{k}'])), k
    hid = len(cfg.model.classifier_hidden_dims)
    noisy = {f'classifier.{4 * i}.bias': 4.2e-3 for i in range(hid)}
    noisy.update({f'classifier.{4 * i + 1}.running_mean': 4.2e-4 for i in range(hid)})
    noisy['imu_encoder.norm.bias'] = 4.2e-4
    sd = clf.state_dict()
    for key in fx.files:
        if not key.startswith(f'{mode}.after.'):
            continue
        name = key[len(mode) + 7:]
        got, want = sd[name].detach().cpu(), fx[key]
        if got.dtype == torch.int64:
            assert (got.numpy() == want).all(), name
            continue
        if name.endswith('in_proj_bias'):                  # key biases: softmax shift invariance
            d = got.shape[0] // 3
            _close(got[d:2 * d], want[d:2 * d], 0.0, 4.2e-4, name)
            got, want = torch.cat([got[:d], got[2 * d:]]), np.concatenate([want[:d], want[2 * d:]])
        _close(got, want, 1e-5 if name not in noisy else 0.0, noisy.get(name, 3e-6), name)


def test_g9_resume_reference_checkpoint_and_step():
    """A `last.pt` written by the REFERENCE's CrossModalTrainer after 2 steps + one scheduler step: model, AdamW
    moments/step count and the LinearLR→Cosine schedule restored into the drop-ins; the next training step must
    land where the reference's third step did."""
    import os
    from cmhar import models
    from cmhar.checkpoint import resume
    from cmhar.losses import SigmoidContrastiveLoss
    from cmhar.trainer import CrossModalTrainer
    fx = load('g9_checkpoint_resume')
    cfg = fixture_config(fx)
    cfg.model.compute_dtype = 'fp32'
    torch.manual_seed(0)
    m = models.CrossModalModel(cfg)
    tr = CrossModalTrainer(m, SigmoidContrastiveLoss().to(DEV), cfg, device=DEV)
    resume(tr, os.path.join(os.path.dirname(__file__), 'golden', 'g9_last.pt'))
    assert tr.optimizer.param_groups[0]['lr'] == pytest.approx(float(fx['lr_epoch1']), rel=1e-12)
    loss = tr.train_epoch([{'imu': torch.tensor(fx['imu3']), 'video': torch.tensor(fx['video3'])}])
    assert loss == pytest.approx(float(fx['loss3']), rel=1e-5)
    lr = float(fx['lr_epoch1'])
    sd = m.state_dict()
    params = list(m.parameters())
    pidx = {id(p): i for i, p in enumerate(params)}
    named = dict(m.named_parameters())
    tight = 0
    emax = max(float(np.abs(fx[k]).max()) for k in fx.files if k.startswith('exp_avg.'))
    for key in fx.files:
        if not key.startswith('after.'):
            continue
        name = key[6:]
        got, want = sd[name].detach().cpu().numpy(), fx[key]
        if name in named and f'exp_avg.{pidx[id(named[name])]}' in fx.files:
            ea = np.abs(fx[f'exp_avg.{pidx[id(named[name])]}'])
            ok = ea > 1e-3 * emax                          # steps driven by real gradients, not rounding noise
            np.testing.assert_allclose(got[ok], want[ok], rtol=1e-5, atol=3e-7, err_msg=name)
            np.testing.assert_allclose(got[~ok], want[~ok], rtol=0, atol=2.1 * lr, err_msg=name)
            tight += int(ok.sum())
        elif got.dtype.kind == 'f':
            np.testing.assert_allclose(got, want, rtol=1e-4, atol=2e-5, err_msg=name)
        else:
            assert (got == want).all(), name
    assert tight > 5_000
