"""Pin the CPU oracle (oracle/cpu_model.py) against golden vectors captured from the reference itself."""
import numpy as np
import pytest
import torch

from fixtures import fixture_config, fixture_state_dict, load, oracle_mcfg, t
from oracle import cpu_model as O

torch.set_num_threads(8)


def _close(a, b, rtol=1e-4, atol=1e-5, msg=''):
    a = a.detach().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
    np.testing.assert_allclose(a, np.asarray(b), rtol=rtol, atol=atol, err_msg=msg)


def _params(sd):
    return {k: (v.clone().requires_grad_(True) if v.is_floating_point() else v.clone()) for k, v in sd.items()}


def _check_grads(fx, sd, prefix='', rtol=2e-4, atol=2e-6):
    n = 0
    for key in fx.files:
        for kind in ('grad.', 'gnorm.', 'gsample.', 'gnone.'):
            if key.startswith(kind):
                name = prefix + key[len(kind):]
                g = sd[name].grad
                if kind == 'gnone.':
                    assert g is None or float(g.abs().max()) == 0.0, name
                elif kind == 'grad.':
                    assert g is not None, name
                    _close(g, fx[key], rtol, atol)
                elif kind == 'gnorm.':
                    assert abs(g.double().norm().item() - float(fx[key])) <= 1e-4 * float(fx[key]) + 1e-7, name
                else:
                    _close(g.reshape(-1)[::997], fx[key], rtol, atol)
                n += 1
    assert n > 0


def test_g1_imu_encoder():
    fx = load('g1_imu_encoder')
    cfg = fixture_config(fx)
    sd = _params(fixture_state_dict(fx))
    cls, tok = O.imu_encoder(sd, t(fx['x']), patch_size=16, stride=16, nhead=8, num_layers=4, prefix='')
    assert tok.shape == (4, 13, 128)                                      # CLS + 12 channel-0 patches
    _close(cls, fx['cls'])
    _close(tok, fx['tokens'])
    ((cls * t(fx['r'])).sum() + 0.1 * tok.pow(2).sum()).backward()
    _check_grads(fx, sd)
    # channels 1..5 projections get zero (not None) gradients
    for c in range(1, 6):
        assert float(sd[f'patch_embed.projections.{c}.weight'].grad.abs().max()) == 0.0
    del cfg


def test_g2_crossmodal_forward_backward():
    fx = load('g2_crossmodal_tiny')
    cfg = fixture_config(fx)
    sd = _params(fixture_state_dict(fx))
    mc = oracle_mcfg(cfg)
    a, b = O.crossmodal(sd, t(fx['imu']), t(fx['video']), mc, training=True)
    _close(a, fx['imu_proj'])
    _close(b, fx['video_proj'])
    log_t = torch.tensor(float(np.log(10.0)), requires_grad=True)
    bias = torch.tensor(-10.0, requires_grad=True)
    loss = O.siglip_loss(a, b, log_t, bias)
    _close(loss, fx['loss'], 1e-6, 1e-6)
    loss.backward()
    _check_grads(fx, sd)
    _close(log_t.grad, fx['loss_grad_temperature'], 1e-5, 1e-6)
    _close(bias.grad, fx['loss_grad_bias'], 1e-5, 1e-6)
    for key in fx.files:
        if key.startswith('bn.'):
            _close(sd[key[3:]], fx[key], 1e-5, 1e-6)


def test_g2_two_trainer_steps():
    """CrossModalTrainer.train_epoch over two batches: lr 1e-5 (LinearLR 0.1x), clip 1.0, AdamW wd 0.01."""
    fx = load('g2_crossmodal_tiny')
    cfg = fixture_config(fx)
    sd = _params(fixture_state_dict(fx))
    mc = oracle_mcfg(cfg)
    names = [k for k, v in sd.items() if v.is_floating_point() and 'running' not in k]
    m = [torch.zeros_like(sd[k]) for k in names]
    v = [torch.zeros_like(sd[k]) for k in names]
    log_t = torch.tensor(float(np.log(10.0)), requires_grad=True)
    bias = torch.tensor(-10.0, requires_grad=True)
    losses = []
    for step, (imu, video) in enumerate([(fx['imu'], fx['video']), (fx['step_imu2'], fx['step_video2'])], 1):
        for k in names:
            sd[k].grad = None
        a, b = O.crossmodal(sd, t(imu), t(video), mc, training=True)
        loss = O.siglip_loss(a, b, log_t, bias)
        loss.backward()
        losses.append(loss.item())
        with torch.no_grad():
            grads = [sd[k].grad for k in names]
            O.clip_grad_norm(grads, 1.0)
            O.adamw_step([sd[k] for k in names], grads, m, v, step, lr=1e-5)
    assert abs(np.mean(losses) - float(fx['step_mean_loss'])) < 1e-5
    # AdamW's first steps move every element by ~lr * g/(|g|+eps); elements whose gradient is mathematically zero
    # (key biases: softmax shift-invariance; biases and features feeding a train-mode BatchNorm: BN removes the
    # batch mean) carry only rounding noise, so their step is noise-determined in the reference as well.  Compare
    # tightly wherever the first-step gradient is well above noise, and to within two steps elsewhere.
    tight = 0
    gscale = max(float(np.abs(fx[k]).max()) for k in fx.files if k.startswith('grad.'))
    for key in fx.files:
        if not key.startswith('after.'):
            continue
        name = key[6:]
        got, want = sd[name].detach().numpy(), fx[key]
        if 'grad.' + name in fx.files:
            g1 = np.abs(fx['grad.' + name])
            ok = g1 > 1e-5 * gscale
            np.testing.assert_allclose(got[ok], want[ok], rtol=1e-5, atol=1e-7, err_msg=name)
            np.testing.assert_allclose(got[~ok], want[~ok], rtol=0, atol=2.1e-5, err_msg=name)
            tight += int(ok.sum())
        else:
            np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-5, err_msg=name)
    assert tight > 50_000
    assert float(fx['after_loss_temperature']) == pytest.approx(np.log(10.0), abs=1e-7)   # never optimised


def test_g3_siglip_degenerate():
    fx = load('g3_siglip')
    a = t(fx['a']).requires_grad_(True)
    b = t(fx['b']).requires_grad_(True)
    log_t = torch.tensor(float(np.log(10.0)), requires_grad=True)
    bias = torch.tensor(-10.0, requires_grad=True)
    loss = O.siglip_loss(a, b, log_t, bias)
    loss.backward()
    _close(loss, fx['loss'], 1e-6, 1e-6)
    _close(a.grad, fx['grad_a'], 1e-5, 1e-8)
    _close(b.grad, fx['grad_b'], 1e-5, 1e-8)
    # all-pairs mean softplus(-S): positives and negatives treated identically
    s = (t(fx['a']) @ t(fx['b']).T) * 10.0 - 10.0
    assert torch.nn.functional.softplus(-s).mean().item() == pytest.approx(float(fx['loss']), rel=1e-6)


def test_g4_classifier():
    fx = load('g4_classifier')
    cfg = fixture_config(fx)
    sd = _params(fixture_state_dict(fx))
    mc = oracle_mcfg(cfg)
    lt = O.imu_classifier(sd, t(fx['x']), mc, training=True)
    _close(lt, fx['logits_train'])
    lt.pow(2).mean().backward()
    _check_grads(fx, sd)
    with torch.no_grad():
        le = O.imu_classifier(sd, t(fx['x']), mc, training=False)
    _close(le, fx['logits_eval'])


@pytest.mark.slow
def test_g5_videomae_base_full_geometry():
    fx = load('g5_videomae_base_16x224')
    sd = fixture_state_dict(fx)
    from seeded import seeded_input
    video = seeded_input(int(fx['video_seed']), tuple(int(s) for s in fx['video_shape']))
    with torch.no_grad():
        h = O.videomae(sd, video, num_heads=12, prefix='backbone.')
        feat = torch.nn.functional.linear(h[:, 0], sd['projection.weight'], sd['projection.bias'])
    _close(h[:, 0], fx['token0'], 1e-4, 1e-4)
    _close(h[:, -1], fx['last_row'], 1e-4, 1e-4)
    _close(feat, fx['feat'], 1e-4, 1e-4)


def _cls_names(sd):
    enc = [k for k, v in sd.items() if k.startswith('imu_encoder.') and v.is_floating_point()]
    head = [k for k, v in sd.items() if k.startswith('classifier.') and v.is_floating_point() and 'running' not in k]
    return enc, head


@pytest.mark.parametrize('mode', ['linear_probe', 'finetune'])
def test_g6_classification_trainer(mode):
    """ClassificationTrainer.train_epoch (trainer.py:287-314) over two batches + validate (:316-353): CE loss, clip
    1.0, AdamW (head lr 1e-3; finetune: encoder group lr 1e-4), BN batch stats, metrics via sklearn."""
    from sklearn.metrics import balanced_accuracy_score, f1_score
    fx = load('g6_classification_trainer')
    cfg = fixture_config(fx)
    sd = _params(fixture_state_dict(fx))
    mc = oracle_mcfg(cfg)
    enc, head = _cls_names(sd)
    groups = [(head, 1e-3)] + ([(enc, 1e-4)] if mode == 'finetune' else [])
    state = {k: (torch.zeros_like(sd[k]), torch.zeros_like(sd[k])) for g, _ in groups for k in g}
    losses, correct, total = [], 0, 0
    for step in (1, 2):
        for g, _ in groups:
            for k in g:
                sd[k].grad = None
        x, y = t(fx[f'imu{step - 1}']), t(fx[f'label{step - 1}'])
        logits = O.imu_classifier(sd, x, mc, training=True)
        loss = O.cross_entropy(logits, y)
        loss.backward()
        losses.append(loss.item())
        correct += int((logits.argmax(1) == y).sum())
        total += len(y)
        with torch.no_grad():
            every = [sd[k].grad for g, _ in groups for k in g]
            O.clip_grad_norm(every, 1.0)
            for g, lr in groups:
                O.adamw_step([sd[k] for k in g], [sd[k].grad for k in g], [state[k][0] for k in g],
                             [state[k][1] for k in g], step, lr=lr)
    assert np.mean(losses) == pytest.approx(float(fx[f'{mode}.train_loss']), rel=1e-5)
    assert 100.0 * correct / total == pytest.approx(float(fx[f'{mode}.train_acc']))
    with torch.no_grad():
        le = O.imu_classifier(sd, t(fx['val_imu']), mc, training=False)
        yv = t(fx['val_label'])
        pred = le.argmax(1)
        # rel 5e-4: eval BN uses running means fed by the noise-driven biases (below)
        assert O.cross_entropy(le, yv).item() == pytest.approx(float(fx[f'{mode}.val_loss']), rel=5e-4)
        assert 100.0 * balanced_accuracy_score(yv.numpy(), pred.numpy()) == pytest.approx(
            float(fx[f'{mode}.val_balanced_accuracy']))
        assert 100.0 * f1_score(yv.numpy(), pred.numpy(), average='macro') == pytest.approx(
            float(fx[f'{mode}.val_f1_macro']))
    # A Linear feeding a train-mode BatchNorm has a mathematically zero bias gradient (BN removes the batch mean):
    # the reference's Adam step on it is driven by rounding noise (|step| ≤ ~lr each), and so is ours, possibly in
    # the other direction: they agree within 2 x steps x lr; the BN running mean it feeds inherits 0.1x that.
    # Everything else is compared tightly.
    noisy = {f'classifier.{4 * i}.bias': 4.2e-3 for i in range(len(mc['classifier_hidden_dims']))}
    noisy.update({f'classifier.{4 * i + 1}.running_mean': 4.2e-4 for i in range(len(mc['classifier_hidden_dims']))})
    noisy['imu_encoder.norm.bias'] = 4.2e-4      # a per-feature constant the first BN removes as well
    # Likewise the attention key biases (softmax is shift-invariant per query): within 2 encoder-lr steps.
    for key in fx.files:
        if key.startswith(f'{mode}.after.'):
            name = key[len(mode) + 7:]
            got, want = sd[name].detach(), fx[key]
            if name.endswith('in_proj_bias'):
                d = got.shape[0] // 3
                _close(got[d:2 * d], want[d:2 * d], 0.0, 4.2e-4, name)
                got, want = torch.cat([got[:d], got[2 * d:]]), np.concatenate([want[:d], want[2 * d:]])
            _close(got, want, 1e-5 if name not in noisy else 0.0, noisy.get(name, 2e-6), name)


def test_g7_alternative_losses():
    """InfoNCE / Focal / LabelSmoothing / CE restatements vs the reference's losses.py (values + input grads)."""
    fx = load('g7_losses')
    a = t(fx['nce_a']).requires_grad_(True)
    b = t(fx['nce_b']).requires_grad_(True)
    loss = O.info_nce(a, b, 0.07)
    loss.backward()
    _close(loss, fx['nce_loss'], 1e-6, 1e-6)
    _close(a.grad, fx['nce_grad_a'], 1e-5, 1e-7)
    _close(b.grad, fx['nce_grad_b'], 1e-5, 1e-7)
    y = t(fx['cls_labels'])
    fns = {'focal': lambda z, r: O.focal_loss(z, y, alpha=0.5, gamma=2.0, reduction=r),
           'label_smoothing': lambda z, r: O.label_smoothing_ce(z, y, 0.1, r),
           'cross_entropy': lambda z, r: O.cross_entropy(z, y, r)}
    for name, fn in fns.items():
        for red in ('mean', 'sum', 'none'):
            z = t(fx['cls_logits']).requires_grad_(True)
            lv = fn(z, red)
            w = t(fx[f'{name}.{red}.w']) if red == 'none' else torch.tensor(1.0)
            (lv * w).sum().backward()
            _close(lv, fx[f'{name}.{red}.loss'], 1e-5, 1e-6)
            _close(z.grad, fx[f'{name}.{red}.grad'], 1e-5, 1e-7)
