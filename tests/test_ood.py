"""Energy-score OOD head (BASELINE config 5).  The reference has no OOD code, so
this is "parity unpinned" w.r.t. the reference: the kernel is checked against a torch fp32/fp64 restatement of
E = −T·logsumexp(logits/T) and torch.max's first-index argmax, the AUROC helper against sklearn, and the evaluator
against the reference's `Evaluator.predict` contract (src/eval/evaluator.py:28-53)."""
import numpy as np
import pytest
import torch

DEV = 'cuda'


def test_auroc_matches_sklearn_with_ties():
    from sklearn.metrics import roc_auc_score
    from cmhar.ood import auroc
    rng = np.random.default_rng(0)
    a = np.round(rng.normal(1.0, 1.0, 300), 1)          # rounding makes many ties across and within the sets
    b = np.round(rng.normal(0.0, 1.0, 200), 1)
    want = roc_auc_score(np.r_[np.ones(a.size), np.zeros(b.size)], np.r_[a, b])
    assert abs(auroc(a, b) - want) < 1e-12
    assert auroc([2.0], [1.0]) == 1.0 and auroc([1.0], [2.0]) == 0.0 and auroc([1.0], [1.0]) == 0.5


@pytest.mark.parametrize('n_in,n_out,decimals', [(1, 5000, 2), (20000, 30000, 1), (50000, 7, 3), (4096, 4096, 0)])
def test_auroc_large_and_lopsided_vs_sklearn(n_in, n_out, decimals):
    """Eval-stream sizes (tens of thousands of clips, one side tiny), heavy ties from rounding."""
    from sklearn.metrics import roc_auc_score
    from cmhar.ood import auroc
    rng = np.random.default_rng(n_in + n_out)
    a = np.round(rng.normal(0.5, 1.0, n_in), decimals)
    b = np.round(rng.normal(0.0, 1.0, n_out), decimals)
    want = roc_auc_score(np.r_[np.ones(n_in), np.zeros(n_out)], np.r_[a, b])
    assert abs(auroc(a, b) - want) < 1e-12


def test_auroc_edge_cases():
    from cmhar.ood import auroc
    assert auroc(np.full(7, 3.0), np.full(9, 3.0)) == 0.5            # one tied run across both sets
    assert auroc(np.arange(10.0) + 10, np.arange(10.0)) == 1.0       # perfect separation
    assert auroc(np.arange(10.0), np.arange(10.0) + 10) == 0.0
    assert auroc(np.ones((2, 3)), np.zeros((3, 1))) == 1.0           # any shape, flattened
    with pytest.raises(ValueError):
        auroc([], [1.0])
    with pytest.raises(ValueError):
        auroc([1.0], np.zeros(0))


@pytest.mark.gpu
@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('C', [1, 7, 32, 1000])
@pytest.mark.parametrize('T', [1.0, 2.5])
def test_logits_energy_vs_torch(dtype, C, T):
    from cmhar.ood import logits_energy
    g = torch.Generator().manual_seed(C)
    x = (torch.randn(513, C, generator=g) * 4).to(dtype)
    pred, e, mx = logits_energy(x.to(DEV), T)
    xf = x.double()
    assert torch.allclose(e.cpu().double(), -T * torch.logsumexp(xf / T, 1), rtol=1e-5, atol=1e-5)
    assert torch.equal(mx.cpu().double(), xf.max(1).values)
    assert torch.equal(pred.cpu(), xf.argmax(1))


@pytest.mark.gpu
def test_logits_energy_first_index_ties_and_strided():
    from cmhar.ood import logits_energy
    g = torch.Generator().manual_seed(3)
    base = torch.randint(-3, 3, (300, 200), generator=g).float()        # many equal maxima per row
    wide = torch.zeros(300, 256)
    wide[:, :200] = base
    pred, e, _ = logits_energy(wide.to(DEV)[:, :200])                   # row stride 256, 200 classes
    want = torch.tensor([int((r == r.max()).nonzero()[0]) for r in base])
    assert torch.equal(pred.cpu(), want)
    assert torch.allclose(e.cpu(), -torch.logsumexp(base, 1), rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
def test_ood_evaluator_contract_and_separation():
    """predict() returns the reference's (preds, labels, logits) + energies; peaked (in-distribution-like) logits
    get lower energy than flat ones, so AUROC(−E) ≈ 1."""
    from cmhar.ood import OODEvaluator, auroc
    from cmhar.config import Config
    from cmhar.imu import IMUEncoder
    from cmhar.models import IMUClassifier
    cfg = Config()
    cfg.model.imu_dropout = 0.0
    torch.manual_seed(0)
    clf = IMUClassifier(IMUEncoder(cfg), cfg)
    ev = OODEvaluator(clf, cfg, DEV)
    g = torch.Generator().manual_seed(1)
    loader = [{'imu': torch.randn(16, 6, cfg.data.imu_window_size, generator=g), 'label': torch.arange(16) % 4}
              for _ in range(3)]
    preds, labels, logits, energies = ev.predict(loader)
    assert preds.shape == (48,) and labels.shape == (48,) and logits.shape == (48, cfg.model.num_classes)
    assert np.array_equal(preds, logits.argmax(1))
    assert np.allclose(energies, -torch.logsumexp(torch.from_numpy(logits).double(), 1).numpy(), rtol=1e-5,
                       atol=1e-5)

    class Fixed(torch.nn.Module):
        def __init__(self, scale):
            super().__init__()
            self.scale = scale

        def forward(self, x):
            z = torch.zeros(x.shape[0], 32, device=x.device)
            z[:, 0] = self.scale
            return z + 0.1 * torch.randn_like(z)

    e_in = OODEvaluator(Fixed(8.0), cfg, DEV).predict(loader)[3]
    e_out = OODEvaluator(Fixed(0.0), cfg, DEV).predict(loader)[3]
    assert auroc(-e_in, -e_out) > 0.99
