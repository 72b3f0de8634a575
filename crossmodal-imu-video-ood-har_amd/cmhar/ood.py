"""Energy-score out-of-distribution scoring on the prediction path (BASELINE config 5).

The reference repository is named for OOD HAR but contains no OOD code; its inference path is
`Evaluator.predict` (`src/eval/evaluator.py:28-53`): `model.eval()`, `logits = model(imu)` per batch under
`torch.no_grad()`, `logits.max(1)` for the predictions, numpy arrays out.  `OODEvaluator` keeps that interface and
adds the energy score E(x) = −T·logsumexp(f(x)/T) (Liu et al., energy-based OOD detection), computed on the device
in the same single pass over the logits as the predictions (`cmhar_logits_energy`).  Lower energy = more
in-distribution; `auroc(in_scores, out_scores)` reports how well a score separates the two (parity unpinned
w.r.t. the reference, which has no such code: checked against torch / sklearn in the tests).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib as L


def logits_energy(logits: torch.Tensor, temperature: float = 1.0):
    """(pred int64 [N], energy fp32 [N], max logit fp32 [N]) of a device [N, C] fp32/bf16 logits matrix."""
    if logits.dim() != 2 or not logits.is_cuda:
        raise ValueError('expected a 2-D device logits matrix')
    if logits.stride(1) != 1:
        logits = logits.contiguous()
    if temperature <= 0:
        raise ValueError('temperature must be positive')
    N, C = logits.shape
    dev = logits.device
    pred = torch.empty(N, dtype=torch.int32, device=dev)
    energy = torch.empty(N, dtype=torch.float32, device=dev)
    mx = torch.empty(N, dtype=torch.float32, device=dev)
    L.call('cmhar_logits_energy', L.dtype_code(logits.dtype), N, C, logits.data_ptr(), logits.stride(0),
           float(temperature), pred.data_ptr(), energy.data_ptr(), mx.data_ptr(), L.stream(dev))
    return pred.long(), energy, mx


def energy_score(logits: torch.Tensor, temperature: float = 1.0) -> torch.Tensor:
    """E = −T·logsumexp(logits/T) per row (fp32, on the device)."""
    return logits_energy(logits, temperature)[1]


def auroc(in_scores, out_scores) -> float:
    """Area under the ROC curve for separating in-distribution (positive, HIGHER score) from OOD samples — the
    Mann–Whitney U statistic with average ranks for ties (equals sklearn.metrics.roc_auc_score).  For energies pass
    −E (lower energy = in-distribution)."""
    a = np.asarray(in_scores, dtype=np.float64).ravel()
    b = np.asarray(out_scores, dtype=np.float64).ravel()
    if a.size == 0 or b.size == 0:
        raise ValueError('both score sets must be non-empty')
    allv = np.concatenate([a, b])
    order = np.argsort(allv, kind='mergesort')
    ranks = np.empty(allv.size, dtype=np.float64)
    sv = allv[order]
    new_run = np.r_[True, sv[1:] != sv[:-1]]    # average ranks over tied runs, vectorised (O(n log n) overall)
    starts = np.flatnonzero(new_run)
    ends = np.r_[starts[1:], sv.size] - 1
    ranks[order] = (0.5 * (starts + ends) + 1.0)[np.cumsum(new_run) - 1]
    u = ranks[:a.size].sum() - a.size * (a.size + 1) / 2.0
    return float(u / (a.size * b.size))


class OODEvaluator:
    """`Evaluator` (`src/eval/evaluator.py:18-53`) with energy scores: same constructor and `predict(dataloader)`
    (batches with 'imu' and 'label'), returning (predictions, labels, logits, energies) numpy arrays.  Batches that
    also carry 'video' are scored by a two-input model — `model(imu, video)`, e.g. the cross-attention fusion
    classifier (`cmhar.fusion.CrossModalFusionClassifier`), whose class logits are the "fused logits" of config 5."""

    def __init__(self, model, config, device='cuda', temperature: float = 1.0):
        self.model = model.to(device)
        self.config = config
        self.device = device
        self.temperature = float(temperature)
        self.model.eval()

    @torch.no_grad()
    def predict(self, dataloader):
        preds, labels, logits, energies = [], [], [], []
        for batch in dataloader:
            imu = batch['imu'].to(self.device)
            if 'video' in batch:
                out = self.model(imu, batch['video'].to(self.device))
            else:
                out = self.model(imu)
            p, e, _ = logits_energy(out.float(), self.temperature)
            preds.append(p.cpu().numpy())
            labels.append(np.asarray(batch['label']))
            logits.append(out.float().cpu().numpy())
            energies.append(e.cpu().numpy())
        return (np.concatenate(preds), np.concatenate(labels), np.vstack(logits), np.concatenate(energies))

    def ood_auroc(self, in_loader, out_loader) -> float:
        """AUROC of −energy for in-distribution vs OOD loaders."""
        e_in = self.predict(in_loader)[3]
        e_out = self.predict(out_loader)[3]
        return auroc(-e_in, -e_out)
