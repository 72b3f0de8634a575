"""Trainer drop-ins for the reference's `src/train/trainer.py` (`BaseTrainer` 29-56, `CrossModalTrainer` 62-230,
`ClassificationTrainer` 236-413) on the cmhar HIP path.

Same constructors, attributes (`model`, `config`, `device`, `optimizer`, `scheduler`, `history`, `current_epoch`,
`best_val_loss` / `best_bal_acc`, `mode`, `loss_fn`), step semantics and checkpoint files (`last.pt`,
`best_model.pt`, `checkpoint_epoch_{e}.pt`, `training_history.json`, same dict keys), so `main.py`-style drivers
switch by changing the import.  What differs is only what the MI355X wants:

* the optimizer is `cmhar.optim.FusedAdamW` (one multi-tensor launch; torch.optim.AdamW arithmetic and state
  layout, so `optimizer_state_dict` interchanges) with the reference's `clip_grad_norm_(..., 1.0)` folded into its
  pass (`max_grad_norm=1.0`: device-side norm and coefficient, bit-identical update and clipped `.grad`); the LR
  schedule is the reference's own torch LinearLR → CosineAnnealingLR (SequentialLR);
* the per-step `loss.item()` host syncs of the reference loop (`trainer.py:143-144,307-310`) are replaced by
  device-side accumulation; the epoch means are read once per epoch (same values);
* data parallel: pass a `cmhar.dist.GradReducer` (one process per GPU, RCCL all-reduce SUM of gradients
  overlapped with backward — `nn.DataParallel`'s reduce-add semantics) as `grad_reducer`.  The
  single-writer semantics of the reference's one process (main.py:89-124) are kept: only rank 0 writes
  checkpoints and `training_history.json`; BatchNorm running statistics are rank 0's (DataParallel keeps the
  device-0 replica's) and are broadcast at the end of every training epoch, before validation and saving; losses
  and metrics are those of the global batch (the classification loss is scaled by B_local / B_global so the
  summed gradient is the global-batch mean's, as DataParallel's gather-then-mean gives).
"""
from __future__ import annotations

import json
from pathlib import Path
from typing import Any, Dict, Optional

import torch
import torch.nn as nn
from torch.optim.lr_scheduler import CosineAnnealingLR, LinearLR, SequentialLR

from . import dist as D
from . import kernels as K
from .losses import CrossEntropyLoss
from .optim import FusedAdamW

__all__ = ['BaseTrainer', 'CrossModalTrainer', 'ClassificationTrainer']


def _shadow_sources(model):
    m = getattr(model, 'module', model)
    venc = getattr(m, 'video_encoder', None)
    bb = getattr(venc, 'backbone', None)
    return [bb] if bb is not None else []


def _progress(it, enabled, desc):
    if not enabled:
        return it
    from tqdm import tqdm
    return tqdm(it, desc=desc, leave=False)


class _DeviceSum:
    """Running fp32 sum of device scalars (cmhar_copy2d with beta = 1): no host sync until `value()`."""

    def __init__(self, device):
        self.t = torch.zeros(1, 1, dtype=torch.float32, device=device)

    def add(self, x):
        K.copy2d(x.detach().reshape(1, 1).float(), self.t, beta=1.0)

    def value(self) -> float:
        return float(self.t.item())


# -----------------------------
#   Base Trainer  (trainer.py:29-56)
# -----------------------------
class BaseTrainer:
    def __init__(self, model, config, device: str = 'cuda'):
        self.model = model.to(device)
        self.config = config
        self.device = device
        self.current_epoch = 0
        self.history = {'train': [], 'val': []}

    def save_checkpoint(self, path: Path, extra: Optional[Dict[str, Any]] = None):
        if not D.is_main():           # one writer under data parallelism (the reference is one process)
            return
        path = Path(path)
        path.parent.mkdir(parents=True, exist_ok=True)
        ckpt = {'epoch': self.current_epoch, 'model_state_dict': self.model.state_dict(), 'history': self.history}
        if extra:
            ckpt.update(extra)
        torch.save(ckpt, str(path))
        print(f'[Checkpoint] saved -> {path}')

    def load_checkpoint(self, path: Path, strict: bool = True) -> Dict[str, Any]:
        ckpt = torch.load(str(path), map_location=self.device, weights_only=True)
        self.model.load_state_dict(ckpt['model_state_dict'], strict=strict)
        self.current_epoch = int(ckpt.get('epoch', 0))
        self.history = ckpt.get('history', {'train': [], 'val': []})
        print(f'[Checkpoint] loaded <- {path}')
        return ckpt


# -----------------------------
#   Cross-modal Pretraining Trainer  (trainer.py:62-230)
# -----------------------------
class CrossModalTrainer(BaseTrainer):
    """Pretraining cross-modal IMU-Video; best = min val_loss."""

    def __init__(self, model, loss_fn, config, device: str = 'cuda', *, grad_reducer=None,
                 show_progress: bool = False):
        super().__init__(model, config, device)
        self.loss_fn = loss_fn
        self.best_val_loss = float('inf')
        self.grad_reducer = grad_reducer
        self.show_progress = show_progress
        # max_grad_norm: trainer.py:140's clip_grad_norm_(model.parameters(), 1.0) folded into the AdamW pass
        # (bit-identical update and post-clip .grad; one scale pass over the gradients less)
        self.optimizer = FusedAdamW(self.model.parameters(), lr=config.training.pretrain_lr,
                                    weight_decay=config.training.pretrain_weight_decay,
                                    shadow_sources=_shadow_sources(self.model), max_grad_norm=1.0,
                                    clip_params=self.model.parameters())
        num_epochs = int(config.training.pretrain_epochs)
        warmup_epochs = int(getattr(config.training, 'pretrain_warmup_epochs', 0))
        if warmup_epochs <= 0:
            self.scheduler = CosineAnnealingLR(self.optimizer, T_max=max(num_epochs, 1), eta_min=1e-6)
        else:
            warmup = LinearLR(self.optimizer, start_factor=0.1, total_iters=warmup_epochs)
            cosine = CosineAnnealingLR(self.optimizer, T_max=max(num_epochs - warmup_epochs, 1), eta_min=1e-6)
            self.scheduler = SequentialLR(self.optimizer, schedulers=[warmup, cosine], milestones=[warmup_epochs])
        self.video_channel_first = bool(getattr(config.data, 'video_channel_first', False))

    def _maybe_permute_video(self, video: torch.Tensor) -> torch.Tensor:
        """trainer.py:110-122 (a view; the backbone's im2col reads (B,T,C,H,W) contiguous)."""
        if self.video_channel_first:
            if video.dim() == 5 and video.shape[1] != 3 and video.shape[2] == 3:
                video = video.permute(0, 2, 1, 3, 4)
        else:
            if video.dim() == 5 and video.shape[1] == 3:
                video = video.permute(0, 2, 1, 3, 4)
        return video

    def _batch(self, batch):
        imu = batch['imu'].to(self.device, non_blocking=True)
        video = batch['video'].to(self.device, non_blocking=True)
        return imu, self._maybe_permute_video(video).contiguous()

    def train_step(self, imu, video):
        """One step of trainer.py:135-141; returns the loss as a device scalar."""
        imu_proj, video_proj = self.model(imu, video)
        loss = self.loss_fn(imu_proj, video_proj)
        self.optimizer.zero_grad(set_to_none=True)
        if self.grad_reducer is not None:
            self.grad_reducer.start_step()
        loss.backward()
        if self.grad_reducer is not None:
            self.grad_reducer.finish()
        self.optimizer.step()          # clip_grad_norm_(model.parameters(), 1.0) + AdamW.step (trainer.py:140-141)
        return loss

    def train_epoch(self, dataloader) -> float:
        self.model.train()
        total = _DeviceSum(self.device)
        for batch in _progress(dataloader, self.show_progress, f'[Pretrain] Epoch {self.current_epoch}'):
            total.add(self.train_step(*self._batch(batch)))
        D.broadcast_buffers(self.model)     # rank 0's BN running statistics (DataParallel's device-0 replica)
        return total.value() / max(len(dataloader), 1)     # global-batch loss: identical on every rank

    @torch.no_grad()
    def validate(self, dataloader) -> float:
        self.model.eval()
        total = _DeviceSum(self.device)
        for batch in _progress(dataloader, self.show_progress, '[Pretrain] Val'):
            imu_proj, video_proj = self.model(*self._batch(batch))
            total.add(self.loss_fn(imu_proj, video_proj))
        return total.value() / max(len(dataloader), 1)

    def _extra(self):
        return {'best_val_loss': self.best_val_loss, 'optimizer_state_dict': self.optimizer.state_dict(),
                'scheduler_state_dict': self.scheduler.state_dict()}

    def fit(self, train_loader, val_loader):
        num_epochs = int(self.config.training.pretrain_epochs)
        save_dir = Path(self.config.paths.checkpoints_dir) / 'cross_modal'
        save_dir.mkdir(parents=True, exist_ok=True)
        patience = int(getattr(self.config.training, 'patience', 10))
        save_every = int(getattr(self.config.training, 'save_every', 5))
        save_best_only = bool(getattr(self.config.training, 'save_best_only', True))
        patience_counter = 0
        for epoch in range(self.current_epoch, num_epochs):
            self.current_epoch = epoch
            train_loss = self.train_epoch(train_loader)
            val_loss = self.validate(val_loader)
            self.history['train'].append(train_loss)
            self.history['val'].append(val_loss)
            self.scheduler.step()
            if D.is_main():
                print(f'[Pretrain] epoch={epoch} train_loss={train_loss:.4f} val_loss={val_loss:.4f}')
            self.save_checkpoint(save_dir / 'last.pt', extra=self._extra())
            if val_loss < self.best_val_loss:
                self.best_val_loss = val_loss
                patience_counter = 0
                if save_best_only:
                    self.save_checkpoint(save_dir / 'best_model.pt', extra=self._extra())
            else:
                patience_counter += 1
            if (epoch + 1) % save_every == 0:
                self.save_checkpoint(save_dir / f'checkpoint_epoch_{epoch}.pt', extra=self._extra())
            if patience_counter >= patience:
                print(f'[Pretrain] Early stopping at epoch {epoch}')
                break
        if D.is_main():
            with open(save_dir / 'training_history.json', 'w') as f:
                json.dump(self.history, f, indent=2)


# -----------------------------
#   Classification Trainer  (trainer.py:236-413)
# -----------------------------
class ClassificationTrainer(BaseTrainer):
    """Downstream IMU classification: mode 'linear_probe' (frozen encoder, head only) or 'finetune' (all params,
    encoder lr `train_lr_encoder`, head lr `train_lr_head`); best = max balanced accuracy."""

    def __init__(self, model, config, device: str = 'cuda', mode: str = 'linear_probe', *, grad_reducer=None,
                 show_progress: bool = False):
        super().__init__(model, config, device)
        assert mode in ['linear_probe', 'finetune']
        self.mode = mode
        self.loss_fn = CrossEntropyLoss()
        self.best_bal_acc = 0.0
        self.grad_reducer = grad_reducer
        self.show_progress = show_progress
        if mode == 'linear_probe':
            for p in model.imu_encoder.parameters():
                p.requires_grad = False
            self.optimizer = FusedAdamW(model.classifier.parameters(), lr=config.training.train_lr_head,
                                        weight_decay=config.training.pretrain_weight_decay, max_grad_norm=1.0,
                                        clip_params=model.parameters())
        else:
            if hasattr(model, 'unfreeze_encoder'):
                model.unfreeze_encoder()
            else:
                for p in model.imu_encoder.parameters():
                    p.requires_grad = True
            self.optimizer = FusedAdamW(
                [{'params': model.imu_encoder.parameters(), 'lr': config.training.train_lr_encoder},
                 {'params': model.classifier.parameters(), 'lr': config.training.train_lr_head}],
                weight_decay=config.training.pretrain_weight_decay, max_grad_norm=1.0,
                clip_params=model.parameters())
        self.scheduler = CosineAnnealingLR(self.optimizer, T_max=max(int(config.training.train_epochs), 1),
                                           eta_min=1e-7)

    def _batch(self, batch):
        imu = batch['imu'].to(self.device, non_blocking=True)
        labels = batch['label']
        if not labels.is_cuda:        # host labels: range-checked on the host, then copied (no device sync)
            C = self.model.classifier[-1].out_features
            bad = (labels < 0) | (labels >= C)
            if bool(bad.any()):
                raise IndexError(f'Target {int(labels[bad][0])} is out of bounds.')
        return imu, labels.to(self.device, dtype=torch.int64, non_blocking=True).contiguous()

    def _score(self, logits, labels, correct_list, preds=None):
        """Accuracy bookkeeping from the fused kernel (first argmax == torch.argmax, correct count on device)."""
        corr = torch.empty(1, dtype=torch.int32, device=logits.device)
        pred = torch.empty(labels.shape[0], dtype=torch.int64, device=logits.device) if preds is not None else None
        K.cross_entropy(logits.detach().float().contiguous(), labels, pred=pred, correct=corr)
        correct_list.append(corr)
        if preds is not None:
            preds.append(pred)

    def _global_share(self, n_local):
        """B_local / B_global as a device scalar (one all-reduce, no host sync); None without data parallelism."""
        if D.world_size() == 1:
            return None
        t = torch.full((1,), float(n_local), dtype=torch.float32, device=self.device)
        D.all_reduce_sum_(t)
        return float(n_local) / t

    def train_step(self, imu, labels):
        """trainer.py:296-305.  Under data parallelism the local mean CE is scaled by B_local / B_global: the
        SUM all-reduce of the gradients then yields the gradient of the global-batch mean, which is what
        DataParallel computes (outputs gathered on device 0, one CE mean over the whole batch).  Returns the
        logits and this rank's share of the global-batch loss (the shares sum to the global loss)."""
        logits = self.model(imu)
        loss = self.loss_fn(logits, labels)
        share = self._global_share(labels.shape[0])
        if share is not None:
            loss = loss * share
        self.optimizer.zero_grad(set_to_none=True)
        if self.grad_reducer is not None:
            self.grad_reducer.start_step()
        loss.backward()
        if self.grad_reducer is not None:
            self.grad_reducer.finish()
        self.optimizer.step()          # clip_grad_norm_(model.parameters(), 1.0) + AdamW.step (trainer.py:303-304)
        return logits, loss

    def train_epoch(self, dataloader) -> Dict[str, float]:
        self.model.train()
        loss_sum = _DeviceSum(self.device)
        correct, total = [], 0
        for batch in _progress(dataloader, self.show_progress, f'[Cls:{self.mode}] Epoch {self.current_epoch}'):
            imu, labels = self._batch(batch)
            logits, loss = self.train_step(imu, labels)
            loss_sum.add(loss)
            self._score(logits, labels, correct)
            total += labels.shape[0]
        D.broadcast_buffers(self.model)     # rank 0's BN running statistics (DataParallel's device-0 replica)
        counts = torch.tensor([float(torch.cat(correct).sum().item()) if correct else 0.0, float(total)],
                              device=self.device)
        D.all_reduce_sum_(counts)
        D.all_reduce_sum_(loss_sum.t)
        n_ok, total = counts.tolist()
        return {'loss': loss_sum.value() / max(len(dataloader), 1), 'accuracy': 100.0 * n_ok / max(total, 1)}

    @torch.no_grad()
    def validate(self, dataloader) -> Dict[str, float]:
        """trainer.py:320-353.  The loss is the mean over batches of each (global) batch's mean CE.  Under data
        parallelism no collective runs per batch: each rank keeps its per-batch Σ CE and row counts on
        the device, and ONE all_gather_object at the end (with the predictions) forms every global batch i as the
        union of the ranks' i-th shards — also when ranks hold different numbers of batches."""
        self.model.eval()
        ce_means, counts = [], []
        correct, preds, labels_all, total = [], [], [], 0
        for batch in _progress(dataloader, self.show_progress, f'[Cls:{self.mode}] Val'):
            imu, labels = self._batch(batch)
            logits = self.model(imu)
            ce_means.append(self.loss_fn(logits, labels).reshape(1))
            counts.append(int(labels.shape[0]))
            self._score(logits, labels, correct, preds)
            labels_all.append(labels)
            total += labels.shape[0]
        from sklearn.metrics import balanced_accuracy_score, f1_score
        all_preds = torch.cat(preds).cpu().numpy().tolist() if preds else []
        all_labels = torch.cat(labels_all).cpu().numpy().tolist() if labels_all else []
        n_ok = int(torch.cat(correct).sum().item()) if correct else 0
        sums = [c * n for c, n in zip(torch.cat(ce_means).double().cpu().tolist(), counts)] if ce_means else []
        if D.world_size() > 1:         # metrics of the whole validation set (every rank's shard)
            import torch.distributed as tdist
            parts = [None] * D.world_size()
            tdist.all_gather_object(parts, (all_preds, all_labels, n_ok, total, sums, counts))
            all_preds = [x for pr in parts for x in pr[0]]
            all_labels = [x for pr in parts for x in pr[1]]
            n_ok, total = sum(pr[2] for pr in parts), sum(pr[3] for pr in parts)
            nb = max(len(pr[4]) for pr in parts)
            sums = [sum(pr[4][i] for pr in parts if i < len(pr[4])) for i in range(nb)]
            counts = [sum(pr[5][i] for pr in parts if i < len(pr[5])) for i in range(nb)]
        batch_means = [s / max(n, 1) for s, n in zip(sums, counts)]
        return {'loss': sum(batch_means) / max(len(batch_means), 1),
                'accuracy': 100.0 * n_ok / max(total, 1),
                'balanced_accuracy': 100.0 * balanced_accuracy_score(all_labels, all_preds),
                'f1_macro': 100.0 * f1_score(all_labels, all_preds, average='macro')}

    def _extra(self):
        return {'best_balanced_accuracy': self.best_bal_acc, 'optimizer_state_dict': self.optimizer.state_dict(),
                'scheduler_state_dict': self.scheduler.state_dict()}

    def fit(self, train_loader, val_loader) -> float:
        num_epochs = int(self.config.training.train_epochs)
        save_dir = Path(self.config.paths.checkpoints_dir) / f'classifier_{self.mode}'
        save_dir.mkdir(parents=True, exist_ok=True)
        patience = int(getattr(self.config.training, 'patience', 10))
        patience_counter = 0
        for epoch in range(self.current_epoch, num_epochs):
            self.current_epoch = epoch
            train_metrics = self.train_epoch(train_loader)
            val_metrics = self.validate(val_loader)
            self.history['train'].append(train_metrics)
            self.history['val'].append(val_metrics)
            self.scheduler.step()
            if D.is_main():
                print(f"[Cls:{self.mode}] epoch={epoch} "
                  f"train_loss={train_metrics['loss']:.4f} train_acc={train_metrics['accuracy']:.2f}% | "
                  f"val_loss={val_metrics['loss']:.4f} val_acc={val_metrics['accuracy']:.2f}% "
                  f"val_bal_acc={val_metrics['balanced_accuracy']:.2f}% val_f1={val_metrics['f1_macro']:.2f}%")
            self.save_checkpoint(save_dir / 'last.pt', extra=self._extra())
            if val_metrics['balanced_accuracy'] > self.best_bal_acc:
                self.best_bal_acc = float(val_metrics['balanced_accuracy'])
                patience_counter = 0
                self.save_checkpoint(save_dir / 'best_model.pt', extra=self._extra())
            else:
                patience_counter += 1
            if patience_counter >= patience:
                print(f'[Cls:{self.mode}] Early stopping at epoch {epoch}')
                break
        if D.is_main():
            with open(save_dir / 'training_history.json', 'w') as f:
                json.dump(self.history, f, indent=2)
        return self.best_bal_acc
