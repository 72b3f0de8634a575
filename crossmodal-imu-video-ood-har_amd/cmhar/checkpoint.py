"""Checkpoint interchange with the reference.

The drop-in modules emit the reference's exact `state_dict` keys and shapes and `FusedAdamW` keeps torch AdamW's
state layout, so the reference's files load unchanged:

* `BaseTrainer.save_checkpoint` dicts (src/train/trainer.py:38-48): {epoch, model_state_dict, history, + extras
  such as optimizer_state_dict / scheduler_state_dict / best_val_loss} — `resume()` restores all of it (the
  reference's own `load_checkpoint`, trainer.py:50-56, restores model/epoch/history only; `resume` also restores the
  optimizer and LR schedule so training continues bit-for-bit where it stopped);
* DataParallel-era files whose keys carry `module.` (main.py:158-161) — `strip_module_prefix`;
* the bare final state_dict of main.py:110-124 — `save_final_state_dict`;
* the classification stage's encoder hand-off (main.py:150-167) — `load_pretrained_encoder`.

Every load uses `torch.load(..., weights_only=True)`: nothing in a checkpoint file is executed.
"""
from __future__ import annotations

import copy
from pathlib import Path
from typing import Dict, Tuple

import torch


def strip_module_prefix(state: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """main.py:158-161: drop one leading `module.` (DataParallel) from every key when present."""
    if any(k.startswith('module.') for k in state):
        return {k.replace('module.', '', 1): v for k, v in state.items()}
    return state


def load_checkpoint_file(path, map_location='cpu') -> dict:
    return torch.load(str(path), map_location=map_location, weights_only=True)


def resume(trainer, path, strict: bool = True, restore_optimizer: bool = True) -> dict:
    """Restore a trainer (cmhar.trainer.CrossModalTrainer / ClassificationTrainer) from a checkpoint written by the
    reference's BaseTrainer.save_checkpoint (or ours: same format)."""
    ckpt = load_checkpoint_file(path, map_location=trainer.device)
    trainer.model.load_state_dict(strip_module_prefix(ckpt['model_state_dict']), strict=strict)
    trainer.current_epoch = int(ckpt.get('epoch', 0))
    trainer.history = ckpt.get('history', {'train': [], 'val': []})
    if restore_optimizer and 'optimizer_state_dict' in ckpt:
        trainer.optimizer.load_state_dict(ckpt['optimizer_state_dict'])
        # (the backbone's bf16 weight packs re-cast themselves: load_state_dict bumped the masters' versions)
    if restore_optimizer and 'scheduler_state_dict' in ckpt:
        trainer.scheduler.load_state_dict(ckpt['scheduler_state_dict'])
    for key in ('best_val_loss', 'best_balanced_accuracy'):
        if key in ckpt:
            setattr(trainer, 'best_val_loss' if key == 'best_val_loss' else 'best_bal_acc', ckpt[key])
    return ckpt


def save_final_state_dict(model, path) -> Path:
    """main.py:110-124: the bare (un-wrapped) state_dict."""
    path = Path(path)
    path.parent.mkdir(parents=True, exist_ok=True)
    m = model.module if isinstance(model, torch.nn.DataParallel) else model
    torch.save(m.state_dict(), str(path))
    return path


def load_pretrained_encoder(config, checkpoint_path, device='cuda') -> Tuple[torch.nn.Module, torch.nn.Module]:
    """main.py:150-167: CrossModalModel from a pretraining checkpoint (strict), returns (model, deep copy of its
    IMU encoder) for the classification stage."""
    from .models import CrossModalModel
    ckpt = load_checkpoint_file(checkpoint_path, map_location='cpu')
    model = CrossModalModel(config)
    model.load_state_dict(strip_module_prefix(ckpt['model_state_dict']), strict=True)
    model = model.to(device)
    return model, copy.deepcopy(model.imu_encoder)
