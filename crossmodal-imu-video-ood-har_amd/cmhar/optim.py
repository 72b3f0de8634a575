"""Gradient clipping and AdamW as multi-tensor HIP launches (replaces `torch.nn.utils.clip_grad_norm_` and
`torch.optim.AdamW.step` as used by `CrossModalTrainer`, src/train/trainer.py:74-78,140-141).

Both are HBM-bound passes over the 88.4 M fp32 parameters.  `clip_grad_norm_` = one sum-of-squares launch over
a chunk table + one tiny final launch (total norm and clip coefficient stay on the device: no host sync) + one
in-place scale launch.  `FusedAdamW.step` = one launch that reads p, g, m, v and writes p, m, v and the
parameter's compute shadow (bf16 weight pack / fp32 bias pack, see cmhar.weights) in the same pass, with
torch.optim.AdamW's arithmetic (step scalars computed on the host in double precision, as torch does).
"""
from __future__ import annotations

import math
from typing import Iterable, List

import numpy as np
import torch

from . import _lib as L
from .weights import MT_TENSOR, chunk_list, to_device_bytes


class _Table:
    """Device tensor + chunk tables for a list of parameters, rebuilt only when a pointer changes."""

    def __init__(self):
        self.key = None
        self.dev_t = self.dev_c = None
        self.nchunks = 0

    def get(self, rows, device):
        key = tuple(tuple(int(x) for x in r) for r in rows)
        if key != self.key:
            tab = np.zeros(len(rows), dtype=MT_TENSOR)
            for i, r in enumerate(rows):
                tab[i] = r
            ch = chunk_list([r[6] for r in rows])
            self.dev_t = to_device_bytes(tab, device)
            self.dev_c = to_device_bytes(ch, device)
            self.nchunks = len(ch)
            self.key = key
        return self.dev_t, self.dev_c, self.nchunks


_NORM_TABLES = {}


def clip_grad_norm_(parameters, max_norm: float, norm_type: float = 2.0, error_if_nonfinite: bool = False,
                    foreach=None) -> torch.Tensor:
    """torch.nn.utils.clip_grad_norm_ (L2): returns the total norm as a 0-dim DEVICE tensor (no sync)."""
    if norm_type != 2.0:
        raise NotImplementedError('only the L2 norm is on the accelerated path')
    if isinstance(parameters, torch.Tensor):
        parameters = [parameters]
    params = [p for p in parameters if p.grad is not None]
    if not params:
        return torch.tensor(0.0)
    return _grad_norm(params, float(max_norm), apply_clip=True)[0]


def _grad_norm(params, max_norm, apply_clip):
    """[total L2 norm, clip coefficient min(max_norm / (norm + 1e-6), 1)] as a device tensor; with apply_clip the
    gradients are scaled in place (clip_grad_norm_)."""
    dev = params[0].grad.device
    rows = [(p.data_ptr(), p.grad.data_ptr(), 0, 0, 0, 0, p.grad.numel(), 0.0, 1.0) for p in params]
    tab = _NORM_TABLES.setdefault(str(dev), _Table())
    t, c, n = tab.get(rows, dev)
    part = torch.empty(max(n, 1), dtype=torch.float32, device=dev)
    out = torch.empty(2, dtype=torch.float32, device=dev)
    L.call('cmhar_mt_grad_norm', t.data_ptr(), c.data_ptr(), n, part.data_ptr(), out.data_ptr(), max_norm,
           int(apply_clip), L.stream(dev))
    return out


class FusedAdamW(torch.optim.Optimizer):
    """torch.optim.AdamW (amsgrad=False, maximize=False) as one multi-tensor HIP launch per step.

    State layout matches torch (`state[p] = {'step', 'exp_avg', 'exp_avg_sq'}`), so optimizer state dicts
    interchange.  `shadow_sources`: modules whose `_packs` (cmhar.weights.PackedWeights) hold compute copies of
    parameters; those copies are rewritten in the same pass.

    `max_grad_norm` (opt-in): `step()` first performs trainer.py:140's `clip_grad_norm_(params, max_grad_norm)` over
    `clip_params` (the reference clips over `model.parameters()`, trainer.py:140/304 — the trainers pass exactly that;
    default: every parameter of the optimizer) that have a gradient — the norm pass as in `clip_grad_norm_`, but the clip
    coefficient is applied inside the AdamW pass instead of by a separate in-place scale pass over the gradients
    (one read + one write of every gradient less).  The update is bit-identical to clip-then-step.  With
    `write_clipped_grad=True` (default) the AdamW pass also stores the clipped gradient back, so `.grad` after the
    step is exactly what `clip_grad_norm_` leaves; `False` leaves `.grad` unclipped (saves that write too).  The
    total norm of the last step is `last_grad_norm` (0-dim device tensor, as `clip_grad_norm_` returns).
    Gradients in `clip_params` that the optimizer does not own enter the norm; with `write_clipped_grad=True` they are
    scaled in place by the clip coefficient (one multi-tensor multiply), exactly as `clip_grad_norm_` would leave them,
    with `False` they are left unclipped like the owned ones (every `.grad` then holds the unclipped gradient)."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, shadow_sources=(),
                 max_grad_norm=None, write_clipped_grad=True, clip_params=None):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self.shadow_sources = list(shadow_sources)
        self._tables = {}
        self.max_grad_norm = max_grad_norm
        self.write_clipped_grad = bool(write_clipped_grad)
        self.last_grad_norm = None
        self.clip_params = None if clip_params is None else list(clip_params)

    def _slots(self):
        slots = {}
        packs = []
        for m in self.shadow_sources:
            pk = getattr(m, '_packs', None)
            if pk is not None and pk.dtype != torch.float16:   # fp16 (inference) packs are refreshed by version
                slots.update(pk.slots)
                packs.append(pk)
        return slots, packs

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        slots, packs = self._slots()
        gscale = None
        if self.max_grad_norm is not None:
            owned = [p for g in self.param_groups for p in g['params'] if p.grad is not None]
            if self.clip_params is None:
                allp, extra = owned, []
            else:
                ids = {id(p) for p in owned}
                allp = [p for p in self.clip_params if p.grad is not None]
                extra = [p.grad for p in allp if id(p) not in ids]
            if allp:
                norm_out = _grad_norm(allp, float(self.max_grad_norm), apply_clip=False)
                self.last_grad_norm = norm_out[0]
                gscale = norm_out
                # gradients this optimizer does not own are scaled in place whatever write_clipped_grad says: another
                # optimizer may step them, and must see them clipped as clip_grad_norm_ leaves them; the
                # owned ones are clipped inside the AdamW pass (written back only with write_clipped_grad)
                if extra:
                    torch._foreach_mul_(extra, norm_out[1])
        for gi, group in enumerate(self.param_groups):
            b1, b2 = group['betas']
            lr, eps, wd = group['lr'], group['eps'], group['weight_decay']
            rows = []
            step_ts = []
            dev = None
            for p in group['params']:
                if p.grad is None:
                    continue
                if p.grad.is_sparse or p.grad.dtype != torch.float32 or p.dtype != torch.float32:
                    raise RuntimeError('FusedAdamW handles dense fp32 parameters and gradients')
                st = self.state[p]
                if len(st) == 0:
                    st['step'] = torch.tensor(0.0)
                    st['exp_avg'] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st['exp_avg_sq'] = torch.zeros_like(p, memory_format=torch.preserve_format)
                step_ts.append(st['step'])
                bf, cp = slots.get(p, (0, 0))
                rows.append((p.data_ptr(), p.grad.data_ptr(), st['exp_avg'].data_ptr(),
                             st['exp_avg_sq'].data_ptr(), bf, cp, p.numel(), float(wd), 1.0))
                dev = p.device
            if not rows:
                continue
            # the per-parameter step counters (torch's state layout: 0-dim CPU tensors) in one foreach op and one
            # host read, not a tensor add + .item() per parameter (~300 per step on the host)
            torch._foreach_add_(step_ts, 1)
            sv = torch.stack(step_ts)
            lo, hi = sv.aminmax()
            if lo.item() != hi.item():
                raise RuntimeError('parameters of one group at different step counts')
            step = int(hi.item())
            bc1 = 1.0 - b1 ** step
            bc2 = 1.0 - b2 ** step
            t, c, n = self._tables.setdefault(gi, _Table()).get(rows, dev)
            L.call('cmhar_mt_adamw_clip', t.data_ptr(), c.data_ptr(), n, float(lr), float(1.0 - b1), float(b2),
                   float(1.0 - b2), float(eps), float(lr / bc1), float(math.sqrt(bc2)),
                   None if gscale is None else gscale.data_ptr(), int(self.write_clipped_grad), L.stream(dev))
        for pk in packs:
            pk.mark_fresh()
        return loss
