"""Where backward kernels write parameter gradients.

`AutogradSink` (default): every gradient is a fresh fp32 tensor returned through autograd — exact torch
semantics for any caller (functional autograd, hooks, accumulation into existing `.grad`).

`FlatGradSink` (opt-in, used by `cmhar.dist.DataParallel` and the benchmark): all parameter gradients live in
ONE persistent fp32 buffer laid out in backward-production order (last layer first, QKV weights adjacent), the
wgrad GEMMs write straight into `param.grad` (β = 0 when `.grad` was None — torch's set_to_none semantics — and
β = 1 accumulation otherwise) and the node returns None for those parameters.  Benefits: no per-step gradient
allocation, stable pointers (the fused optimizer's tensor table is built once), and contiguous buckets that the
data-parallel reducer all-reduces while earlier layers are still in backward.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import torch


class AutogradSink:
    direct = False

    def __init__(self):
        self.grads: Dict[torch.nn.Parameter, torch.Tensor] = {}

    def dest(self, params: Sequence[torch.nn.Parameter], shape, device):
        """Destination for the concatenation of `params`' gradients, viewed as `shape`; returns (tensor, beta)."""
        out = torch.empty(shape, dtype=torch.float32, device=device)
        off = 0
        flat = out.view(-1)
        for p in params:
            self.grads[p] = flat[off:off + p.numel()].view(p.shape)
            off += p.numel()
        return out, 0.0

    def done(self, params):
        pass

    def result(self, p):
        return self.grads.get(p)


class FlatGradSink:
    direct = True

    def __init__(self, order: List[torch.nn.Parameter], device, on_ready=None):
        self.order = [p for p in order if p.requires_grad]
        self.offsets = {}
        off = 0
        for p in self.order:
            self.offsets[p] = off
            off += p.numel()
        self.numel = off
        self.flat = torch.zeros(off, dtype=torch.float32, device=device)
        self.on_ready = on_ready

    def view(self, p):
        o = self.offsets[p]
        return self.flat[o:o + p.numel()].view(p.shape)

    def _contiguous(self, params):
        o = self.offsets[params[0]]
        for p in params:
            if self.offsets.get(p) != o:
                return None
            o += p.numel()
        return self.offsets[params[0]]

    def dest(self, params, shape, device):
        for p in params:
            if p not in self.offsets:
                raise KeyError('parameter not registered with the gradient buffer')
        fresh = [p.grad is None for p in params]
        if any(fresh) and not all(fresh):
            raise RuntimeError('mixed None / existing gradients inside one fused gradient group')
        start = self._contiguous(params)
        if start is None:
            raise RuntimeError('fused gradient group is not contiguous in the flat buffer')
        n = sum(p.numel() for p in params)
        out = self.flat[start:start + n].view(shape)
        if all(fresh):
            for p in params:
                p.grad = self.view(p)
            return out, 0.0
        for p in params:
            if p.grad.data_ptr() != self.view(p).data_ptr():
                raise RuntimeError('.grad was replaced by a tensor outside the flat gradient buffer')
        return out, 1.0

    def done(self, params):
        if self.on_ready is not None:
            self.on_ready(params)

    def result(self, p):
        return None          # gradient already in p.grad
