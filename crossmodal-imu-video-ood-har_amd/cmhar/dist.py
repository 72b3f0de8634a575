"""Data parallelism: one process per GPU, torch.distributed over RCCL (backend "nccl") / gloo on CPU.

Replaces the reference's single-process `nn.DataParallel` (main.py:89-93) with the same semantics:
* the SigLIP loss is taken over the GLOBAL batch (cmhar.losses all-gathers the two embedding matrices);
* BatchNorm statistics are per replica (each rank normalises its own shard);
* parameter gradients are SUMMED over replicas (DataParallel's reduce-add), then clipped and stepped
  identically on every rank (weights stay bit-identical without a broadcast).

Gradient traffic: the VideoMAE backbone (98 % of the parameters) writes its gradients into one flat fp32 buffer
(cmhar.grads.FlatGradSink) in backward-production order; the buffer is cut into ~32 MB buckets and each bucket
is all-reduced asynchronously (RCCL runs on its own stream, so it overlaps the remaining backward layers) as
soon as its last layer finishes.  The few small remaining gradients (IMU encoder, heads) are reduced in one
flattened all-reduce at the end of backward.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from .grads import FlatGradSink

_LOSS_GROUP = None
_ENABLED = False


def init_from_env(backend: Optional[str] = None):
    """Initialise the default process group from torchrun's env (RANK/WORLD_SIZE/MASTER_*); returns
    (rank, world_size, local_rank)."""
    global _ENABLED
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = 'nccl' if torch.cuda.is_available() else 'gloo'
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        dist.init_process_group(backend=backend, rank=rank, world_size=world)
    _ENABLED = world > 1
    return rank, world, local


def set_loss_group(group):
    global _LOSS_GROUP
    _LOSS_GROUP = group


def loss_group():
    if _LOSS_GROUP is not None:
        return _LOSS_GROUP
    if _ENABLED and dist.is_initialized() and dist.get_world_size() > 1:
        return dist.group.WORLD
    return None


def backbone_param_order(backbone) -> List[torch.nn.Parameter]:
    """Backward-production order of a VideoMAEBackbone's parameters (final LN, layers last→first, each layer
    in the order its backward emits them, QKV weights and biases adjacent), then the patch embedding."""
    order = []
    if backbone.layernorm is not None:
        order += [backbone.layernorm.weight, backbone.layernorm.bias]
    for layer in reversed(list(backbone.encoder.layer)):
        a = layer.attention.attention
        order += [layer.output.dense.weight, layer.output.dense.bias,
                  layer.intermediate.dense.weight, layer.intermediate.dense.bias,
                  layer.layernorm_after.weight, layer.layernorm_after.bias,
                  layer.attention.output.dense.weight, layer.attention.output.dense.bias,
                  a.query.weight, a.key.weight, a.value.weight]
        if a.query.bias is not None:
            order += [a.query.bias, a.key.bias, a.value.bias]
        order += [layer.layernorm_before.weight, layer.layernorm_before.bias]
    pe = backbone.embeddings.patch_embeddings.projection
    order += [pe.weight, pe.bias]
    return order


class GradReducer:
    """Bucketed, backward-overlapped gradient all-reduce (SUM) for one model replica per process."""

    def __init__(self, model: torch.nn.Module, backbone=None, bucket_mb: float = 32.0, group=None):
        self.model = model
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.backbone = backbone
        self.sink = None
        self.pending = []
        self.buckets = []
        if backbone is not None:
            order = backbone_param_order(backbone)
            dev = order[0].device
            self.sink = FlatGradSink(order, dev, on_ready=self._on_ready)
            backbone._grad_sink = self.sink
            # cut the flat buffer into buckets at parameter boundaries
            limit = int(bucket_mb * (1 << 20) / 4)
            cur, start = [], 0
            for p in self.sink.order:
                cur.append(p)
                size = self.sink.offsets[p] + p.numel() - start
                if size >= limit:
                    self.buckets.append((start, start + size, set(cur)))
                    start += size
                    cur = []
            if cur:
                end = self.sink.numel
                self.buckets.append((start, end, set(cur)))
            self._ready = [set() for _ in self.buckets]
            self._launched = [False] * len(self.buckets)
            self._bucket_of = {p: i for i, b in enumerate(self.buckets) for p in b[2]}
        bb = set(backbone.parameters()) if backbone is not None else set()
        self.rest = [p for p in model.parameters() if p.requires_grad and p not in bb]

    def _on_ready(self, params):
        if self.world == 1:
            return
        for p in params:
            bi = self._bucket_of.get(p)
            if bi is None:
                continue
            self._ready[bi].add(p)
            if not self._launched[bi] and len(self._ready[bi]) == len(self.buckets[bi][2]):
                s, e, _ = self.buckets[bi]
                self.pending.append(dist.all_reduce(self.sink.flat[s:e], group=self.group, async_op=True))
                self._launched[bi] = True

    def start_step(self):
        if self.sink is not None:
            self._ready = [set() for _ in self.buckets]
            self._launched = [False] * len(self.buckets)

    def finish(self):
        """Call after loss.backward(): completes the bucket all-reduces and reduces the remaining grads."""
        if self.world == 1:
            return
        grads = [p.grad for p in self.rest if p.grad is not None]
        if grads:
            flat = torch._utils._flatten_dense_tensors(grads)
            dist.all_reduce(flat, group=self.group)
            for g, r in zip(grads, torch._utils._unflatten_dense_tensors(flat, grads)):
                g.copy_(r)
        for i, launched in enumerate(self._launched if self.sink is not None else []):
            if not launched:   # bucket whose params were not all produced (e.g. frozen) — reduce now
                s, e, _ = self.buckets[i]
                self.pending.append(dist.all_reduce(self.sink.flat[s:e], group=self.group, async_op=True))
        for w in self.pending:
            w.wait()
        self.pending = []


def broadcast_parameters(model: torch.nn.Module, src: int = 0, group=None):
    """Make every replica start from rank `src`'s parameters and buffers."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    with torch.no_grad():
        for t in list(model.parameters()) + list(model.buffers()):
            dist.broadcast(t.data, src, group=group)
