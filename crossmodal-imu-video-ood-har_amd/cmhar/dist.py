"""Data parallelism: one process per GPU, torch.distributed over RCCL (backend "nccl") / gloo on CPU.

Replaces the reference's single-process `nn.DataParallel` (main.py:89-93) with the same semantics:
* the SigLIP loss is taken over the GLOBAL batch (cmhar.losses all-gathers the two embedding matrices);
* BatchNorm statistics are per replica (each rank normalises its own shard); the running statistics that count
  are rank 0's — DataParallel keeps those of the device-0 replica — and `broadcast_buffers` copies them to every
  rank before evaluation and checkpointing (the trainers call it at the end of each training epoch);
* parameter gradients are SUMMED over replicas (DataParallel's reduce-add), then clipped and stepped
  identically on every rank (weights stay bit-identical without a broadcast);
* only rank 0 writes files (`is_main()`; the reference process saves once, trainer.py:188-230).

Gradient traffic, two kinds of buckets, both all-reduced asynchronously (RCCL runs on its own stream, so each
bucket overlaps the rest of backward) and launched strictly in bucket order, so every rank issues the same
collective sequence whatever order its hooks fire in:
* sink buckets — a VideoMAE backbone (98 % of the parameters at VideoMAE-B) writes its gradients straight into
  one flat fp32 buffer (cmhar.grads.FlatGradSink) in backward-production order; the buffer is cut into ~32 MB
  buckets at parameter boundaries, each launched when its last layer is done — no copies;
* hook buckets — every other trainable parameter (IMU encoder, heads, and any other backbone: R3D-18, the
  cross-attention fusion model) in reverse registration order (≈ backward order), cut into ~32 MB buckets; a
  `post_accumulate_grad` hook marks each gradient final, a full bucket is flattened into its persistent buffer
  and launched, and `finish()` scatters the reduced values back into `.grad`.
Parameters whose gradient stays None on every rank (unused parameters such as `CrossModalModel.temperature`)
are skipped consistently: a bucket that never fills is reduced in `finish()` over its non-None gradients.
"""
from __future__ import annotations

import os
from typing import List, Optional

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


def world_size(group=None) -> int:
    return dist.get_world_size(group) if dist.is_initialized() else 1


def is_main(group=None) -> bool:
    """True on the one process that writes checkpoints / history files (rank 0, or no process group)."""
    return not dist.is_initialized() or dist.get_rank(group) == 0


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


def _is_sink_backbone(backbone) -> bool:
    from .videomae import VideoMAEBackbone
    return isinstance(backbone, VideoMAEBackbone)


class _Bucket:
    __slots__ = ('params', 'kind', 'start', 'end', 'ready', 'launched', 'flat', 'live')

    def __init__(self, params, kind, start=0, end=0):
        self.params, self.kind, self.start, self.end = params, kind, start, end
        self.ready, self.launched, self.flat, self.live = set(), False, None, None


class GradReducer:
    """Bucketed, backward-overlapped gradient all-reduce (SUM) for one model replica per process.

    `backbone`: the model's video backbone.  A VideoMAE backbone gets the zero-copy flat gradient sink; any other
    backbone (or None) is covered by the hook buckets like the rest of the model."""

    def __init__(self, model: torch.nn.Module, backbone=None, bucket_mb: float = 32.0, group=None):
        self.model = model
        self.group = group
        self.world = world_size(group)
        self.sink = None
        self.pending = []
        self.active = False
        self.buckets: List[_Bucket] = []
        limit = max(int(bucket_mb * (1 << 20) / 4), 1)
        sink_params = set()
        if backbone is not None and _is_sink_backbone(backbone):
            order = backbone_param_order(backbone)
            self.sink = FlatGradSink(order, order[0].device, on_ready=self._on_sink_ready)
            backbone._grad_sink = self.sink
            cur, start = [], 0
            for p in self.sink.order:               # cut the flat buffer at parameter boundaries
                cur.append(p)
                size = self.sink.offsets[p] + p.numel() - start
                if size >= limit:
                    self.buckets.append(_Bucket(cur, 'sink', start, start + size))
                    start += size
                    cur = []
            if cur:
                self.buckets.append(_Bucket(cur, 'sink', start, self.sink.numel))
            sink_params = set(self.sink.order)
        self.rest = [p for p in model.parameters() if p.requires_grad and p not in sink_params]
        cur, size = [], 0
        for p in reversed(self.rest):
            cur.append(p)
            size += p.numel()
            if size >= limit:
                self.buckets.append(_Bucket(cur, 'hook'))
                cur, size = [], 0
        if cur:
            self.buckets.append(_Bucket(cur, 'hook'))
        self._bucket_of = {p: i for i, b in enumerate(self.buckets) for p in b.params}
        self._next = 0                              # buckets launch strictly in index order
        self._hooks = []
        if self.world > 1:
            for p in self.rest:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_hook))

    # -- readiness -------------------------------------------------------------------------------------------
    def _mark(self, p):
        bi = self._bucket_of.get(p)
        if bi is None:
            return
        b = self.buckets[bi]
        b.ready.add(p)
        self._launch_ready()

    def _on_sink_ready(self, params):
        if self.world == 1:
            return
        for p in params:
            self._mark(p)

    def _on_hook(self, p):
        if self.active:
            self._mark(p)

    def _launch_ready(self):
        while self._next < len(self.buckets):
            b = self.buckets[self._next]
            if len(b.ready) != len(b.params):
                return
            self._launch(b)
            self._next += 1

    def _launch(self, b: _Bucket):
        if b.kind == 'sink':
            self.pending.append(dist.all_reduce(self.sink.flat[b.start:b.end], group=self.group, async_op=True))
        else:
            live = [p for p in b.params if p.grad is not None]
            b.live = live
            if live:
                n = sum(p.numel() for p in live)
                if b.flat is None or b.flat.numel() != n or b.flat.device != live[0].grad.device:
                    b.flat = torch.empty(n, dtype=torch.float32, device=live[0].grad.device)
                torch.cat([p.grad.reshape(-1).float() for p in live], out=b.flat)
                self.pending.append(dist.all_reduce(b.flat, group=self.group, async_op=True))
        b.launched = True

    # -- step protocol ---------------------------------------------------------------------------------------
    def start_step(self):
        for b in self.buckets:
            b.ready, b.launched, b.live = set(), False, None
        self._next = 0
        self.pending = []
        self.active = self.world > 1

    def finish(self):
        """Call after loss.backward(): launches the buckets that never filled (parameters without a gradient),
        waits for every all-reduce and writes the hook buckets' reduced values back into `.grad`."""
        self.active = False
        if self.world == 1:
            return
        for b in self.buckets[self._next:]:
            self._launch(b)
        self._next = len(self.buckets)
        for w in self.pending:
            w.wait()
        self.pending = []
        for b in self.buckets:
            if b.kind == 'hook' and b.live:
                off = 0
                for p in b.live:
                    n = p.numel()
                    p.grad.copy_(b.flat[off:off + n].view_as(p.grad))
                    off += n

    def close(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []


def broadcast_parameters(model: torch.nn.Module, src: int = 0, group=None):
    """Make every replica start from rank `src`'s parameters and buffers."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    with torch.no_grad():
        for t in list(model.parameters()) + list(model.buffers()):
            dist.broadcast(t.data, src, group=group)


def broadcast_buffers(model: torch.nn.Module, src: int = 0, group=None):
    """Copy rank `src`'s buffers (BatchNorm running_mean / running_var / num_batches_tracked) to every rank:
    under DataParallel the module's running statistics are the device-0 replica's (torch data_parallel.py
    `replicate` shares device 0's buffers with the module), so evaluation and checkpoints use rank 0's."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    with torch.no_grad():
        for t in model.buffers():
            dist.broadcast(t.data, src, group=group)


def all_reduce_sum_(t: torch.Tensor, group=None) -> torch.Tensor:
    """In-place SUM over ranks (no-op without a process group)."""
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, group=group)
    return t
