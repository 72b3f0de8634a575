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
  cross-attention fusion model), cut into ~32 MB buckets in the order the first step's backward produced them
  (reverse registration order until then); a `post_accumulate_grad` hook marks each gradient final, a full
  bucket is flattened into its persistent buffer on a communication stream that waits on every stream that
  produced its gradients, and launched; `finish()` scatters the reduced values back into `.grad`.
Parameters whose gradient stays None on every rank (unused parameters such as `CrossModalModel.temperature`)
sit, after the first step, in one trailing bucket reduced in `finish()`.  Every hook bucket is all-reduced at its
full size on every rank (a gradient that is None on this rank contributes zeros), so ranks that disagree on which
gradients are None in a later step still issue identical collectives: a parameter that received gradients in the
first step gets the sum of the other ranks' even where its own is None (DataParallel's reduce-add over replicas);
one of the trailing bucket's keeps None where it had none locally (the first step's agreement check covers that
step only).
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
    from .cnn2d import MobileNetV2Features, ResNet18Features
    from .r3d import R3D18
    from .videomae import VideoMAEBackbone
    return isinstance(backbone, (VideoMAEBackbone, R3D18, ResNet18Features, MobileNetV2Features))


def sink_param_order(backbone) -> List[torch.nn.Parameter]:
    """The flat gradient buffer's layout for a sink backbone: its backward-production order."""
    from . import cnn2d, r3d
    if isinstance(backbone, r3d.R3D18):
        return r3d.unit_param_order(backbone)
    if isinstance(backbone, (cnn2d.ResNet18Features, cnn2d.MobileNetV2Features)):
        return cnn2d.unit_param_order(backbone)
    return backbone_param_order(backbone)


class _Bucket:
    __slots__ = ('params', 'kind', 'start', 'end', 'ready', 'launched', 'flat', 'live', 'streams', 'fill', 'ones')

    def __init__(self, params, kind, start=0, end=0, fill=False):
        self.params, self.kind, self.start, self.end = params, kind, start, end
        self.ready, self.launched, self.flat, self.live, self.streams = set(), False, None, None, {}
        self.ones = None      # presence flags of a fully-live hook bucket (see GradReducer._flatten_and_reduce)
        self.fill = fill      # hook bucket filled in the learning step (the trailing one holds never-used parameters)


def _cut(params, limit):
    """Consecutive groups of `params` of at least `limit` elements (the last may be smaller)."""
    out, cur, size = [], [], 0
    for p in params:
        cur.append(p)
        size += p.numel()
        if size >= limit:
            out.append(cur)
            cur, size = [], 0
    if cur:
        out.append(cur)
    return out


class GradReducer:
    """Bucketed, backward-overlapped gradient all-reduce (SUM) for one model replica per process.

    `backbone`: the model's video backbone.  Every cmhar video backbone (VideoMAE, R3D-18, the per-frame ResNet-18 /
    MobileNetV2) gets the zero-copy flat gradient sink (its backward writes every parameter gradient straight into
    the bucket buffer); any other backbone (or None) is covered by the hook buckets like the rest of the model.

    Hook buckets are first cut in reverse registration order.  That order is only a guess at backward order, and a
    bucket holding a parameter that never receives a gradient (`CrossModalModel.temperature` / `bias`,
    models.py:267-268) would never fill and would hold back every later bucket until `finish()`.  So the first
    step records the order in which the hooks actually fire; `finish()` of that step takes rank 0's order (one
    `broadcast_object_list`, so every rank cuts identical buckets), rebuilds the hook buckets from it and puts the
    parameters that never fired into one trailing bucket reduced in `finish()`.  From the second step on every
    hook bucket goes out as soon as its last gradient is accumulated (DDP's bucket-rebuild rule).

    Streams: a hook bucket's gradients can come from different HIP streams (the IMU branch of `CrossModalModel`
    runs its backward on a side stream, the video backbone on the main stream).  Each hook records the stream
    its gradient was produced on; the bucket is flattened and launched on a dedicated communication stream that
    first waits on every one of those streams, and `finish()` makes the caller's stream wait on the collectives
    before the reduced values are copied back into `.grad`."""

    def __init__(self, model: torch.nn.Module, backbone=None, bucket_mb: float = 32.0, group=None,
                 reduce_single: bool = False):
        self.model = model
        self.group = group
        self.world = world_size(group)
        # reduce_single: run the whole bucket / hook / collective protocol even in a one-rank group (a SUM over one
        # rank is the identity) — exercises the RCCL path on a one-GPU machine, where two ranks cannot share the GPU
        self._reduce = self.world > 1 or (reduce_single and dist.is_initialized())
        self.sink = None
        self.pending = []
        self.active = False
        self._next = 0                              # first bucket not yet launched (reset by start_step)
        self.buckets: List[_Bucket] = []
        self.limit = max(int(bucket_mb * (1 << 20) / 4), 1)
        sink_params = set()
        if backbone is not None and _is_sink_backbone(backbone):
            order = sink_param_order(backbone)
            self.sink = FlatGradSink(order, order[0].device, on_ready=self._on_sink_ready)
            backbone._grad_sink = self.sink
            self._sink_owner = backbone
            cur, start = [], 0
            for p in self.sink.order:               # cut the flat buffer at parameter boundaries
                cur.append(p)
                size = self.sink.offsets[p] + p.numel() - start
                if size >= self.limit:
                    self.buckets.append(_Bucket(cur, 'sink', start, start + size))
                    start += size
                    cur = []
            if cur:
                self.buckets.append(_Bucket(cur, 'sink', start, self.sink.numel))
            sink_params = set(self.sink.order)
        self.n_sink = len(self.buckets)
        self.rest = [p for p in model.parameters() if p.requires_grad and p not in sink_params]
        self._set_hook_buckets(_cut(list(reversed(self.rest)), self.limit))
        self.learned = False                        # hook-bucket order taken from an observed backward yet?
        self._fired = []                            # hook firing order of the current step (learning step only)
        self._comm = None
        self.launched_before_finish = 0             # buckets in flight when backward returned (last step)
        self.n_collectives = 0                      # all-reduces issued (last step)
        self._hooks = []
        if self._reduce:
            for p in self.rest:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_hook))

    def _set_hook_buckets(self, groups, n_fill=0):
        self.buckets = self.buckets[:self.n_sink] + [_Bucket(g, 'hook', fill=i < n_fill) for i, g in enumerate(groups)]
        self._bucket_of = {p: i for i, b in enumerate(self.buckets) for p in b.params}

    def _comm_stream(self, device):
        if device.type != 'cuda':
            return None
        if self._comm is None:
            self._comm = torch.cuda.Stream(device)
        return self._comm

    # -- readiness -------------------------------------------------------------------------------------------
    def _mark(self, p):
        bi = self._bucket_of.get(p)
        if bi is None:
            return
        b = self.buckets[bi]
        if b.launched:
            raise RuntimeError('a parameter received a second gradient contribution after its bucket was '
                               'all-reduced: a second backward inside one start_step()/finish() window (gradient '
                               'accumulation) or a parameter used twice in one step; not supported by GradReducer')
        b.ready.add(p)
        self._launch_ready()

    def _on_sink_ready(self, params):
        # a backward outside a start_step()/finish() window (after finish() or close(), an evaluation backward)
        # leaves its gradients local: launching buckets from it would start an all-reduce on this rank only
        if not self._reduce or not self.active:
            return
        for p in params:
            self._mark(p)

    def _on_hook(self, p):
        if not self.active:
            return
        if p.grad is not None and p.grad.is_cuda:
            s = torch.cuda.current_stream(p.grad.device)
            bi = self._bucket_of.get(p)
            if bi is not None:
                self.buckets[bi].streams[s.cuda_stream] = s
        if not self.learned:
            self._fired.append(p)
        self._mark(p)

    def _launch_ready(self):
        while self._next < len(self.buckets):
            b = self.buckets[self._next]
            if len(b.ready) != len(b.params):
                return
            if b.kind == 'hook' and not self.learned:
                return     # learning step: hook buckets wait for finish(), which first checks the ranks agree
            self._launch(b)
            self._next += 1

    def _launch(self, b: _Bucket):
        if b.kind == 'sink':
            self.pending.append(dist.all_reduce(self.sink.flat[b.start:b.end], group=self.group, async_op=True))
            self.n_collectives += 1
        else:
            # every rank reduces the bucket at its full size (zeros for gradients that are None here), so the
            # collective is the same on every rank whichever gradients each produced
            b.live = [p for p in b.params if p.grad is not None]
            dev = b.params[0].device
            comm = self._comm_stream(dev)
            if comm is None:
                self._flatten_and_reduce(b)
            else:
                cur = torch.cuda.current_stream(dev)
                comm.wait_stream(cur)
                for s in b.streams.values():
                    if s.cuda_stream != comm.cuda_stream:
                        comm.wait_stream(s)
                with torch.cuda.stream(comm):
                    self._flatten_and_reduce(b)
        b.launched = True

    def _flatten_and_reduce(self, b):
        # [gradients | one presence flag per parameter]: the reduced flags count the ranks that produced each
        # gradient, so that finish() can give a parameter the sum when ANY rank has one and leave it None when none
        # does — the same decision on every rank (a trailing-bucket parameter used by some ranks only)
        n = sum(p.numel() for p in b.params)
        k = len(b.params)
        dev = b.params[0].device
        if b.flat is None or b.flat.numel() != n + k or b.flat.device != dev:
            b.flat = torch.empty(n + k, dtype=torch.float32, device=dev)
            b.ones = torch.ones(k, dtype=torch.float32, device=dev)
        if len(b.live) == k:
            torch.cat([p.grad.reshape(-1).float() for p in b.params] + [b.ones], out=b.flat)
        else:
            b.flat.zero_()
            off = 0
            for p in b.params:
                if p.grad is not None:
                    b.flat[off:off + p.numel()].copy_(p.grad.reshape(-1))
                off += p.numel()
            b.flat[n:].copy_(torch.tensor([float(p.grad is not None) for p in b.params], dtype=torch.float32))
        self.pending.append(dist.all_reduce(b.flat, group=self.group, async_op=True))
        self.n_collectives += 1

    # -- step protocol ---------------------------------------------------------------------------------------
    def start_step(self):
        for b in self.buckets:
            b.ready, b.launched, b.live, b.streams = set(), False, None, {}
        self._next = 0
        self.pending = []
        self.n_collectives = 0
        self._fired = []
        self.active = self._reduce

    def finish(self):
        """Call after loss.backward(): launches the buckets that never filled (parameters without a gradient),
        waits for every all-reduce and writes the hook buckets' reduced values back into `.grad`."""
        self.active = False
        if not self._reduce:
            return
        self.launched_before_finish = self._next
        orders = None if self.learned else self._gather_fired()
        for b in self.buckets[self._next:]:
            self._launch(b)
        self._next = len(self.buckets)
        for w in self.pending:
            w.wait()               # NCCL: the caller's current stream waits on the collective
        self.pending = []
        dst, src = [], []
        for b in self.buckets:
            if b.kind == 'hook' and b.launched and b.flat is not None:
                # a parameter without a local gradient takes the sum when some rank produced one, else stays None;
                # the ranks' counts are read only for such buckets (one small device -> host read, none in a step
                # where every hook parameter has its gradient)
                counts = None
                if any(p.grad is None for p in b.params):
                    counts = b.flat[b.flat.numel() - len(b.params):].tolist()
                off = 0
                for i, p in enumerate(b.params):
                    n = p.numel()
                    red = b.flat[off:off + n].view_as(p)
                    if p.grad is not None:
                        dst.append(p.grad)
                        src.append(red)
                    elif counts[i] > 0:    # produced on another rank this step
                        p.grad = red.to(p.dtype, copy=True)
                    off += n
        if dst:
            torch._foreach_copy_(dst, src)     # the reduced values back into .grad: one multi-tensor launch
        if orders is not None:
            self._learn_order(orders)

    def _gather_fired(self):
        """Every rank's observed hook order of the learning step.  The ranks must agree on WHICH parameters
        received a gradient (as under DataParallel) — otherwise their hook buckets would differ in size and the
        all-reduce would hang — so a mismatch raises here, before any hook bucket is launched."""
        index = {p: i for i, p in enumerate(self.rest)}
        seen, order = set(), []
        for p in self._fired:
            if p not in seen:
                seen.add(p)
                order.append(index[p])
        orders = [None] * self.world
        dist.all_gather_object(orders, order, group=self.group)
        ref = set(orders[0])
        for r, o in enumerate(orders):
            if set(o) != ref:
                self._fired = []
                for w in self.pending:     # the sink buckets' all-reduces (identical on every rank) complete
                    w.wait()
                self.pending = []
                raise RuntimeError(f'GradReducer: rank {r} produced gradients for a different parameter set than '
                                   f'rank 0 in its first step ({len(o)} vs {len(ref)} parameters); every rank must '
                                   f'compute gradients for the same parameters')
        return orders

    def _learn_order(self, orders):
        """Rebuild the hook buckets in rank 0's observed gradient order (identical on every rank)."""
        order = orders[0]
        fired = [self.rest[i] for i in order]
        fired_set = set(fired)
        never = [p for p in reversed(self.rest) if p not in fired_set]
        groups = _cut(fired, self.limit)
        n_fill = len(groups)
        if never:
            groups.append(never)   # unused parameters: one trailing bucket, reduced in finish()
        self._set_hook_buckets(groups, n_fill)
        self._fired = []
        self.learned = True

    def close(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
        self.active = False
        if self.sink is not None:      # detach the flat sink: the backbone allocates its own gradients again
            self.sink.on_ready = None
            if getattr(self._sink_owner, '_grad_sink', None) is self.sink:
                self._sink_owner._grad_sink = None


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
