"""SigmoidContrastiveLoss (`src/models/losses.py:9-54`) on the fused cmhar loss kernel.

Same constructor (`init_temperature=10.0, init_bias=-10.0, learnable=True`), same parameters / buffers
(`temperature` = log(init_temperature), `bias`), same value: the reference's BCE-with-logits over
`logits*labels` vs `(labels+1)/2`, which equals mean softplus(-S) over ALL pairs — the
kernel evaluates the reference's per-element formula literally and returns analytic gradients for the
embeddings, the temperature and the bias.

Data parallel (`group=` a torch.distributed process group, or `cmhar.dist` enabled): like the reference's
`nn.DataParallel`, the loss is taken over the GLOBAL batch.  Each rank all-gathers the two (B_local, D) embedding
matrices (RCCL), every rank evaluates the full B_global² similarity matrix (identical loss everywhere) and
keeps the gradient rows of its own shard; summing parameter gradients over ranks then reproduces the single
global-batch gradient DataParallel's reduce-add produces.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _lib as L
from . import kernels as K


def gather_global(a_local, b_local, group):
    """All-gather the two (B_local, D) fp32 embedding matrices of every rank in `group` (rank order) — the
    global batch DataParallel's gather forms on device 0 (torch `data_parallel.py:173-198`).  Returns
    (a_all, b_all, row offset of this rank's shard).  `group=None`: single process, no copy."""
    if group is None:
        return a_local, b_local, 0
    import torch.distributed as dist
    ws = dist.get_world_size(group)
    rk = dist.get_rank(group)
    Bl, D = a_local.shape
    a_all = torch.empty(ws * Bl, D, dtype=a_local.dtype, device=a_local.device)
    b_all = torch.empty(ws * Bl, D, dtype=b_local.dtype, device=b_local.device)
    dist.all_gather_into_tensor(a_all, a_local, group=group)
    dist.all_gather_into_tensor(b_all, b_local, group=group)
    return a_all, b_all, rk * Bl


class _SigLIPFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a_local, b_local, t, bias, group):
        dev = a_local.device
        a_local = a_local.contiguous().float()
        b_local = b_local.contiguous().float()
        Bl, D = a_local.shape
        a_all, b_all, off = gather_global(a_local, b_local, group)
        Bg = a_all.shape[0]
        t_dev = t.detach().reshape(1).to(device=dev, dtype=torch.float32)
        b_dev = bias.detach().reshape(1).to(device=dev, dtype=torch.float32)
        loss = torch.empty((), dtype=torch.float32, device=dev)
        da = torch.empty(Bl, D, dtype=torch.float32, device=dev)
        db = torch.empty(Bl, D, dtype=torch.float32, device=dev)
        gt = torch.empty(1, dtype=torch.float32, device=dev)
        gb = torch.empty(1, dtype=torch.float32, device=dev)
        ws_n = L.lib().cmhar_siglip_ws(Bg, Bg)
        wsb = K.workspace(ws_n, dev)
        L.call('cmhar_siglip_loss', Bg, Bg, D, a_all.data_ptr(), b_all.data_ptr(), t_dev.data_ptr(),
               b_dev.data_ptr(), loss.data_ptr(), da.data_ptr(), off, Bl, db.data_ptr(), off, Bl, gt.data_ptr(),
               gb.data_ptr(), wsb.data_ptr(), L.stream(dev))
        ctx.save_for_backward(da, db, gt, gb)
        ctx.t_meta = (t.shape, t.device, t.dtype)
        ctx.b_meta = (bias.shape, bias.device, bias.dtype)
        return loss

    @staticmethod
    def backward(ctx, g):
        da, db, gt, gb = ctx.saved_tensors
        ga = gbv = gtt = gbb = None
        # scaling by the incoming (device) scalar gradient: a B×D elementwise product, no host sync
        if ctx.needs_input_grad[0]:
            ga = da * g
        if ctx.needs_input_grad[1]:
            gbv = db * g
        if ctx.needs_input_grad[2]:
            shape, dev, dt = ctx.t_meta
            gtt = (gt * g).reshape(shape).to(device=dev, dtype=dt)
        if ctx.needs_input_grad[3]:
            shape, dev, dt = ctx.b_meta
            gbb = (gb * g).reshape(shape).to(device=dev, dtype=dt)
        return ga, gbv, gtt, gbb, None


class SigmoidContrastiveLoss(nn.Module):
    """Reference `losses.py:9-54`."""

    def __init__(self, init_temperature=10.0, init_bias=-10.0, learnable=True, group=None):
        super().__init__()
        if learnable:
            self.temperature = nn.Parameter(torch.tensor(init_temperature).log())
            self.bias = nn.Parameter(torch.tensor(init_bias))
        else:
            self.register_buffer('temperature', torch.tensor(init_temperature).log())
            self.register_buffer('bias', torch.tensor(init_bias))
        self.group = group

    def forward(self, imu_embeds, video_embeds):
        if imu_embeds.shape != video_embeds.shape or imu_embeds.dim() != 2:
            raise ValueError('expected two (batch, dim) embedding matrices of equal shape')
        group = self.group
        if group is None:
            from . import dist as _d
            group = _d.loss_group()
        return _SigLIPFn.apply(imu_embeds, video_embeds, self.temperature, self.bias, group)
