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
    """Reference `losses.py:9-54`.  `group`: process group of the global batch (None: `cmhar.dist`'s default, False:
    this process's batch only)."""

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
        if group is False:                 # explicitly local: this process's batch only
            group = None
        elif group is None:
            from . import dist as _d
            group = _d.loss_group()
        return _SigLIPFn.apply(imu_embeds, video_embeds, self.temperature, self.bias, group)


# ------------------------------------------------------------------------------------------------------------------
# Cross-entropy family (reference src/models/losses.py:57-167 and the nn.CrossEntropyLoss of ClassificationTrainer,
# src/train/trainer.py:249) on the fused row-softmax kernel `cmhar_cross_entropy`: forward = loss (+ argmax) in two
# launches; backward = one more pass writing dlogits scaled by the incoming (device) gradient — no host sync.
# ------------------------------------------------------------------------------------------------------------------
def _labels_on(labels, device, C, ignore_index):
    if labels.dtype not in (torch.int64, torch.int32, torch.int16, torch.uint8):
        raise TypeError(f'expected integer class labels, got {labels.dtype}')
    if not labels.is_cuda:                       # host labels (the DataLoader case): validate without a device sync
        bad = (labels != ignore_index) & ((labels < 0) | (labels >= C))
        if bool(bad.any()):
            raise IndexError(f'Target {int(labels[bad][0])} is out of bounds.')
    return labels.to(device=device, dtype=torch.int64, non_blocking=True).contiguous()


class _CrossEntropyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, ignore_index, eps, gamma, alpha, reduction):
        z = logits.float() if logits.dtype != torch.float32 else logits
        N = z.shape[0]
        out = torch.empty((N,) if reduction == 'none' else (), dtype=torch.float32, device=z.device)
        K.cross_entropy(z, labels, ignore_index=ignore_index, label_smoothing=eps, gamma=gamma, alpha=alpha,
                        reduction=reduction, loss=None if reduction == 'none' else out,
                        row_loss=out if reduction == 'none' else None)
        ctx.save_for_backward(z, labels)
        ctx.args = (ignore_index, eps, gamma, alpha, reduction, logits.dtype)
        return out

    @staticmethod
    def backward(ctx, g):
        z, labels = ctx.saved_tensors
        ignore_index, eps, gamma, alpha, reduction, dt = ctx.args
        dz = torch.empty_like(z)
        K.cross_entropy(z, labels, ignore_index=ignore_index, label_smoothing=eps, gamma=gamma, alpha=alpha,
                        reduction=reduction, dlogits=dz, g_up=g.contiguous().float())
        return dz.to(dt), None, None, None, None, None, None


def cross_entropy(logits, target, ignore_index=-100, reduction='mean', label_smoothing=0.0, *, gamma=0.0,
                  alpha=1.0):
    """F.cross_entropy for (N, C) logits and class-index targets (+ the focal weighting of FocalLoss)."""
    if logits.dim() != 2:
        raise ValueError(f'expected (N, C) logits, got {tuple(logits.shape)}')
    if reduction not in ('none', 'mean', 'sum'):
        raise ValueError(f'{reduction} is not a valid value for reduction')
    labels = _labels_on(target, logits.device, logits.shape[1], ignore_index)
    return _CrossEntropyFn.apply(logits, labels, int(ignore_index), float(label_smoothing), float(gamma),
                                 float(alpha), reduction)


class CrossEntropyLoss(nn.Module):
    """nn.CrossEntropyLoss (class-index targets, no class weights) — ClassificationTrainer's loss (trainer.py:249)."""

    def __init__(self, weight=None, ignore_index=-100, reduction='mean', label_smoothing=0.0):
        super().__init__()
        if weight is not None:
            raise NotImplementedError('class weights are not used by the reference')
        self.ignore_index = ignore_index
        self.reduction = reduction
        self.label_smoothing = label_smoothing

    def forward(self, inputs, targets):
        return cross_entropy(inputs, targets, self.ignore_index, self.reduction, self.label_smoothing)


class FocalLoss(nn.Module):
    """Reference losses.py:90-116: alpha·(1-pt)^gamma·CE, reduction mean / sum / none."""

    def __init__(self, alpha=1.0, gamma=2.0, reduction='mean'):
        super().__init__()
        self.alpha = alpha
        self.gamma = gamma
        self.reduction = reduction

    def forward(self, inputs, targets):
        return cross_entropy(inputs, targets, reduction=self.reduction, gamma=self.gamma, alpha=self.alpha)


class LabelSmoothingCrossEntropy(nn.Module):
    """Reference losses.py:119-150: targets (1-eps)·onehot + eps/C against log_softmax."""

    def __init__(self, epsilon=0.1, reduction='mean'):
        super().__init__()
        self.epsilon = epsilon
        self.reduction = reduction

    def forward(self, inputs, targets):
        return cross_entropy(inputs, targets, reduction=self.reduction, label_smoothing=self.epsilon)


class _InfoNCEFn(torch.autograd.Function):
    """S = a·bᵀ/τ (fp32 GEMM), loss = (CE(S, arange) + CE(Sᵀ, arange))/2; the transposed CE reads S through a
    (1, B) stride view and accumulates its gradient into the same dS buffer."""

    @staticmethod
    def forward(ctx, a, b, inv_t):
        a = a.contiguous().float()
        b = b.contiguous().float()
        B = a.shape[0]
        S = torch.empty(B, B, dtype=torch.float32, device=a.device)
        K.gemm(0, a, b, S, alpha=inv_t)
        l1 = torch.empty((), dtype=torch.float32, device=a.device)
        l2 = torch.empty((), dtype=torch.float32, device=a.device)
        K.cross_entropy(S, None, loss=l1)
        K.cross_entropy(S.t(), None, loss=l2)
        ctx.save_for_backward(a, b, S)
        ctx.inv_t = inv_t
        loss = torch.empty((), dtype=torch.float32, device=a.device)
        K.copy2d(l1.view(1, 1), loss.view(1, 1), alpha=0.5)
        K.copy2d(l2.view(1, 1), loss.view(1, 1), alpha=0.5, beta=1.0)
        return loss

    @staticmethod
    def backward(ctx, g):
        a, b, S = ctx.saved_tensors
        g = g.reshape(1).contiguous().float()
        dS = torch.empty_like(S)
        K.cross_entropy(S, None, dlogits=dS, grad_scale=0.5, g_up=g)
        K.cross_entropy(S.t(), None, dlogits=dS.t(), grad_scale=0.5, grad_beta=1.0, g_up=g)
        da = db = None
        if ctx.needs_input_grad[0]:
            da = torch.empty_like(a)
            K.gemm(1, dS, b, da, alpha=ctx.inv_t)
        if ctx.needs_input_grad[1]:
            db = torch.empty_like(b)
            K.gemm(2, dS, a, db, alpha=ctx.inv_t)
        return da, db, None


class InfoNCELoss(nn.Module):
    """Reference losses.py:57-87 (symmetric NT-Xent over the batch similarity matrix)."""

    def __init__(self, temperature=0.07):
        super().__init__()
        self.temperature = temperature

    def forward(self, imu_embeds, video_embeds):
        if imu_embeds.shape != video_embeds.shape or imu_embeds.dim() != 2:
            raise ValueError('expected two (batch, dim) embedding matrices of equal shape')
        return _InfoNCEFn.apply(imu_embeds, video_embeds, 1.0 / self.temperature)


def get_loss_function(loss_name, **kwargs):
    """Reference losses.py:153-167."""
    if loss_name == 'sigmoid_contrastive':
        return SigmoidContrastiveLoss(**kwargs)
    if loss_name == 'infonce':
        return InfoNCELoss(**kwargs)
    if loss_name == 'cross_entropy':
        return CrossEntropyLoss(**kwargs)
    if loss_name == 'focal':
        return FocalLoss(**kwargs)
    if loss_name == 'label_smoothing':
        return LabelSmoothingCrossEntropy(**kwargs)
    raise ValueError(f'Loss function inconnue: {loss_name}')
