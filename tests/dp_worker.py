"""One rank of the on-device data-parallel check (launched by tests/test_dist_gpu.py, never collected by pytest).

Every rank runs the real `CrossModalModel` (HIP path, `CMHAR_DP_DTYPE` fp32 parity mode or bf16, tiny geometry) on
its shard of a fixed global batch: forward → SigLIP loss over the all-gathered global batch → backward with
`GradReducer` (SUM all-reduce of gradients, bucketed) on process group backend `CMHAR_DP_BACKEND` (gloo: both ranks
share the one GPU of the test box).  A first step teaches the reducer the hook order; the second, measured step
records how many buckets were in flight when backward returned.

Rank 0 then computes the reference's `nn.DataParallel` step (main.py:89-93) on the CPU ORACLE (oracle/cpu_model.py,
pinned to the reference by g1-g9; oracle/r3d_cpu.py for the R3D-18 backbone): the same weights, each shard through
the model separately (per-replica train-mode BatchNorm, as DataParallel's replicas), one `siglip_loss` over the
concatenated embeddings, one backward — and writes the loss and every parameter gradient's error.  For bf16 it also
runs the oracle with the HIP path's bf16 storage emulated, whose distance to the fp32 oracle bounds the bf16 errors.
Rank 0 also repeats the step single-process on the HIP path (the bit-level "DP = single process" check).  Also
checked: `broadcast_buffers` leaves rank 0's BN running statistics on every rank, and only rank 0 writes checkpoints.
Results go to `$CMHAR_DP_OUT/rank{r}.json`.
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'crossmodal-imu-video-ood-har_amd'))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def build(backbone, dtype):
    from cmhar.config import Config
    from cmhar.models import CrossModalModel
    cfg = Config()
    cfg.data.imu_window_size = 64
    cfg.data.video_frames_per_window = 4
    cfg.data.video_resize = (32, 32)
    m = cfg.model
    m.video_pretrained = False
    m.compute_dtype = dtype
    m.imu_d_model, m.imu_nhead, m.imu_num_layers, m.imu_dropout = 32, 4, 2, 0.0
    m.video_d_model, m.projection_hidden_dim, m.projection_dim = 64, 64, 32
    if backbone == 'videomae':
        m.video_backbone = '/nonexistent/videomae-dp'
        m.videomae_hidden_size, m.videomae_num_layers, m.videomae_num_heads = 128, 2, 2
        m.videomae_intermediate_size, m.videomae_patch_size = 256, 16
    else:
        m.video_backbone = backbone           # 'r3d_18', or the per-frame 'resnet18' / 'mobilenet_v2'
    torch.manual_seed(0)
    return CrossModalModel(cfg)


def classify(D, rank, world, dev, out_dir):
    """ClassificationTrainer.train_step under data parallelism: the summed gradients must be those of the
    global-batch mean CE (DataParallel gathers the logits and takes one mean), not world_size times it."""
    from cmhar.models import IMUClassifier
    from cmhar.optim import clip_grad_norm_
    from cmhar.trainer import ClassificationTrainer
    from cmhar.losses import CrossEntropyLoss
    model0 = build('videomae', 'fp32')
    cfg = model0.config
    cfg.training.train_lr_head = 1e-3
    cfg.model.classifier_dropout = 0.0     # per-call dropout masks would differ between the two runs
    bl = 4
    g = torch.Generator().manual_seed(5)
    imu_all = torch.randn(world * bl, 6, 64, generator=g)
    lab_all = torch.randint(0, cfg.model.num_classes, (world * bl,), generator=g)

    def make():
        torch.manual_seed(3)
        return IMUClassifier(build('videomae', 'fp32').imu_encoder, cfg)
    clf = make()
    init_sd = {k: v.clone() for k, v in clf.state_dict().items()}
    clf = clf.to(dev)
    reducer = D.GradReducer(clf, backbone=None, bucket_mb=0.05)
    tr = ClassificationTrainer(clf, cfg, device=dev, mode='finetune', grad_reducer=reducer)
    sl = slice(rank * bl, (rank + 1) * bl)
    clf.train()
    _, share = tr.train_step(imu_all[sl].to(dev), lab_all[sl].to(dev))
    torch.cuda.synchronize()
    tot = share.detach().clone().reshape(1)
    D.all_reduce_sum_(tot)
    res = {'rank': rank, 'loss': float(tot.item())}
    grads = {n: p.grad.detach().cpu() for n, p in clf.named_parameters() if p.grad is not None}
    if rank == 0:
        ref = make()
        ref.load_state_dict(init_sd)
        ref = ref.to(dev).train()
        logits = torch.cat([ref(imu_all[r * bl:(r + 1) * bl].to(dev)) for r in range(world)])
        rloss = CrossEntropyLoss()(logits, lab_all.to(dev))
        rloss.backward()
        clip_grad_norm_(list(ref.parameters()), 1.0)
        torch.cuda.synchronize()
        res['ref_loss'] = float(rloss.item())
        errs = {}
        for n, p in ref.named_parameters():
            if p.grad is None or n not in grads:
                continue
            rg = p.grad.detach().cpu()
            errs[n] = (float((grads[n] - rg).norm()) / max(float(rg.norm()), 1e-30), float(rg.norm()))
        res['grad_errs'] = errs
        res['missing'] = sorted(set(grads) ^ {n for n, p in ref.named_parameters() if p.grad is not None})
    # validate() with uneven shards: rank 0 holds two batches, rank 1 one; no per-batch collective,
    # and the loss is the mean over GLOBAL batches (batch 0 = both ranks' first shards, batch 1 = rank 0's second)
    D.broadcast_buffers(clf)
    gv = torch.Generator().manual_seed(9)
    shards = [[(torch.randn(3, 6, 64, generator=gv), torch.randint(0, cfg.model.num_classes, (3,), generator=gv))
               for _ in range(2)],
              [(torch.randn(3, 6, 64, generator=gv), torch.randint(0, cfg.model.num_classes, (3,), generator=gv))]]
    mine = shards[rank] if rank < 2 else []
    vm = tr.validate([{'imu': x, 'label': y} for x, y in mine])
    res['val_loss'] = vm['loss']
    if rank == 0:
        clf.eval()
        with torch.no_grad():
            glob = [[shards[0][0], shards[1][0]], [shards[0][1]]]
            ces = []
            for parts in glob:
                lg = torch.cat([clf(x.to(dev)) for x, _ in parts])
                ces.append(float(CrossEntropyLoss()(lg, torch.cat([y for _, y in parts]).to(dev)).item()))
        res['ref_val_loss'] = sum(ces) / len(ces)
    with open(os.path.join(out_dir, f'rank{rank}.json'), 'w') as f:
        json.dump(res, f)
    flat = torch.cat([grads[n].reshape(-1) for n in sorted(grads)])
    objs = [None] * world
    dist.all_gather_object(objs, float(flat.double().sum()))
    with open(os.path.join(out_dir, f'rank{rank}.sum'), 'w') as f:
        json.dump(objs, f)
    dist.destroy_process_group()


def oracle_step(backbone, init_sd, cfg, imu_all, video_all, world, bl, bf16):
    """The reference's DataParallel step on the CPU oracle: per-shard forward with train-mode BN, SigLIP over the
    gathered global batch, one backward.  Returns (loss, {param name: grad})."""
    import numpy as np
    import torch.nn.functional as F
    for d in (REPO, os.path.join(REPO, 'tests'), os.path.join(REPO, 'tests', 'golden')):
        sys.path.insert(0, d)
    from fixtures import oracle_mcfg
    from oracle import cpu_model as O
    from oracle.r3d_cpu import BF16, r3d18_features
    sd = {k: (v.clone().requires_grad_(True) if v.is_floating_point() and 'running' not in k else v.clone())
          for k, v in init_sd.items()}
    mc = oracle_mcfg(cfg)
    outs = []
    for r in range(world):
        imu, video = imu_all[r * bl:(r + 1) * bl], video_all[r * bl:(r + 1) * bl]
        if backbone == 'videomae':
            outs.append(O.crossmodal(sd, imu, video, mc, training=True, bf16=bf16))
            continue
        pre = 'video_encoder.backbone.'
        bsd = {k[len(pre):]: v for k, v in sd.items() if k.startswith(pre)}
        cls, _ = O.imu_encoder(sd, imu, patch_size=mc['imu_patch_size'], stride=mc['imu_stride'],
                               nhead=mc['imu_nhead'], num_layers=mc['imu_num_layers'])
        feat = r3d18_features(bsd, video.transpose(1, 2), training=True, **(BF16 if bf16 else {}))
        vf = F.linear(feat, sd['video_encoder.projection.weight'], sd['video_encoder.projection.bias'])
        outs.append((O.l2_normalize(O.projection_head(sd, cls, 'imu_proj.', True)),
                     O.l2_normalize(O.projection_head(sd, vf, 'video_proj.', True))))
    loss = O.siglip_loss(torch.cat([o[0] for o in outs]), torch.cat([o[1] for o in outs]),
                         torch.tensor(float(np.log(10.0))), torch.tensor(-10.0))
    loss.backward()
    return float(loss.item()), {k: v.grad for k, v in sd.items() if v.is_floating_point() and v.grad is not None}


def _errs(grads, ref):
    return {n: (float((grads[n] - g).norm()) / max(float(g.norm()), 1e-30), float(g.norm()), float(g.abs().max()))
            for n, g in ref.items() if n in grads}


def main():
    from cmhar import dist as D
    from cmhar.losses import SigmoidContrastiveLoss
    from cmhar.trainer import BaseTrainer
    backbone = os.environ.get('CMHAR_DP_BACKBONE', 'videomae')
    dtype = os.environ.get('CMHAR_DP_DTYPE', 'fp32')
    out_dir = os.environ['CMHAR_DP_OUT']
    rank, world, _ = D.init_from_env(os.environ.get('CMHAR_DP_BACKEND', 'gloo'))
    torch.cuda.set_device(0)
    force = os.environ.get('CMHAR_DP_FORCE_REDUCE') == '1'
    if world == 1 and not dist.is_initialized():
        # one rank over RCCL: the reducer runs its full protocol (GradReducer(reduce_single=True))
        dist.init_process_group(os.environ.get('CMHAR_DP_BACKEND', 'gloo'), rank=0, world_size=1)
    dev = torch.device('cuda', 0)
    if backbone == 'classify':
        return classify(D, rank, world, dev, out_dir)
    bl = 4
    g = torch.Generator().manual_seed(11)
    imu_all = torch.randn(world * bl, 6, 64, generator=g)
    video_all = torch.randn(world * bl, 4, 3, 32, 32, generator=g)

    model = build(backbone, dtype)
    init_sd = {k: v.clone() for k, v in model.state_dict().items()}
    model = model.to(dev).train()
    if rank != 0:                        # a different start on rank 1: broadcast_parameters must fix it
        with torch.no_grad():
            for p in model.parameters():
                p.add_(0.5)
    D.broadcast_parameters(model)
    reducer = D.GradReducer(model, backbone=model.video_encoder.backbone,
                            bucket_mb=0.25 if backbone == 'videomae' else 8.0, reduce_single=force)
    loss_fn = SigmoidContrastiveLoss().to(dev)
    sl = slice(rank * bl, (rank + 1) * bl)
    for step in range(2):                # step 0 teaches the reducer the hook order; step 1 is the one checked
        model.zero_grad(set_to_none=True)
        a, b = model(imu_all[sl].to(dev), video_all[sl].to(dev))
        loss = loss_fn(a, b)
        reducer.start_step()
        loss.backward()
        reducer.finish()
    torch.cuda.synchronize()
    grads = {n: p.grad.detach().cpu() for n, p in model.named_parameters() if p.grad is not None}
    res = {'rank': rank, 'loss': float(loss.item()), 'n_buckets': len(reducer.buckets),
           'backend': dist.get_backend(), 'n_collectives': reducer.n_collectives,
           'sink': reducer.sink is not None, 'n_grads': len(grads), 'learned': reducer.learned,
           'launched_before_finish': reducer.launched_before_finish,
           'trailing_unused': [n for n, p in model.named_parameters()
                               if any(p is q for q in reducer.buckets[-1].params)]}

    # BN running statistics: rank 0's everywhere after broadcast_buffers
    bn_key = 'video_proj.net.1.running_mean'
    before = model.state_dict()[bn_key].detach().cpu().clone()
    D.broadcast_buffers(model)
    after = model.state_dict()[bn_key].detach().cpu()
    obj = [None] * world
    dist.all_gather_object(obj, before.tolist())
    res['bn_broadcast_ok'] = bool(torch.equal(after, torch.tensor(obj[0])))
    res['bn_differed_before'] = obj[0] != obj[-1]

    # single writer
    tr = BaseTrainer.__new__(BaseTrainer)
    tr.model, tr.current_epoch, tr.history = model, 0, {'train': [], 'val': []}
    ck = os.path.join(out_dir, f'ckpt_written_by_{rank}.pt')
    BaseTrainer.save_checkpoint(tr, os.path.join(out_dir, 'ckpt.pt') if rank == 0 else ck)
    res['wrote_checkpoint'] = os.path.exists(ck) or (rank == 0 and os.path.exists(os.path.join(out_dir, 'ckpt.pt')))

    if rank == 0:
        # (1) the reference's DataParallel step on the CPU oracle (fp32), and its bf16-storage emulation (VideoMAE
        # and R3D-18; the per-frame CNN backbones' gradients are pinned to their oracle by tests/test_cnn2d_gpu.py)
        cfg = model.config
        if backbone in ('videomae', 'r3d_18'):
            res['oracle_loss'], og = oracle_step(backbone, init_sd, cfg, imu_all, video_all, world, bl, False)
            res['missing_oracle'] = sorted(set(og) ^ set(grads))
            res['oracle_errs'] = _errs(grads, og)
            if dtype == 'bf16':
                res['emul_loss'], eg = oracle_step(backbone, init_sd, cfg, imu_all, video_all, world, bl, True)
                res['emul_errs'] = _errs(eg, og)
        # (2) single-process DataParallel equivalent on the same device and kernels
        ref = build(backbone, dtype)
        ref.load_state_dict(init_sd)
        ref = ref.to(dev).train()
        lf = SigmoidContrastiveLoss(group=False).to(dev)
        outs = [ref(imu_all[r * bl:(r + 1) * bl].to(dev), video_all[r * bl:(r + 1) * bl].to(dev))
                for r in range(world)]
        rloss = lf(torch.cat([o[0] for o in outs]), torch.cat([o[1] for o in outs]))
        rloss.backward()
        torch.cuda.synchronize()
        rgrads = {n: p.grad.detach().cpu() for n, p in ref.named_parameters() if p.grad is not None}
        res['ref_loss'] = float(rloss.item())
        res['missing'] = sorted(set(rgrads) ^ set(grads))
        res['grad_errs'] = {n: e[:2] for n, e in _errs(grads, rgrads).items()}
    with open(os.path.join(out_dir, f'rank{rank}.json'), 'w') as f:
        json.dump(res, f)
    # every rank must hold the same reduced gradients
    flat = torch.cat([grads[n].reshape(-1) for n in sorted(grads)])
    objs = [None] * world
    dist.all_gather_object(objs, float(flat.double().sum()))
    with open(os.path.join(out_dir, f'rank{rank}.sum'), 'w') as f:
        json.dump(objs, f)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
