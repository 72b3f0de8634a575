"""Data-parallel path on CPU: world_size-2 `gloo` process groups (the RCCL path on the GPU box uses the same
code with backend "nccl").

What is checked:
* `losses.gather_global` forms the global batch in rank order (the gather `nn.DataParallel` does on device 0,
  reference `main.py:89-93`);
* DataParallel semantics end to end on a small two-tower stand-in model (Linear → BatchNorm1d(train) → ReLU →
  Linear per modality, L2-normalised, oracle SigLIP loss over the GLOBAL batch, each rank back-propagating its
  local rows): after `GradReducer.finish()` every rank holds exactly the gradient of the single-process
  computation with per-replica BN — i.e. gradients are SUMMED, not averaged;
* `GradReducer` with a VideoMAE backbone: the flat gradient buffer is cut into several buckets, each bucket's
  all-reduce is launched as soon as its last parameter is produced (before `finish()`, so it overlaps the rest of
  backward), and the reduced buffer equals the sum over ranks; the non-backbone parameters are reduced too.
"""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, 'crossmodal-imu-video-ood-har_amd')


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _init(rank, world, port):
    for p in (REPO, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    torch.set_num_threads(1)
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)


def _spawn(fn, world=2):
    port = _free_port()
    mp.spawn(fn, args=(world, port), nprocs=world, join=True)


# ---------------------------------------------------------------------------------------------------------------
def _gather_worker(rank, world, port):
    _init(rank, world, port)
    from cmhar.losses import gather_global
    a = torch.full((3, 4), float(rank)) + torch.arange(12.).view(3, 4)
    b = -a
    a_all, b_all, off = gather_global(a, b, dist.group.WORLD)
    assert off == 3 * rank
    want = torch.cat([torch.full((3, 4), float(r)) + torch.arange(12.).view(3, 4) for r in range(world)])
    assert torch.equal(a_all, want) and torch.equal(b_all, -want)
    a1, b1, off1 = gather_global(a, b, None)
    assert a1 is a and b1 is b and off1 == 0
    dist.destroy_process_group()


def test_gather_global_rank_order():
    _spawn(_gather_worker)


# ---------------------------------------------------------------------------------------------------------------
class _Tower(nn.Module):
    def __init__(self, din):
        super().__init__()
        self.net = nn.Sequential(nn.Linear(din, 16), nn.BatchNorm1d(16), nn.ReLU(), nn.Linear(16, 8))

    def forward(self, x):
        return F.normalize(self.net(x), dim=1)


class _TwoTower(nn.Module):
    def __init__(self):
        super().__init__()
        self.imu = _Tower(6)
        self.video = _Tower(10)

    def forward(self, x, y):
        return self.imu(x), self.video(y)


def _data(world, bl=4):
    g = torch.Generator().manual_seed(7)
    return torch.randn(world * bl, 6, generator=g), torch.randn(world * bl, 10, generator=g)


def _dp_worker(rank, world, port):
    _init(rank, world, port)
    from cmhar.dist import GradReducer, broadcast_parameters
    from cmhar.losses import gather_global
    from oracle.cpu_model import siglip_loss
    torch.manual_seed(100 + rank)               # different init per rank: broadcast must fix it
    model = _TwoTower().train()
    broadcast_parameters(model)
    reducer = GradReducer(model, backbone=None)
    X, Y = _data(world)
    bl = X.shape[0] // world
    a, b = model(X[rank * bl:(rank + 1) * bl], Y[rank * bl:(rank + 1) * bl])
    a_all, b_all, off = gather_global(a.detach().contiguous(), b.detach().contiguous(), dist.group.WORLD)
    # this rank's rows carry the autograd graph, the others are constants (what the fused loss kernel does)
    a_all = torch.cat([a_all[:off], a, a_all[off + bl:]])
    b_all = torch.cat([b_all[:off], b, b_all[off + bl:]])
    loss = siglip_loss(a_all, b_all, torch.tensor(10.0).log(), torch.tensor(-10.0))
    reducer.start_step()
    loss.backward()
    reducer.finish()
    # single-process DataParallel equivalent: per-replica BN (each shard through the model separately), one loss
    torch.manual_seed(100)
    ref = _TwoTower().train()
    ref.load_state_dict({k: v for k, v in model.state_dict().items() if 'running' not in k and 'num_batches' not in k},
                        strict=False)
    outs = [ref(X[r * bl:(r + 1) * bl], Y[r * bl:(r + 1) * bl]) for r in range(world)]
    ra = torch.cat([o[0] for o in outs])
    rb = torch.cat([o[1] for o in outs])
    rloss = siglip_loss(ra, rb, torch.tensor(10.0).log(), torch.tensor(-10.0))
    rloss.backward()
    assert abs(loss.item() - rloss.item()) < 1e-6
    for (n, p), (_, q) in zip(model.named_parameters(), ref.named_parameters()):
        torch.testing.assert_close(p.grad, q.grad, rtol=1e-5, atol=1e-7, msg=n)
    dist.destroy_process_group()


def test_dataparallel_semantics_global_loss_summed_grads():
    _spawn(_dp_worker)


# ---------------------------------------------------------------------------------------------------------------
class _TwoTowerUnused(_TwoTower):
    """two parameters that never get a gradient (like `CrossModalModel.temperature` / `bias`) in a
    submodule registered last, so the reverse-registration guess puts them in the FIRST hook bucket."""

    def __init__(self):
        super().__init__()
        self.unused = nn.Module()
        self.unused.temperature = nn.Parameter(torch.ones([]))
        self.unused.bias = nn.Parameter(torch.ones([]))


def _hook_order_worker(rank, world, port):
    _init(rank, world, port)
    from cmhar.dist import GradReducer, broadcast_parameters
    from cmhar.losses import gather_global
    from oracle.cpu_model import siglip_loss
    torch.manual_seed(100)
    model = _TwoTowerUnused().train()
    broadcast_parameters(model)
    reducer = GradReducer(model, backbone=None, bucket_mb=60 * 4 / (1 << 20))   # ~60-element buckets
    n_hook = len(reducer.buckets)
    assert n_hook >= 3
    X, Y = _data(world)
    bl = X.shape[0] // world
    launched = []
    for step in range(3):
        model.zero_grad(set_to_none=True)
        a, b = model(X[rank * bl:(rank + 1) * bl], Y[rank * bl:(rank + 1) * bl])
        a_all, b_all, off = gather_global(a.detach().contiguous(), b.detach().contiguous(), dist.group.WORLD)
        a_all = torch.cat([a_all[:off], a, a_all[off + bl:]])
        b_all = torch.cat([b_all[:off], b, b_all[off + bl:]])
        loss = siglip_loss(a_all, b_all, torch.tensor(10.0).log(), torch.tensor(-10.0))
        reducer.start_step()
        loss.backward()
        launched.append(sum(bk.launched for bk in reducer.buckets))
        reducer.finish()
        assert model.unused.temperature.grad is None and model.unused.bias.grad is None
        # gradients = the single-process DataParallel computation (summed over replicas)
        ref = _TwoTowerUnused().train()
        ref.load_state_dict(model.state_dict())
        outs = [ref(X[r * bl:(r + 1) * bl], Y[r * bl:(r + 1) * bl]) for r in range(world)]
        rloss = siglip_loss(torch.cat([o[0] for o in outs]), torch.cat([o[1] for o in outs]),
                            torch.tensor(10.0).log(), torch.tensor(-10.0))
        rloss.backward()
        for (n, p), (_, q) in zip(model.named_parameters(), ref.named_parameters()):
            if q.grad is None:
                assert p.grad is None, n
            else:
                torch.testing.assert_close(p.grad, q.grad, rtol=1e-5, atol=1e-7, msg=n)
    assert reducer.learned
    # step 1: the unused parameters' bucket stalls every hook bucket until finish(); afterwards every bucket
    # except the trailing never-fired one is in flight when backward returns
    assert launched[0] == 0, launched
    assert launched[1] == launched[2] == len(reducer.buckets) - 1, (launched, len(reducer.buckets))
    assert [id(p) for p in reducer.buckets[-1].params] == [id(model.unused.bias), id(model.unused.temperature)]
    dist.destroy_process_group()


def test_grad_reducer_learns_hook_order_and_overlaps():
    """hook buckets must launch during backward, not all in finish()."""
    _spawn(_hook_order_worker)


# ---------------------------------------------------------------------------------------------------------------
def _bucket_worker(rank, world, port):
    _init(rank, world, port)
    from cmhar.dist import GradReducer, backbone_param_order
    from cmhar.videomae import VideoMAEBackbone, default_videomae_config
    cfg = default_videomae_config(image_size=16, patch_size=8, num_frames=4, hidden_size=64, num_hidden_layers=3,
                                  num_attention_heads=4, intermediate_size=128)
    torch.manual_seed(0)

    class Wrap(nn.Module):
        def __init__(self):
            super().__init__()
            self.backbone = VideoMAEBackbone(cfg, compute_dtype='fp32')
            self.head = nn.Linear(64, 5)

    model = Wrap()
    reducer = GradReducer(model, backbone=model.backbone, bucket_mb=0.05)
    sink = reducer.sink
    assert len(reducer.buckets) >= 3
    order = backbone_param_order(model.backbone)
    assert [id(p) for p in sink.order] == [id(p) for p in order if p.requires_grad]
    assert set(map(id, sink.order)) == set(map(id, model.backbone.parameters()))
    # simulate backward: parameters are produced in sink order, one at a time (β = 0: fresh gradients)
    reducer.start_step()
    for i, p in enumerate(sink.order):
        dst, beta = sink.dest([p], p.shape, 'cpu')
        assert beta == 0.0 and p.grad is not None
        dst.copy_(torch.full(p.shape, float(rank + 1)) * (i + 1))
        sink.done([p])
    assert all(b.launched for b in reducer.buckets if b.kind == 'sink'), 'every sink bucket must be in flight'
    model.head.weight.grad = torch.full_like(model.head.weight, float(rank + 1))
    model.head.bias.grad = torch.full_like(model.head.bias, 2.0 * (rank + 1))
    reducer.finish()
    tot = sum(r + 1 for r in range(world))
    for i, p in enumerate(sink.order):
        assert torch.equal(p.grad, torch.full(p.shape, float(tot) * (i + 1))), i
    assert torch.equal(model.head.weight.grad, torch.full_like(model.head.weight, float(tot)))
    assert torch.equal(model.head.bias.grad, torch.full_like(model.head.bias, 2.0 * tot))
    # second step reuses the same buffer: accumulation (β = 1) when .grad is kept
    reducer.start_step()
    p0 = sink.order[0]
    dst, beta = sink.dest([p0], p0.shape, 'cpu')
    assert beta == 1.0 and dst.data_ptr() == p0.grad.data_ptr()
    dist.destroy_process_group()


def test_grad_reducer_buckets_overlap_and_sum():
    _spawn(_bucket_worker)


# ---------------------------------------------------------------------------------------------------------------
def _lifecycle_worker(rank, world, port):
    """a sink backward before the first start_step(), after finish() and after close() stays local
    (no bucket launched, no AttributeError, no 'used twice' error); a parameter-set mismatch between ranks in the
    learning step raises instead of hanging the next all-reduce."""
    _init(rank, world, port)
    from cmhar.dist import GradReducer
    from cmhar.videomae import VideoMAEBackbone, default_videomae_config
    cfg = default_videomae_config(image_size=16, patch_size=8, num_frames=4, hidden_size=32, num_hidden_layers=1,
                                  num_attention_heads=2, intermediate_size=64)
    torch.manual_seed(0)

    class Wrap(nn.Module):
        def __init__(self):
            super().__init__()
            self.backbone = VideoMAEBackbone(cfg, compute_dtype='fp32')
            self.head = nn.Linear(32, 3)
            self.extra = nn.Linear(3, 3)

    model = Wrap()
    reducer = GradReducer(model, backbone=model.backbone, bucket_mb=0.01)
    sink = reducer.sink

    def sink_backward():
        for p in sink.order:
            dst, _ = sink.dest([p], p.shape, 'cpu')
            dst.fill_(1.0)
            sink.done([p])

    sink_backward()                       # before any start_step(): gradients stay local
    assert reducer.n_collectives == 0 and not any(b.launched for b in reducer.buckets)
    reducer.start_step()
    sink_backward()
    x = torch.randn(4, 32)
    out = model.head(x)
    if rank == 0:
        out = model.extra(out)            # rank 1 never produces gradients for `extra`
    out.sum().backward()
    with pytest.raises(RuntimeError, match='different parameter set'):
        reducer.finish()
    sink_backward()                       # after finish(): local, no error
    reducer.close()
    assert model.backbone._grad_sink is None and sink.on_ready is None
    sink_backward()                       # after close(): local, no error
    dist.destroy_process_group()


def test_grad_reducer_lifecycle_outside_step_window():
    _spawn(_lifecycle_worker)


# ---------------------------------------------------------------------------------------------------------------
def _partial_use_worker(rank, world, port):
    """after the learning step a rank may leave gradients None that other ranks produce (here rank 1
    skips the video tower in step 2).  Hook buckets are reduced at full size on every rank (zeros for the missing
    gradients), so the collectives still match — no hang, no mixed-up slices — and every rank ends with the
    DataParallel sum: Σ over ranks of each rank's local gradient (a missing one counting as zero)."""
    _init(rank, world, port)
    from cmhar.dist import GradReducer, broadcast_parameters
    torch.manual_seed(100)
    model = _TwoTowerUnused().train()
    broadcast_parameters(model)
    reducer = GradReducer(model, backbone=None, bucket_mb=60 * 4 / (1 << 20))
    X, Y = _data(world)
    bl = X.shape[0] // world

    def local_loss(m, r, step):
        a, b = m(X[r * bl:(r + 1) * bl], Y[r * bl:(r + 1) * bl])
        if step == 1 and r % 2 == 1:
            return (a * (r + 1)).sum()              # odd ranks: the video tower unused in this step
        return (a * (r + 1)).sum() + (b * b).sum()

    for step in range(3):
        model.zero_grad(set_to_none=True)
        start = {k: v.clone() for k, v in model.state_dict().items()}
        reducer.start_step()
        local_loss(model, rank, step).backward()
        reducer.finish()
        want = {}
        for r in range(world):           # every rank's local gradients, recomputed from the same state
            ref = _TwoTowerUnused().train()
            ref.load_state_dict(start)
            local_loss(ref, r, step).backward()
            for n, q in ref.named_parameters():
                if q.grad is not None:
                    want[n] = want[n] + q.grad if n in want else q.grad.clone()
        for n, p in model.named_parameters():
            if n not in want:
                assert p.grad is None, (step, n)
            else:
                assert p.grad is not None, (step, n)
                torch.testing.assert_close(p.grad, want[n], rtol=1e-5, atol=1e-6, msg=f'{step} {n}')
    dist.destroy_process_group()


def test_grad_reducer_partial_use_after_learning():
    _spawn(_partial_use_worker)


def _presence_worker(rank, world, port):
    """None gradients decided the same on every rank from the reduced presence counts.  Step 1 (after
    the learning step): NO rank uses the video tower — its parameters (a filled hook bucket) keep .grad None instead
    of an all-zero gradient that AdamW would decay.  Step 2: only rank 1 uses `unused.temperature` (a parameter of the
    trailing bucket, never used in the learning step) — every rank ends with rank 1's gradient, so all replicas step
    it; `unused.bias` stays None everywhere."""
    _init(rank, world, port)
    from cmhar.dist import GradReducer, broadcast_parameters
    torch.manual_seed(101)
    model = _TwoTowerUnused().train()
    broadcast_parameters(model)
    reducer = GradReducer(model, backbone=None, bucket_mb=60 * 4 / (1 << 20))
    X, Y = _data(world)
    bl = X.shape[0] // world

    def local_loss(m, r, step):
        a, b = m(X[r * bl:(r + 1) * bl], Y[r * bl:(r + 1) * bl])
        loss = (a * (r + 1)).sum()
        if step != 1:
            loss = loss + (b * b).sum()
        if step == 2 and r == 1:
            loss = loss + 3.0 * m.unused.temperature
        return loss

    for step in range(3):
        model.zero_grad(set_to_none=True)
        start = {k: v.clone() for k, v in model.state_dict().items()}
        reducer.start_step()
        local_loss(model, rank, step).backward()
        reducer.finish()
        want = {}
        for r in range(world):
            ref = _TwoTowerUnused().train()
            ref.load_state_dict(start)
            local_loss(ref, r, step).backward()
            for n, q in ref.named_parameters():
                if q.grad is not None:
                    want[n] = want[n] + q.grad if n in want else q.grad.clone()
        for n, p in model.named_parameters():
            if n not in want:
                assert p.grad is None, (step, n)
            else:
                assert p.grad is not None, (step, n)
                assert p.grad.dtype == p.dtype
                torch.testing.assert_close(p.grad, want[n], rtol=1e-5, atol=1e-6, msg=f'{step} {n}')
        if step == 1:
            assert all(p.grad is None for p in model.video.parameters())
        if step == 2:
            assert model.unused.temperature.grad is not None and model.unused.bias.grad is None
    dist.destroy_process_group()


def test_grad_reducer_presence_counts():
    _spawn(_presence_worker)


# ---------------------------------------------------------------------------------------------------------------
# 8 ranks (the reference's DataParallel over every GPU of an 8-GPU node, main.py:89-93; BASELINE config 3): the
# protocol rehearsed at the rank count the scaling bench uses, gloo on CPU
def test_dataparallel_semantics_8_ranks():
    """Global-batch SigLIP loss over 8 shards = the single-process loss on the concatenation; gradients summed."""
    _spawn(_dp_worker, world=8)


def test_grad_reducer_learned_order_8_ranks():
    """Learned hook order (rank 0's) at 8 ranks, unused parameters in the trailing bucket, hook buckets in flight
    before backward returns from the second step on."""
    _spawn(_hook_order_worker, world=8)


def _real_layout_worker(rank, world, port):
    """The production bucket layout: CrossModalModel (VideoMAE-B 16×224² + IMU encoder + heads, 88.4 M parameters)
    with the reducer the bench builds (32 MiB buckets, the backbone's flat gradient sink).  The backward is
    simulated — this is a CPU process, the backbone's kernels are HIP — by writing each sink gradient in
    production order (`sink.dest` / `sink.done`, as the backward does) and producing the hook parameters'
    gradients by autograd, with the hooks firing in a different order on odd ranks.  Checked: the layout (10 sink
    buckets + 1 hook bucket + the trailing bucket of the two never-used parameters) is identical on
    all 8 ranks, the learned hook order is rank 0's, every sink bucket is in flight as soon as its last parameter
    is written, every bucket but the trailing one is in flight before backward returns from step 2 on, and every
    gradient is the exact sum over ranks."""
    _init(rank, world, port)
    os.environ['CMHAR_ALLOW_RANDOM_INIT'] = '1'
    import warnings
    from cmhar.config import Config
    from cmhar.dist import GradReducer
    from cmhar.models import CrossModalModel
    torch.manual_seed(0)
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        model = CrossModalModel(Config())
    reducer = GradReducer(model, backbone=model.video_encoder.backbone, bucket_mb=32.0)
    sink = reducer.sink
    assert reducer.n_sink == 10, reducer.n_sink
    unused = {id(model.temperature), id(model.bias)}
    hook_params = [p for p in reducer.rest if id(p) not in unused]
    names = {id(p): n for n, p in model.named_parameters()}
    pos = {id(p): j for j, p in enumerate(hook_params)}
    tot = sum(r + 1 for r in range(world))
    for step in range(2):
        model.zero_grad(set_to_none=True)
        reducer.start_step()
        inflight = []
        for i, p in enumerate(sink.order):
            dst, _ = sink.dest([p], p.shape, 'cpu')
            dst.fill_(float((rank + 1) * (i % 7 + 1)))
            sink.done([p])
            b = reducer.buckets[reducer._bucket_of[p]]
            if p is b.params[-1]:
                inflight.append(b.launched)
        assert all(inflight) and len(inflight) == 10, inflight
        seq = hook_params if rank % 2 == 0 else list(reversed(hook_params))
        loss = sum(((rank + 1) * (pos[id(p)] % 5 + 1)) * p.sum() for p in seq)
        loss.backward()
        launched = sum(b.launched for b in reducer.buckets)
        reducer.finish()
        if step == 1:
            assert reducer.learned and launched == len(reducer.buckets) - 1, (launched, len(reducer.buckets))
            assert reducer.launched_before_finish == len(reducer.buckets) - 1
        for i, p in enumerate(sink.order):
            assert bool((p.grad == float(tot * (i % 7 + 1))).all()), names[id(p)]
        for j, p in enumerate(hook_params):
            assert bool((p.grad == float(tot * (j % 5 + 1))).all()), names[id(p)]
        assert model.temperature.grad is None and model.bias.grad is None
    layout = [[names[id(p)] for p in b.params] for b in reducer.buckets]
    hooks = layout[reducer.n_sink:]
    assert len(hooks) == 2 and sorted(hooks[-1]) == ['bias', 'temperature'], [len(h) for h in hooks]
    every = [None] * world
    dist.all_gather_object(every, layout)
    assert all(lay == every[0] for lay in every)
    dist.destroy_process_group()


def test_grad_reducer_real_layout_8_ranks():
    _spawn(_real_layout_worker, world=8)


# ---------------------------------------------------------------------------------------------------------------
# BASELINE config 4 (cross-attention fusion classifier, global batch 64 = 8 ranks x 8 clips, CE loss) at its rank count
class _FusionHead(nn.Module):
    """CrossAttentionFusion + classifier parameters under cmhar/fusion.py's state_dict names, computed by the CPU
    restatement (oracle/fusion_cpu.fusion_forward) — the HIP module cannot run in a CPU process."""

    def __init__(self, imu_dim=128, video_dim=768, d=256, classes=32):
        super().__init__()
        self.q_proj = nn.Linear(imu_dim, d)
        self.kv_proj = nn.Linear(video_dim, 2 * d)
        self.res_proj = nn.Linear(imu_dim, d)
        self.out_proj = nn.Linear(d, d)
        self.norm = nn.LayerNorm(d)
        self.classifier = nn.Linear(d, classes)

    def forward(self, imu_tokens, video_tokens):
        from oracle.fusion_cpu import fusion_forward
        return fusion_forward(dict(self.named_parameters()), imu_tokens, video_tokens, num_heads=4)[0]


def _fusion_dp_worker(rank, world, port):
    """Config 4's data parallelism (reference main.py:89-93, DataParallel over every GPU): each rank runs the fusion
    classifier on its 8 clips (26 IMU tokens x 784 video tokens each), scales its local mean CE by B_local / B_global
    (ClassificationTrainer._global_share: one SUM all-reduce of the local counts) and the GradReducer SUMs the
    gradients.  Checked against ONE process on the 64-clip concatenation (oracle/fusion_cpu as the model): the ranks'
    loss shares sum to the global-batch mean CE and every reduced gradient equals its gradient; two steps (the second
    on the learned hook order)."""
    _init(rank, world, port)
    from cmhar.dist import GradReducer, all_reduce_sum_, broadcast_parameters
    torch.manual_seed(200 + rank)               # different init per rank: broadcast must fix it
    model = _FusionHead()
    broadcast_parameters(model)
    reducer = GradReducer(model, backbone=None)
    bl, Lq, Lk = 8, 26, 784
    g = torch.Generator().manual_seed(5)
    imu = torch.randn(world * bl, Lq, 128, generator=g)
    video = 0.5 * torch.randn(world * bl, Lk, 768, generator=g)
    labels = torch.randint(0, 32, (world * bl,), generator=g)
    sl = slice(rank * bl, (rank + 1) * bl)
    for step in range(2):
        model.zero_grad(set_to_none=True)
        loss = F.cross_entropy(model(imu[sl], video[sl]), labels[sl])
        n = all_reduce_sum_(torch.full((1,), float(bl)))
        loss = loss * (bl / n)
        reducer.start_step()
        loss.backward()
        reducer.finish()
        total = all_reduce_sum_(loss.detach().clone())
        ref = _FusionHead()
        ref.load_state_dict(model.state_dict())
        rloss = F.cross_entropy(ref(imu, video), labels)
        rloss.backward()
        assert abs(total.item() - rloss.item()) <= 1e-5 * abs(rloss.item()), (step, total.item(), rloss.item())
        for (name, p), (_, q) in zip(model.named_parameters(), ref.named_parameters()):
            torch.testing.assert_close(p.grad, q.grad, rtol=1e-4, atol=1e-6, msg=f'{step} {name}')
    if step == 1:
        assert reducer.learned
    dist.destroy_process_group()


def test_fusion_classifier_dataparallel_8_ranks():
    """config 4's global-mean CE over 8 shards = the single-process loss on the 64-clip
    concatenation, summed gradients = its gradient."""
    _spawn(_fusion_dp_worker, world=8)
