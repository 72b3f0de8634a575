"""Throughput benchmark of the cross-modal pretraining step (BASELINE.json metric):
clips/sec of forward + backward + clip_grad_norm_(1.0) + AdamW over 16×224² video + 200×6 IMU clips,
batch 32 per GPU, VideoMAE-B video backbone (the reference default), bf16 MFMA compute.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 --master-port P \
        bench.py --gpus N --steps K --warmup W

One step = the body of CrossModalTrainer.train_epoch (src/train/trainer.py:130-144) on synthetic inputs already
resident in HBM: model(imu, video) → SigmoidContrastiveLoss → zero_grad → backward (+ RCCL gradient all-reduce
when N > 1) → clip_grad_norm_(1.0) → AdamW.step.  Weak scaling: every rank processes its own 32 clips; the loss
is over the gathered global batch (DataParallel semantics).  Rank 0 prints one JSON line.
"""
import argparse
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, 'crossmodal-imu-video-ood-har_amd'))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0      # MI355X dense bf16 MFMA (MI355X_MICROARCH.md; sparsity excluded)
PEAK_HBM_GBS = 8000.0


TRAFFIC_JSON = os.path.join(REPO, 'profiles', 'r01_pmc_traffic.json')


def pmc_traffic(label):
    """HBM bytes per launch of the traced kernel `label` (e.g. 'gemm256_kernel<true,false,bf16>') from the committed
    PMC summary of this same bench command (tools/pmc_traffic.py), or None when it has no entry."""
    if not os.path.exists(TRAFFIC_JSON) or '<' not in label:
        return None
    base, args = label.split('<', 1)
    code = {'true': 'Lb1E', 'false': 'Lb0E', 'bf16': 'DF16b', 'float': 'f'}
    mangled = base + 'I' + ''.join(code[a.strip()] for a in args.rstrip('>').split(','))
    with open(TRAFFIC_JSON) as f:
        ks = json.load(f)['kernels']
    demangled = base + '<' + ', '.join(a.strip() for a in args.rstrip('>').split(','))   # rocprof demangles some
    hits = [v for k, v in ks.items() if mangled in k or demangled in k]
    if not hits:
        return None
    n = sum(v['dispatches'] for v in hits)
    return int(sum(v['hbm_bytes_per_launch'] * v['dispatches'] for v in hits) / n)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=50)     # >= 50 timed steps after >= 10 warm-up
    ap.add_argument('--warmup', type=int, default=10)
    ap.add_argument('--batch', type=int, default=32)
    ap.add_argument('--frames', type=int, default=16)
    ap.add_argument('--image', type=int, default=224)
    ap.add_argument('--imu-len', type=int, default=200)
    ap.add_argument('--dtype', default='bf16', choices=['bf16', 'fp32'])
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-batch', type=int, default=2)
    ap.add_argument('--cpu-steps', type=int, default=2)
    ap.add_argument('--no-trace', action='store_true')
    ap.add_argument('--imu-stream', choices=['side', 'main'], default='side',
                    help='run the IMU branch on its own HIP stream (overlapping the video branch) or on the main one')
    return ap.parse_args()


def videomae_flops_per_clip(T, H, W, hd=768, layers=12, inter=3072, P=16, tub=2, C=3):
    """Algorithmic forward FLOPs of VideoMAE-B per clip."""
    N = (T // tub) * (H // P) * (W // P)
    embed = 2 * N * (C * tub * P * P) * hd
    per_layer = 2 * N * hd * (4 * hd + 2 * inter) + 4 * N * N * hd
    return embed, embed + layers * per_layer


def cpu_baseline(cfg_builder, batch, steps, frames, image, imu_len):
    """The CPU oracle (torch-eager fp32 restatement of the reference path) timed on the host cores."""
    sys.path.insert(0, REPO)
    from oracle import cpu_model as O
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    cfg = cfg_builder()
    from cmhar.models import CrossModalModel
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        model = CrossModalModel(cfg)
    sd = {k: (v.detach().clone().requires_grad_(True) if v.is_floating_point() else v.clone())
          for k, v in model.state_dict().items()}
    del model
    mc = dict(imu_patch_size=16, imu_stride=16, imu_nhead=8, imu_num_layers=4, video_num_heads=12)
    g = torch.Generator().manual_seed(0)
    imu = torch.randn(batch, 6, imu_len, generator=g)
    video = torch.randn(batch, frames, 3, image, image, generator=g)
    lt, lb = torch.tensor(math.log(10.0)), torch.tensor(-10.0)
    names = [k for k, v in sd.items() if v.is_floating_point() and 'running' not in k]
    m = [torch.zeros_like(sd[k]) for k in names]
    v = [torch.zeros_like(sd[k]) for k in names]

    def step(i):
        for k in names:
            sd[k].grad = None
        a, b = O.crossmodal(sd, imu, video, mc, training=True, imu_dropout=0.1, gen=g)
        loss = O.siglip_loss(a, b, lt, lb)
        loss.backward()
        with torch.no_grad():
            grads = [sd[k].grad for k in names]
            O.clip_grad_norm(grads, 1.0)
            O.adamw_step([sd[k] for k in names], grads, m, v, i, lr=1e-5)

    step(1)
    t0 = time.perf_counter()
    for i in range(steps):
        step(i + 2)
    dt = time.perf_counter() - t0
    return {'value': round(batch * steps / dt, 4), 'unit': 'clips/sec', 'cores': threads, 'kind': 'port',
            'sample': f'oracle/cpu_model.py fp32 fwd+bwd+clip+AdamW, batch {batch}, {steps} timed steps after '
                      f'1 warm-up, {frames}x{image}^2 video + 6x{imu_len} IMU, {threads} threads'}


def main():
    args = parse()
    from cmhar import dist as cdist
    from cmhar import kernels as K
    from cmhar.config import Config
    from cmhar.losses import SigmoidContrastiveLoss
    from cmhar.models import CrossModalModel
    from cmhar.optim import FusedAdamW, clip_grad_norm_

    # CMHAR_BENCH_BACKEND / CMHAR_BENCH_DEVICE: rehearsal knobs only (e.g. two gloo ranks sharing the one GPU of a
    # test box); the measured configuration is one RCCL rank per GPU
    rank, world, local = cdist.init_from_env(os.environ.get('CMHAR_BENCH_BACKEND') or None)
    local = int(os.environ.get('CMHAR_BENCH_DEVICE', local))
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)

    def make_cfg():
        cfg = Config()
        cfg.model.allow_random_init = True   # synthetic benchmark: random-init weights
        cfg.data.imu_window_size = args.imu_len
        cfg.data.video_frames_per_window = args.frames
        cfg.data.video_resize = (args.image, args.image)
        cfg.model.compute_dtype = args.dtype
        return cfg

    import warnings
    torch.manual_seed(0)
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')          # hub checkpoint not fetchable offline → random init
        model = CrossModalModel(make_cfg())
    model = model.to(dev).train()
    model.overlap_imu = args.imu_stream == 'side'
    backbone = model.video_encoder.backbone
    cdist.broadcast_parameters(model)
    reducer = cdist.GradReducer(model, backbone=backbone)
    loss_fn = SigmoidContrastiveLoss().to(dev)
    # LinearLR(start_factor=0.1) of trainer.py:80-105 → step-0 lr = 0.1 * pretrain_lr
    opt = FusedAdamW(model.parameters(), lr=0.1 * 1e-4, weight_decay=0.01, shadow_sources=[backbone])

    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    B = args.batch
    video = torch.randn(B, args.frames, 3, args.image, args.image, device=dev, generator=g)
    imu = torch.randn(B, 6, args.imu_len, device=dev, generator=g)
    params = list(model.parameters())

    def step():
        a, b = model(imu, video)
        loss = loss_fn(a, b)
        opt.zero_grad(set_to_none=True)
        reducer.start_step()
        loss.backward()
        reducer.finish()
        clip_grad_norm_(params, 1.0)
        opt.step()
        return loss

    # Warm-up; its last step runs with every GEMM / attention launch bracketed by HIP events, which gives the
    # per-kernel-family breakdown and picks the dominant single kernel.  The timed loop then brackets ONLY that
    # kernel's launches (the events of all ~180 traced launches cost ~1.5 ms/step of stream bubbles).
    breakdown = {}
    for i in range(args.warmup):
        full = not args.no_trace and i == args.warmup - 1
        if full:
            K.TRACE.records, K.TRACE.only, K.TRACE.active = [], None, True
        loss = step()
        if full:
            torch.cuda.synchronize()
            K.TRACE.active = False
            breakdown = K.TRACE.summary()
    torch.cuda.synchronize()
    first_loss = float(loss.item()) if args.warmup else float('nan')
    single = {k: v for k, v in breakdown.items() if '+' not in k and '(' not in k}
    dominant = max(single.items(), key=lambda kv: kv[1][1])[0] if single else None
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    K.TRACE.records = []
    K.TRACE.only = {dominant} if dominant else None
    K.TRACE.active = not args.no_trace and dominant is not None
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    K.TRACE.active = False
    if world > 1:
        dist.barrier()
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    clips = world * B * args.steps
    value = clips / elapsed
    ms = 1000 * elapsed / args.steps

    # dominant kernel: the single HIP kernel (not a multi-kernel entry such as attention backward or split-K +
    # reduce) with the largest traced time in the traced warm-up step; achieved = its algorithmic FLOPs / its
    # HIP-event-measured time over the timed region
    roof = None
    summ = K.TRACE.summary() if not args.no_trace else {}
    if dominant in summ:
        name = dominant
        n, tot_ms, fl, nb = summ[name]
        achieved = fl / (tot_ms / 1e3) / 1e12
        roof = {'bound': 'mfma', 'achieved': round(achieved, 1), 'peak': PEAK_BF16_TFLOPS, 'unit': 'TFLOP/s',
                'frac': round(achieved / PEAK_BF16_TFLOPS, 4), 'traffic': pmc_traffic(name), 'kernel': name,
                'launches': n, 'avg_launch_ms': round(tot_ms / n, 4),
                'algorithmic_bytes_per_launch': int(nb / n)}
    embed_f, fwd_f = videomae_flops_per_clip(args.frames, args.image, args.image)
    step_flops_clip = 3 * fwd_f - embed_f           # fwd + 2x bwd, no pixel gradient for the tubelet conv
    whole_tflops = step_flops_clip * clips / elapsed / 1e12

    out = {'metric': 'clips/sec fwd+bwd, 16x224^2 video + 200x6 IMU, batch 32, 1/2/4/8 GPU', 'value': round(value, 3),
           'unit': 'clips/sec', 'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
           'ms_per_step': round(ms, 3), 'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
           'dtype': args.dtype, 'data': 'synthetic (randn video/IMU resident in HBM, random-init VideoMAE-B weights)',
           'config': {'workload': f'CrossModalModel pretrain step: VideoMAE-B {args.frames}x{args.image}^2 + '
                                  f'IMU 6x{args.imu_len} PatchTST, SigLIP loss, clip 1.0, AdamW',
                      'global_batch': world * B, 'per_gpu_batch': B, 'parallelism': f'dp{world}'},
           'roofline': roof,
           'whole_step_model_tflops': round(whole_tflops, 1),
           'whole_step_mfma_frac': round(whole_tflops / PEAK_BF16_TFLOPS, 4),
           'first_warmup_loss': first_loss,
           'max_mem_gb': round(torch.cuda.max_memory_allocated(dev) / 2 ** 30, 1)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out['cpu_baseline'] = cpu_baseline(make_cfg, args.cpu_batch, args.cpu_steps, args.frames, args.image,
                                           args.imu_len)
    if rank == 0:
        if breakdown:   # one traced warm-up step
            out['kernels'] = {k: {'launches': n, 'ms_per_step': round(tm, 3),
                                  'tflops': round(f / (tm / 1e3) / 1e12, 1)} for k, (n, tm, f, b) in breakdown.items()}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
