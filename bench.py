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

`--workload` selects the other BASELINE configs with the same JSON schema (so a driver rerun can confirm them):
  videomae  (default) the headline: VideoMAE-B 16×224² + IMU 6×200, batch 32 per GPU, bf16 (configs 2/3 geometry at
            `--image 112`);
  r3d       config 2 with its named backbone: the R3D-18 extension, 16×112² + IMU 6×200, batch 32 per GPU, bf16;
  fusion    config 4 per GPU: CrossModalFusionClassifier (IMU 400 tokens × VideoMAE-B 32×224² tokens), batch 8
            per GPU (global 64 on 8 GPUs), CE loss, bf16;
  ood_fp16  config 5: the OOD evaluation stream, fp16 inference: forward → SigLIP logits → energy score, one step =
            one batch of 32 clips from a ring of 8 distinct resident batches; default 313 steps = 10 016 clips.
  imu       config 1 on the HIP path (the reference runs it on the CPU): IMU-only classifier (IMUEncoder + the
            256-128 MLP head, models.py:296-348) fine-tune step of ClassificationTrainer (CE, clip 1.0, AdamW over
            encoder + head), 6x200 windows, batch 8; `clips/sec` = windows/s.  Its CPU counterpart is the headline
            line's `cpu_baseline.imu_only_b8_train_windows_per_sec`.
For the non-headline workloads `roofline` is the whole step's algorithmic FLOP rate against the bf16 / fp16 peak
(`kernel`: "whole step"); the headline's is the dominant single kernel's (HIP events) with PMC traffic.
"""
import argparse
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, 'crossmodal-imu-video-ood-har_amd'))

# kernel arguments in device memory (see cmhar/__init__.py; set before the HIP runtime initialises)
os.environ.setdefault('HIP_FORCE_DEV_KERNARG', '1')
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0      # MI355X dense bf16 MFMA (MI355X_MICROARCH.md; sparsity excluded)
PEAK_F32_TFLOPS = 157.3        # f32-input MFMA (= the f32 vector rate; no xf32 on gfx950)
PEAK_HBM_GBS = 8000.0


TRAFFIC_JSON = os.path.join(REPO, 'profiles', 'r06_pmc_traffic.json')
MFMA_JSON = os.path.join(REPO, 'profiles', 'r06_pmc_mfma.json')

# per-workload defaults of --batch / --frames / --image / --imu-len / --dtype (BASELINE.json configs)
WORKLOADS = {
    'videomae': dict(batch=32, frames=16, image=224, imu_len=200, dtype='bf16'),
    'r3d': dict(batch=32, frames=16, image=112, imu_len=200, dtype='bf16'),
    'fusion': dict(batch=8, frames=32, image=224, imu_len=400, dtype='bf16'),
    'ood_fp16': dict(batch=32, frames=16, image=224, imu_len=200, dtype='fp16'),
    'imu': dict(batch=8, frames=16, image=224, imu_len=200, dtype='fp32'),
}


# rocprofv3 prints some instantiations half-demangled — the bf16 type as "bool _Accum", later template arguments
# as "E" — so their PMC records carry no mangled codes to match.  The prefetching-epilogue (PFS = true)
# instantiations of the forward-layout 256² kernels are such; they are launched under the same trace label as the
# plain ones, so the label's traffic is the launch-weighted mean over both (the same launches its algorithmic bytes
# average over).
PMC_ALIASES = {
    'gemm8p_kernel<true,true,bf16>': ('gemm8p_kernel<bool _Accum, bool, E, true, bool _Accum, bool, E, 2>',),
}


def _pmc_hits(label, path):
    """Per-kernel records of a committed PMC summary (tools/pmc_traffic.py / tools/pmc_mfma.py JSON) that belong to
    the traced kernel `label` (e.g. 'gemm256_kernel<false,false,float>'), and the file's provenance."""
    if not path or not os.path.exists(path) or '<' not in label:
        return None, None
    base, args = label.split('<', 1)
    code = {'true': 'Lb1E', 'false': 'Lb0E', 'bf16': 'DF16b', 'float': 'f'}
    codes = ''.join(code[a.strip()] for a in args.rstrip('>').split(','))
    # the GEMM kernels take the MFMA number format E (bf16 on this path) as their first template argument
    mangled = (base + 'I' + codes, base + 'IDF16b' + codes)
    with open(path) as f:
        doc = json.load(f)
    ks = doc['kernels']
    demangled = base + '<' + ', '.join(a.strip() for a in args.rstrip('>').split(','))   # rocprof demangles some
    aliases = PMC_ALIASES.get(label.replace(' ', ''), ())
    hits = [v for k, v in ks.items() if any(mg in k for mg in mangled) or demangled in k or
            any(a in k for a in aliases)]
    return hits, {'file': os.path.relpath(path, REPO), 'commit': doc.get('commit'), 'cmd': doc.get('cmd')}


def pmc_traffic(label, path=TRAFFIC_JSON):
    """HBM bytes per launch of the traced kernel `label` from a committed PMC summary of this same bench command
    (tools/pmc_traffic.py: FETCH_SIZE x2 + WRITE_SIZE per dispatch), with the commit of the build it was measured
    on; None when the file or the kernel is absent."""
    hits, src = _pmc_hits(label, path)
    if not hits:
        return None, src
    n = sum(v['dispatches'] for v in hits)
    return int(sum(v['hbm_bytes_per_launch'] * v['dispatches'] for v in hits) / n), src


def mfma_util(label, path=MFMA_JSON):
    """MFMA-pipe utilisation of the traced kernel from a committed PMC pass of this same bench command
    (tools/pmc_mfma.py: SQ_VALU_MFMA_BUSY_CYCLES / (4 SIMDs x 256 CUs x GRBM_GUI_ACTIVE / 8 XCDs), i.e. the share of
    the kernel's SIMD-cycles with the matrix pipe busy at the clock it actually ran), or None."""
    hits, src = _pmc_hits(label, path)
    if not hits:
        return None
    busy = sum(v['mfma_busy_cycles_per_launch'] * v['dispatches'] for v in hits)
    grbm = sum(v['grbm_gui_active_per_launch'] * v['dispatches'] for v in hits)
    n = sum(v['dispatches'] for v in hits)
    return {'util': round(busy / (grbm / 8 * 256 * 4), 4) if grbm else None,
            'mfma_busy_cycles_per_launch': int(busy / n), 'grbm_gui_active_per_launch': int(grbm / n),
            'effective_clock_ghz': hits[0].get('effective_clock_ghz'), 'source': src}


def _videomae_overlap():
    from cmhar import videomae
    return bool(videomae._OVERLAP_WGRAD)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=50)     # >= 50 timed steps after >= 10 warm-up
    ap.add_argument('--warmup', type=int, default=10)
    ap.add_argument('--workload', default='videomae', choices=sorted(WORKLOADS))
    ap.add_argument('--batch', type=int, default=None)
    ap.add_argument('--frames', type=int, default=None)
    ap.add_argument('--image', type=int, default=None)
    ap.add_argument('--imu-len', type=int, default=None)
    ap.add_argument('--dtype', default=None, choices=['bf16', 'fp32', 'fp16'])
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-batch', type=int, default=4)       # BASELINE.md CPU-baseline plan: batch 4,
    ap.add_argument('--cpu-warmup', type=int, default=2)      # 2 warm-up + 3 timed steps, all host cores
    ap.add_argument('--cpu-steps', type=int, default=3)
    ap.add_argument('--traffic-json', default=TRAFFIC_JSON)
    ap.add_argument('--mfma-json', default=MFMA_JSON)
    ap.add_argument('--no-trace', action='store_true')
    ap.add_argument('--imu-stream', choices=['side', 'main'], default='side',
                    help='run the IMU branch on its own HIP stream (overlapping the video branch) or on the main one')
    args = ap.parse_args()
    for k, v in WORKLOADS[args.workload].items():
        if getattr(args, k) is None:
            setattr(args, k, v)
    if args.workload == 'ood_fp16' and '--steps' not in sys.argv:
        args.steps = 313                 # BASELINE config 5: a 10k-clip stream (313 batches of 32)
    return args


def measure_mfma_peak(dev, blocks=2048, iters=10000, reps=3, per_shape=None):
    """The on-box dense bf16 MFMA rate: csrc/probe.hip's back-to-back bf16 MFMAs (8 chains per wave) on
    random fragments over every SIMD (2048 workgroups × 4 waves), both shapes — v_mfma_f32_32x32x16_bf16 (attention)
    and v_mfma_f32_16x16x32_bf16 (GEMMs), which the chip runs at different clocks on random data — one launch each
    ≈ 10–20 ms, timed with HIP events on the launch stream; the best of `reps` after one warm launch per shape.
    Returns the larger rate in TFLOP/s; `per_shape` (a dict) receives both."""
    from cmhar import _lib as L
    g = torch.Generator(device=dev).manual_seed(77)
    ops = torch.randn(512 * 8, device=dev, generator=g).bfloat16()
    out = torch.empty(blocks * 256, device=dev)
    st = torch.cuda.current_stream(dev)
    rates = {}
    for shape, name in ((0, '32x32x16'), (1, '16x16x32')):
        flops = L.lib().cmhar_mfma_peak_probe_flops(shape, blocks, iters)
        best = 0.0
        for r in range(reps + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            L.call('cmhar_mfma_peak_probe', shape, blocks, iters, ops.data_ptr(), 512, out.data_ptr(), L.stream(dev))
            e1.record(st)
            e1.synchronize()
            if r:
                best = max(best, flops / (e0.elapsed_time(e1) / 1e3) / 1e12)
        if not torch.isfinite(out).all():
            raise RuntimeError('MFMA peak probe produced non-finite sums')
        rates[name] = round(best, 1)
    if per_shape is not None:
        per_shape.update(rates)
    return max(rates.values())


def videomae_flops_per_clip(T, H, W, hd=768, layers=12, inter=3072, P=16, tub=2, C=3):
    """Algorithmic forward FLOPs of VideoMAE-B per clip."""
    N = (T // tub) * (H // P) * (W // P)
    embed = 2 * N * (C * tub * P * P) * hd
    per_layer = 2 * N * hd * (4 * hd + 2 * inter) + 4 * N * N * hd
    return embed, embed + layers * per_layer


def token0_last_layer_saving(T, H, W, hd=768, inter=3072, P=16, tub=2):
    """(forward, forward+backward) FLOPs per clip that the token-0 last layer (cmhar/videomae.py
    _last_layer_token0_fwd / _bwd) does not execute: the query projection, attention, out-projection and MLP of the
    N − 1 rows whose outputs the model never returns.  Backward = 2× forward for the GEMMs, 2.5× for attention
    (10·L²·D vs 4·L²·D), the convention of SURVEY §8d's 3·F_fwd total."""
    N = (T // tub) * (H // P) * (W // P)
    gemm = 2 * (N - 1) * hd * (2 * hd + 2 * inter)       # Q projection + out-projection + FC1 + FC2
    attn = 4 * (N * N - N) * hd
    return gemm + attn, 3 * gemm + 3.5 * attn


def host_cpu():
    """(model name, cores this process may run on): the box's CPU share, not the whole machine's count."""
    name = 'unknown'
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    name = line.split(':', 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    try:                      # a cgroup CPU quota (e.g. '1600000 100000' = 16 cores) caps the usable cores
        with open('/sys/fs/cgroup/cpu.max') as f:
            quota, period = f.read().split()[:2]
        if quota != 'max':
            cores = max(1, min(cores, int(quota) // int(period)))
    except (OSError, ValueError):
        pass
    return name, cores


def log(msg):
    print(f'[bench] {msg}', file=sys.stderr, flush=True)


def cpu_baseline(cfg_builder, batch, warmup, steps, frames, image, imu_len):
    """The CPU oracle (torch-eager fp32 restatement of the reference path, validated against the reference's
    golden vectors) timed on every host core this process may use: the training step (fwd+bwd+clip+AdamW) and,
    as a second row, the eval-mode forward."""
    sys.path.insert(0, REPO)
    from oracle import cpu_model as O
    cpu_name, threads = host_cpu()
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

    def fwd():
        with torch.no_grad():
            O.crossmodal(sd, imu, video, mc, training=False)

    log(f'cpu baseline: {threads} threads on {cpu_name}, batch {batch}, {warmup} + {steps} steps')
    for i in range(warmup):
        step(i + 1)
        log(f'cpu warm-up step {i + 1} done')
    t0 = time.perf_counter()
    for i in range(steps):
        step(warmup + i + 1)
        log(f'cpu timed step {i + 1}: {time.perf_counter() - t0:.1f} s')
    dt = time.perf_counter() - t0
    fwd()
    t1 = time.perf_counter()
    for i in range(steps):
        fwd()
        log(f'cpu eval forward {i + 1}: {time.perf_counter() - t1:.1f} s')
    dte = time.perf_counter() - t1
    rows = {}
    if image > 112:
        # BASELINE.md plan: the same procedure at 16x112^2 (the sinusoid position table follows the token count)
        video112 = torch.randn(batch, frames, 3, 112, 112, generator=g)
        vsave = video

        def run112(train):
            nonlocal video
            video = video112
            try:
                if train:
                    step(warmup + steps + 1)
                else:
                    fwd()
            finally:
                video = vsave
        run112(True)
        t2 = time.perf_counter()
        for i in range(steps):
            run112(True)
        rows['train_112_clips_per_sec'] = round(batch * steps / (time.perf_counter() - t2), 4)
        run112(False)
        t2 = time.perf_counter()
        for i in range(steps):
            run112(False)
        rows['eval_fwd_112_clips_per_sec'] = round(batch * steps / (time.perf_counter() - t2), 4)
        log(f'cpu 112^2 rows: {rows}')
    # IMU-only (batch 8): the IMU encoder + its projection head + F.normalize, fwd+bwd against fixed unit targets
    # through the SigLIP loss, clip + AdamW over the IMU-side parameters
    imu8 = torch.randn(8, 6, imu_len, generator=g)
    tgt = O.l2_normalize(torch.randn(8, 256, generator=g))
    inames = [k for k in names if k.startswith(('imu_encoder.', 'imu_proj.'))]
    im = [torch.zeros_like(sd[k]) for k in inames]
    iv = [torch.zeros_like(sd[k]) for k in inames]

    def imu_step(i):
        for k in inames:
            sd[k].grad = None
        cls, _ = O.imu_encoder(sd, imu8, patch_size=16, stride=16, nhead=8, num_layers=4, dropout=0.1, training=True,
                               gen=g)
        a = O.l2_normalize(O.projection_head(sd, cls, 'imu_proj.', True))
        O.siglip_loss(a, tgt, lt, lb).backward()
        with torch.no_grad():
            grads = [sd[k].grad for k in inames]
            O.clip_grad_norm(grads, 1.0)
            O.adamw_step([sd[k] for k in inames], grads, im, iv, i, lr=1e-5)
    try:
        for i in range(warmup):
            imu_step(i + 1)
        t3 = time.perf_counter()
        for i in range(steps):
            imu_step(warmup + i + 1)
        rows['imu_only_b8_train_windows_per_sec'] = round(8 * steps / (time.perf_counter() - t3), 2)
    except (TypeError, KeyError) as e:   # an oracle signature mismatch must not take the bench line down
        log(f'cpu IMU-only row skipped: {e!r}')
    return {'value': round(batch * steps / dt, 4), 'unit': 'clips/sec', 'cores': threads, 'kind': 'port', **rows,
            'cpu_model': cpu_name,
            'eval_fwd_clips_per_sec': round(batch * steps / dte, 4),
            'sample': f'oracle/cpu_model.py fp32 fwd+bwd+clip+AdamW, batch {batch}, {warmup} warm-up + {steps} timed '
                      f'steps, {frames}x{image}^2 video + 6x{imu_len} IMU, {threads} threads on {cpu_name}; eval row: '
                      f'eval-mode forward, {steps} timed batches after 1 warm-up; 112 rows: the same two procedures on '
                      f'16x112^2 clips (1 warm-up, {steps} timed); IMU-only row: batch 8 IMU encoder + projection head '
                      f'+ normalize, SigLIP loss against fixed unit targets, fwd+bwd+clip+AdamW over the IMU-side '
                      f'parameters, {warmup} warm-up + {steps} timed'}


def r3d_flops(m, B, T, H, W):
    """(forward, stem forward) algorithmic FLOPs of the R3D-18 backbone for B clips: 2·M·Cout·K per conv."""
    from cmhar.r3d import _out_shape
    shape = (B, T, H, W, 3)
    tot = 0

    def conv(shp, c):
        nonlocal tot
        o = _out_shape(shp, c)
        f = 2 * math.prod(o[:4]) * c.out_channels * c.weight[0].numel()
        tot += f
        return o, f

    shape, stem = conv(shape, m.stem[0])
    for blk in m.blocks():
        s1, _ = conv(shape, blk.conv1[0])
        if blk.downsample is not None:
            conv(shape, blk.downsample[0])
        shape, _ = conv(s1, blk.conv2[0])
    return tot, stem


class Workload:
    """One benchmark configuration: `step()` runs one step on this rank's resident batch; `flops_per_clip` is the
    step's algorithmic FLOPs per clip (the whole-step roofline numerator)."""


def imu_flops_per_window(T, d=128, layers=4, ff=512, patch=16, hidden=(256, 128), classes=32):
    """Algorithmic FLOPs of one IMU window's forward: patch embedding, `layers` post-LN encoder layers over
    n = (T - patch) // patch + 2 tokens (patches + CLS), the MLP head."""
    n = (T - patch) // patch + 2
    embed = 2 * (n - 1) * patch * d
    layer = 2 * n * (4 * d * d + 2 * d * ff) + 4 * n * n * d
    dims = (d,) + tuple(hidden) + (classes,)
    head = sum(2 * a * b for a, b in zip(dims, dims[1:]))
    return embed + layers * layer + head


def _imu_workload(args, W, dev, rank, world):
    """BASELINE config 1: ClassificationTrainer.train_step (finetune) of the IMU-only classifier."""
    from cmhar import dist as cdist
    from cmhar.models import IMUClassifier, IMUEncoder
    from cmhar.trainer import ClassificationTrainer
    cfg = W.make_cfg()
    model = IMUClassifier(IMUEncoder(cfg), cfg).to(dev).train()
    cdist.broadcast_parameters(model)
    reducer = cdist.GradReducer(model) if world > 1 else None
    tr = ClassificationTrainer(model, cfg, device=dev, mode='finetune', grad_reducer=reducer)
    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    B = args.batch
    imu = torch.randn(B, 6, args.imu_len, device=dev, generator=g)
    labels = torch.randint(0, cfg.model.num_classes, (B,), device=dev, generator=g)

    def step():
        return tr.train_step(imu, labels)[1]
    W.model, W.B, W.step, W.training = model, B, step, True
    W.flops_per_clip = 3 * imu_flops_per_window(args.imu_len, ff=4 * cfg.model.imu_d_model,
                                                hidden=tuple(cfg.model.classifier_hidden_dims),
                                                classes=cfg.model.num_classes)
    W.metric = f'windows/sec IMU-only classifier train step (BASELINE config 1), 6x{args.imu_len}, batch {B}'
    W.workload = (f'IMUClassifier fine-tune step (ClassificationTrainer.train_step): PatchTST IMU encoder 6x'
                  f'{args.imu_len} + 256-128 MLP head, CE, clip 1.0, AdamW; fp32')
    return W


def build_workload(args, dev, rank, world):
    import warnings
    from cmhar import dist as cdist
    from cmhar import kernels as K
    from cmhar.config import Config
    from cmhar.losses import SigmoidContrastiveLoss, cross_entropy
    from cmhar.models import CrossModalModel
    from cmhar.optim import FusedAdamW

    def make_cfg():
        cfg = Config()
        cfg.model.allow_random_init = True   # synthetic benchmark: random-init weights
        cfg.data.imu_window_size = args.imu_len
        cfg.data.video_frames_per_window = args.frames
        cfg.data.video_resize = (args.image, args.image)
        cfg.model.compute_dtype = args.dtype
        if args.workload == 'r3d':
            cfg.model.video_backbone = 'r3d_18'
        return cfg

    W = Workload()
    W.make_cfg = make_cfg
    torch.manual_seed(0)
    if args.workload == 'imu':
        return _imu_workload(args, W, dev, rank, world)
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')          # hub checkpoint not fetchable offline → random init
        if args.workload == 'fusion':
            from cmhar.fusion import CrossModalFusionClassifier
            model = CrossModalFusionClassifier(make_cfg())
        else:
            model = CrossModalModel(make_cfg())
    B = args.batch
    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    embed_f, fwd_f = videomae_flops_per_clip(args.frames, args.image, args.image)
    W.model, W.B = model, B
    if args.workload == 'ood_fp16':
        from cmhar.ood import logits_energy
        model = model.to(dev).eval()
        ring = [(torch.randn(B, 6, args.imu_len, device=dev, generator=g),
                 torch.randn(B, args.frames, 3, args.image, args.image, device=dev, generator=g)) for _ in range(8)]
        S = torch.empty(B, B, device=dev)
        bias = torch.full((B,), -10.0, device=dev)
        it = [0]

        def step():
            imu, video = ring[it[0] % len(ring)]
            it[0] += 1
            with torch.no_grad():
                a, b = model(imu, video)
                K.gemm(0, a, b, S, bias=bias, alpha=10.0)       # SigLIP logits exp(log 10)·a·bᵀ + bias
                pred, energy, _ = logits_energy(S)
            return energy
        W.step, W.flops_per_clip = step, fwd_f
        W.metric = 'clips/sec OOD energy-score eval stream, fp16 inference, 16x224^2 video + 200x6 IMU, batch 32'
        W.workload = (f'OOD eval stream (BASELINE config 5): CrossModalModel eval forward, VideoMAE-B {args.frames}x'
                      f'{args.image}^2 + IMU 6x{args.imu_len}, SigLIP logits, energy score; ring of 8 distinct batches')
        W.training = False
        return W

    model = model.to(dev).train()
    if args.workload != 'fusion':
        model.overlap_imu = args.imu_stream == 'side'
    backbone = model.video_encoder.backbone
    cdist.broadcast_parameters(model)
    # CMHAR_BENCH_REDUCE_SINGLE=1 (rehearsal): on one GPU, the reducer runs its whole bucket / RCCL protocol in a
    # one-rank group — the per-step cost of the data-parallel machinery without the transfers
    reducer = cdist.GradReducer(model, backbone=backbone,
                                reduce_single=os.environ.get('CMHAR_BENCH_REDUCE_SINGLE') == '1')
    # LinearLR(start_factor=0.1) of trainer.py:80-105 → step-0 lr = 0.1 * pretrain_lr
    params = [p for n, p in model.named_parameters() if not (args.workload == 'fusion' and
                                                              n.startswith('video_encoder.projection.'))]
    # max_grad_norm: clip_grad_norm_(params, 1.0) folded into the AdamW pass, as CrossModalTrainer does
    opt = FusedAdamW(params, lr=0.1 * 1e-4, weight_decay=0.01,
                     shadow_sources=[backbone] if args.workload != 'r3d' else [], max_grad_norm=1.0)
    video = torch.randn(B, args.frames, 3, args.image, args.image, device=dev, generator=g)
    imu = torch.randn(B, 6, args.imu_len, device=dev, generator=g)
    if args.workload == 'fusion':
        labels = torch.randint(0, model.fusion.classifier.out_features, (B,), device=dev, generator=g)

        def loss_of():
            # global-batch mean CE under data parallelism (equal shards): the SUM all-reduce of the gradients of
            # mean/world gives the gradient of DataParallel's gathered mean
            loss = cross_entropy(model(imu, video), labels)
            return loss * (1.0 / world) if world > 1 else loss
        Lk = (args.frames // 2) * (args.image // 16) ** 2
        Lq = 1 + (args.imu_len - 16) // 16 + 1
        fus = 2 * Lk * 768 * 512 + 4 * Lq * Lk * 256          # K|V projection + attention (fwd, per clip)
        W.flops_per_clip = 3 * fwd_f - embed_f + 3 * fus
        W.metric = (f'clips/sec fwd+bwd, cross-attention fusion {args.frames}x{args.image}^2 video + '
                    f'{args.imu_len}x6 IMU, batch {B} per GPU')
        W.workload = (f'CrossModalFusionClassifier train step (BASELINE config 4): IMU 6x{args.imu_len} tokens x '
                      f'VideoMAE-B {args.frames}x{args.image}^2 tokens, CE loss, clip 1.0, AdamW')
    else:
        loss_fn = SigmoidContrastiveLoss().to(dev)

        def loss_of():
            a, b = model(imu, video)
            return loss_fn(a, b)
        if args.workload == 'r3d':
            fwd_r, stem = r3d_flops(backbone, B, args.frames, args.image, args.image)
            W.flops_per_clip = (3 * fwd_r - stem) / B
            W.metric = f'clips/sec fwd+bwd, R3D-18 {args.frames}x{args.image}^2 video + 200x6 IMU, batch {B}'
            W.workload = (f'CrossModalModel pretrain step, video_backbone=r3d_18 (BASELINE config 2): R3D-18 '
                          f'{args.frames}x{args.image}^2 + IMU 6x{args.imu_len}, SigLIP loss, clip 1.0, AdamW')
        else:
            W.flops_per_clip = 3 * fwd_f - embed_f     # fwd + 2x bwd, no pixel gradient for the tubelet conv
            if os.environ.get('CMHAR_TOKEN0_LAST', '1') != '0' and (B % 8 == 0 or args.dtype == 'fp32'):
                W.executed_flops_per_clip = W.flops_per_clip - token0_last_layer_saving(args.frames, args.image,
                                                                                        args.image)[1]
            W.metric = 'clips/sec fwd+bwd, 16x224^2 video + 200x6 IMU, batch 32, 1/2/4/8 GPU'
            W.workload = (f'CrossModalModel pretrain step: VideoMAE-B {args.frames}x{args.image}^2 + '
                          f'IMU 6x{args.imu_len} PatchTST, SigLIP loss, clip 1.0, AdamW')

    def step():
        loss = loss_of()
        opt.zero_grad(set_to_none=True)
        reducer.start_step()
        loss.backward()
        reducer.finish()
        opt.step()               # clip_grad_norm_(params, 1.0) + AdamW (trainer.py:140-141)
        return loss
    W.step, W.training = step, True
    return W


def main():
    args = parse()
    from cmhar import dist as cdist
    from cmhar import kernels as K

    # CMHAR_BENCH_BACKEND / CMHAR_BENCH_DEVICE: rehearsal knobs only (e.g. two gloo ranks sharing the one GPU of a
    # test box); the measured configuration is one RCCL rank per GPU
    rank, world, local = cdist.init_from_env(os.environ.get('CMHAR_BENCH_BACKEND') or None)
    local = int(os.environ.get('CMHAR_BENCH_DEVICE', local))
    torch.cuda.set_device(local)
    if world == 1 and os.environ.get('CMHAR_BENCH_REDUCE_SINGLE') == '1' and not dist.is_initialized():
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        os.environ.setdefault('MASTER_PORT', '29533')
        dist.init_process_group(os.environ.get('CMHAR_BENCH_BACKEND') or 'nccl', rank=0, world_size=1)
    dev = torch.device('cuda', local)
    W = build_workload(args, dev, rank, world)
    step, B = W.step, W.B
    headline = args.workload == 'videomae'
    trace = headline and not args.no_trace

    # Warm-up; its last step runs with every GEMM / attention launch bracketed by HIP events, which gives the
    # per-kernel-family breakdown and picks the dominant single kernel.  The timed loop then brackets ONLY that
    # kernel's launches (the events of all ~180 traced launches cost ~1.5 ms/step of stream bubbles).
    # The traced warm-up step runs the backward's weight gradients on the main stream (overlap_wgrad off): its
    # per-kernel times are then each kernel alone on the chip, not shares of two concurrent streams.
    breakdown = {}
    loss = None
    bb = getattr(getattr(W.model, 'video_encoder', None), 'backbone', None)
    for i in range(args.warmup):
        full = trace and i == args.warmup - 1
        if full:
            K.TRACE.records, K.TRACE.only, K.TRACE.active = [], None, True
            if bb is not None:
                bb.overlap_wgrad = False
        loss = step()
        if full:
            torch.cuda.synchronize()
            K.TRACE.active = False
            breakdown = K.TRACE.summary()
            if bb is not None:
                del bb.overlap_wgrad
    torch.cuda.synchronize()
    first_loss = float(loss.float().mean().item()) if loss is not None else float('nan')
    # every traced label is one kernel symbol except the two-kernel attention backward entry
    # (the hipBLASLt label spans several vendor kernels, one per shape: not a single-kernel candidate)
    single = {k: v for k, v in breakdown.items() if '(' not in k and k != 'hipblaslt_linear'}
    dominant = max(single.items(), key=lambda kv: kv[1][1])[0] if single else None
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    K.TRACE.records = []
    K.TRACE.only = {dominant} if dominant else None
    K.TRACE.active = trace and dominant is not None
    if rank == 0:
        log(f'warm-up done ({args.warmup} steps, loss {first_loss:.5f}); timing {args.steps} steps')
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if rank == 0:
        log(f'timed region: {elapsed:.3f} s')
    K.TRACE.active = False
    last_losses = None
    if world > 1:
        dist.barrier()
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        # the loss is taken over the gathered global batch (DataParallel semantics): identical on every rank
        last_losses = [None] * world
        dist.all_gather_object(last_losses, float(loss.float().mean().item()) if loss is not None else None)
    clips = world * B * args.steps
    value = clips / elapsed
    ms = 1000 * elapsed / args.steps
    peak = PEAK_F32_TFLOPS if args.dtype == 'fp32' else PEAK_BF16_TFLOPS     # fp16 dense MFMA = bf16 rate
    # model FLOP rate over the FLOPs the step EXECUTES (the token-0 last layer skips rows the model never returns);
    # the reference model's algorithmic total is reported beside it
    exec_flops = getattr(W, 'executed_flops_per_clip', W.flops_per_clip)
    whole_tflops = exec_flops * clips / elapsed / 1e12

    # dominant kernel: the single HIP kernel with the largest traced time in the traced warm-up step (split-K GEMMs
    # are traced without their reduce launch); achieved = its algorithmic FLOPs / its HIP-event-measured time over
    # the timed region.  In the timed region the backward's weight gradients run on a second stream, so a backward
    # kernel's launch duration there is its share of a chip it splits with the other stream; `isolated_*` is the same
    # kernel in the serial traced warm-up step.
    roof = None
    peak_meas = None
    peak_shapes = {}
    if headline and rank == 0 and os.environ.get('CMHAR_BENCH_PEAK_PROBE', '1') == '1':
        peak_meas = measure_mfma_peak(dev, per_shape=peak_shapes)   # after the timed region: no perturbation
        log(f'on-box MFMA peak probe: {peak_meas:.1f} TFLOP/s')
    summ = K.TRACE.summary() if trace else {}
    if dominant in summ:
        name = dominant
        n, tot_ms, fl, nb = summ[name]
        achieved = fl / (tot_ms / 1e3) / 1e12
        traffic, tsrc = pmc_traffic(name, args.traffic_json)
        roof = {'bound': 'mfma', 'achieved': round(achieved, 1), 'peak': PEAK_BF16_TFLOPS, 'unit': 'TFLOP/s',
                'frac': round(achieved / PEAK_BF16_TFLOPS, 4),
                'peak_measured': round(peak_meas, 1) if peak_meas else None,
                'frac_of_measured_peak': round(achieved / peak_meas, 4) if peak_meas else None,
                'peak_measured_per_shape': peak_shapes or None,
                'peak_note': 'frac divides by the vendor dense bf16 peak (2.5 PF); peak_measured = csrc/probe.hip '
                             'back-to-back bf16 MFMAs on random fragments (the faster of the 32x32x16 and 16x16x32 '
                             'shapes), every SIMD, this box',
                'traffic': traffic, 'traffic_source': tsrc,
                'kernel': name,
                'launches': n, 'avg_launch_ms': round(tot_ms / n, 4),
                'algorithmic_bytes_per_launch': int(nb / n),
                # both per launch over the same launches of the label (PMC: dispatch-weighted over its instantiations)
                'traffic_over_algorithmic': round(traffic / (nb / n), 3) if traffic else None}
        if name in breakdown:
            bn_, btm, bfl, _ = breakdown[name]
            iso = bfl / (btm / 1e3) / 1e12
            roof.update({'isolated_avg_launch_ms': round(btm / bn_, 4), 'isolated_achieved': round(iso, 1),
                         'isolated_frac': round(iso / PEAK_BF16_TFLOPS, 4),
                         'concurrent_streams': 'backward weight gradients on a second stream'
                         if bb is not None and _videomae_overlap() else None})
        mf = mfma_util(name, args.mfma_json)
        if mf is not None:
            roof['mfma_util'] = mf
    elif not headline:
        roof = {'bound': 'mfma', 'achieved': round(whole_tflops, 1), 'peak': peak, 'unit': 'TFLOP/s',
                'frac': round(whole_tflops / peak, 4), 'traffic': None, 'kernel': 'whole step (all kernels)'}

    out = {'metric': W.metric, 'value': round(value, 3),
           'unit': 'clips/sec', 'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
           'ms_per_step': round(ms, 3), 'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
           'dtype': args.dtype, 'data': f'synthetic (randn video/IMU resident in HBM, random-init weights)',
           'config': {'workload': W.workload, 'global_batch': world * B, 'per_gpu_batch': B,
                      'parallelism': f'dp{world}'},
           'roofline': roof,
           'whole_step_model_tflops': round(whole_tflops, 1),
           'whole_step_mfma_frac': round(whole_tflops / peak, 4),
           'whole_step_frac_of_measured_peak': round(whole_tflops / peak_meas, 4) if peak_meas else None,
           'executed_gflop_per_clip': round(exec_flops / 1e9, 2),
           'reference_algorithmic_gflop_per_clip': round(W.flops_per_clip / 1e9, 2),
           'first_warmup_loss': first_loss,
           'last_loss_per_rank': last_losses,
           'max_mem_gb': round(torch.cuda.max_memory_allocated(dev) / 2 ** 30, 1)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline and headline:
        out['cpu_baseline'] = cpu_baseline(W.make_cfg, args.cpu_batch, args.cpu_warmup, args.cpu_steps, args.frames,
                                           args.image, args.imu_len)
    if rank == 0:
        if breakdown:   # one traced warm-up step
            out['kernels'] = {k: {'launches': n, 'ms_per_step': round(tm, 3),
                                  'tflops': round(f / (tm / 1e3) / 1e12, 1)} for k, (n, tm, f, b) in breakdown.items()}
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
