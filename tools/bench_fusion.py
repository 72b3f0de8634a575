"""BASELINE config 4's model on one GPU: CrossModalFusionClassifier (IMU encoder tokens x VideoMAE-B tokens through
the cross-attention fusion, cmhar/fusion.py) training step — forward, cross-entropy, backward, clip 1.0, fused AdamW —
at 32x224^2 clips + 6x400 IMU, 8 clips per GPU (config 4's global batch 64 over 8 GPUs), bf16, synthetic inputs
resident in HBM.  Prints one JSON line (clips/s, ms/step, model TFLOP/s from the VideoMAE-B FLOP formula of
SURVEY §8d plus the fusion's K|V projection and attention).
    python tools/bench_fusion.py [--steps 10 --warmup 3 --batch 8 --frames 32 --image 224 --imu-len 400]
"""
import argparse
import json
import os
import sys
import time
import warnings

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'crossmodal-imu-video-ood-har_amd'))
from bench import videomae_flops_per_clip  # noqa: E402
from cmhar.config import Config  # noqa: E402
from cmhar.fusion import CrossModalFusionClassifier  # noqa: E402
from cmhar.losses import cross_entropy  # noqa: E402
from cmhar.optim import FusedAdamW, clip_grad_norm_  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--batch', type=int, default=8)
    ap.add_argument('--frames', type=int, default=32)
    ap.add_argument('--image', type=int, default=224)
    ap.add_argument('--imu-len', type=int, default=400)
    args = ap.parse_args()
    dev = torch.device('cuda')
    cfg = Config()
    cfg.model.allow_random_init = True   # synthetic benchmark: random-init weights
    cfg.model.compute_dtype = 'bf16'
    cfg.data.video_frames_per_window = args.frames
    cfg.data.video_resize = (args.image, args.image)
    cfg.data.imu_window_size = args.imu_len
    torch.manual_seed(0)
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        model = CrossModalFusionClassifier(cfg).to(dev).train()
    params = [p for n, p in model.named_parameters() if not n.startswith('video_encoder.projection.')]
    opt = FusedAdamW(params, lr=1e-5, weight_decay=0.01, shadow_sources=[model.video_encoder.backbone])
    g = torch.Generator(device=dev).manual_seed(1000)
    B = args.batch
    video = torch.randn(B, args.frames, 3, args.image, args.image, device=dev, generator=g)
    imu = torch.randn(B, 6, args.imu_len, device=dev, generator=g)
    labels = torch.randint(0, cfg.model.num_classes, (B,), device=dev, generator=g)

    def step():
        loss = cross_entropy(model(imu, video), labels)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        clip_grad_norm_(params, 1.0)
        opt.step()
        return loss

    for _ in range(args.warmup):
        loss = step()
    torch.cuda.synchronize()
    first = float(loss.item())
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    embed, fwd = videomae_flops_per_clip(args.frames, args.image, args.image)
    Lk = (args.frames // 2) * (args.image // 16) ** 2
    Lq = 1 + (args.imu_len - 16) // 16 + 1
    fus = 2 * Lk * 768 * 512 + 4 * Lq * Lk * 256          # K|V projection + attention (fwd, per clip)
    step_flops = B * (3 * fwd - embed + 3 * fus)
    tf = step_flops * args.steps / el / 1e12
    print(json.dumps({
        'metric': f'clips/sec fwd+bwd, cross-attention fusion {args.frames}x{args.image}^2 video + '
                  f'{args.imu_len}x6 IMU, batch {B} per GPU, 1 GPU',
        'value': round(B * args.steps / el, 3), 'unit': 'clips/sec', 'n_gpus': 1, 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': round(1000 * el / args.steps, 3), 'dtype': 'bf16',
        'data': 'synthetic (randn video/IMU/labels resident in HBM, random-init VideoMAE-B + fusion)',
        'config': {'workload': 'CrossModalFusionClassifier train step (IMU tokens x VideoMAE-B tokens, CE loss)',
                   'per_gpu_batch': B, 'parallelism': 'dp1'},
        'model_gflop_per_clip': round(step_flops / B / 1e9, 1), 'model_tflops': round(tf, 1),
        'mfma_frac': round(tf / PEAK_BF16_TFLOPS, 4), 'loss_after_warmup': first,
        'max_mem_gb': round(torch.cuda.max_memory_allocated() / 2 ** 30, 1)}))


if __name__ == '__main__':
    main()
