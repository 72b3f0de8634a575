"""CrossModalModel pretraining step with the reference's per-frame 2-D CNN video backbones (`video_backbone`
'resnet18' / 'mobilenet_v2', src/models/models.py:163-173,208-216) at 16x224^2 clips (the reference's default
video geometry, 512 frames per batch of 32) + 6x200 IMU, bf16, one MI355X.

Same step as bench.py (forward, SigLIP loss, backward, clip 1.0, fused AdamW) on synthetic inputs resident in HBM.
Prints one JSON line: clips/s, frames/s, ms/step and the backbone's algorithmic TFLOP/s (conv FLOPs from the layer
geometry: 2·Ho·Wo·Cout·(Cin/groups)·k² per conv per frame; fwd+bwd = 3x minus the stem's input gradient).
    python tools/bench_cnn2d.py --video-backbone resnet18|mobilenet_v2 [--steps 10 --warmup 3 --batch 32]
"""
import argparse
import json
import os
import sys
import time
import warnings

import torch
import torch.nn as nn

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'crossmodal-imu-video-ood-har_amd'))
from cmhar.config import Config  # noqa: E402
from cmhar.losses import SigmoidContrastiveLoss  # noqa: E402
from cmhar.models import CrossModalModel  # noqa: E402
from cmhar.optim import FusedAdamW, clip_grad_norm_  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0


def conv_flops(backbone, H, W):
    """(forward FLOPs per frame, stem forward FLOPs per frame), walking the convs in execution order with their
    output sizes (every conv of both networks is square with 'same'-style padding, so sizes follow the strides)."""
    tot, stem = 0, None
    h, w = H, W
    for mod in backbone.modules():
        if isinstance(mod, nn.Conv2d):
            k, s, p = mod.kernel_size[0], mod.stride[0], mod.padding[0]
            # a downsample 1x1 conv runs on its block's input: its stride equals the block's first conv's stride, and
            # the spatial size was already reduced by that conv — undo for this one conv
            if isinstance(mod, nn.Conv2d) and k == 1 and s == 2:
                hi, wi = h * 2, w * 2
            else:
                hi, wi = h, w
            ho, wo = (hi + 2 * p - k) // s + 1, (wi + 2 * p - k) // s + 1
            f = 2 * ho * wo * mod.out_channels * (mod.in_channels // mod.groups) * k * k
            tot += f
            if stem is None:
                stem = f
            h, w = ho, wo
        elif isinstance(mod, nn.MaxPool2d):
            h, w = (h + 2 * mod.padding - mod.kernel_size) // mod.stride + 1, \
                (w + 2 * mod.padding - mod.kernel_size) // mod.stride + 1
    return tot, stem


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--video-backbone', choices=['resnet18', 'mobilenet_v2'], default='resnet18')
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--batch', type=int, default=32)
    ap.add_argument('--frames', type=int, default=16)
    ap.add_argument('--image', type=int, default=224)
    args = ap.parse_args()
    dev = torch.device('cuda')
    cfg = Config()
    cfg.model.allow_random_init = True   # synthetic benchmark: random-init weights (ImageNet weights not fetchable)
    cfg.model.video_backbone = args.video_backbone
    cfg.model.compute_dtype = 'bf16'
    cfg.data.video_frames_per_window = args.frames
    cfg.data.video_resize = (args.image, args.image)
    torch.manual_seed(0)
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        model = CrossModalModel(cfg).to(dev).train()
    loss_fn = SigmoidContrastiveLoss().to(dev)
    params = list(model.parameters())
    opt = FusedAdamW(params, lr=1e-5, weight_decay=0.01)
    g = torch.Generator(device=dev).manual_seed(1000)
    B = args.batch
    video = torch.randn(B, args.frames, 3, args.image, args.image, device=dev, generator=g)
    imu = torch.randn(B, 6, 200, device=dev, generator=g)

    def step():
        a, b = model(imu, video)
        loss = loss_fn(a, b)
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
    fwd, stem = conv_flops(model.video_encoder.backbone, args.image, args.image)
    frames = B * args.frames
    step_flops = (3 * fwd - stem) * frames
    tf = step_flops * args.steps / el / 1e12
    print(json.dumps({
        'metric': f'clips/sec fwd+bwd, {args.video_backbone} per-frame {args.frames}x{args.image}^2 video + 200x6 IMU, '
                  f'batch {B}, 1 GPU',
        'value': round(B * args.steps / el, 3), 'unit': 'clips/sec', 'frames_per_sec': round(frames * args.steps / el, 1),
        'n_gpus': 1, 'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': round(1000 * el / args.steps, 3),
        'dtype': 'bf16', 'data': f'synthetic (randn video/IMU resident in HBM, random-init {args.video_backbone})',
        'config': {'workload': f'CrossModalModel pretrain step, video_backbone={args.video_backbone}',
                   'global_batch': B, 'parallelism': 'dp1'},
        'model_gflop_per_frame_fwd': round(fwd / 1e9, 3), 'model_tflops': round(tf, 1),
        'mfma_frac': round(tf / PEAK_BF16_TFLOPS, 4), 'loss_after_warmup': first,
        'max_mem_gb': round(torch.cuda.max_memory_allocated() / 2 ** 30, 1)}))


if __name__ == '__main__':
    main()
