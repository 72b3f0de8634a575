"""How much of the bench step the IMU branch costs: step time with the IMU branch on its side stream (product),
on the main stream, and replaced by a zero-cost stub (a learnable (B, 128) feature; the video branch unchanged).
    python tools/debug/imu_cost.py [r3d_18]     (r3d_18: the config-2 step, R3D-18 at 16x112^2)"""
import os
import sys
import time
import warnings

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, 'crossmodal-imu-video-ood-har_amd'))
import torch  # noqa: E402

from cmhar.config import Config  # noqa: E402
from cmhar.losses import SigmoidContrastiveLoss  # noqa: E402
from cmhar.models import CrossModalModel  # noqa: E402
from cmhar.optim import FusedAdamW, clip_grad_norm_  # noqa: E402


def main():
    dev = torch.device('cuda')
    cfg = Config()
    cfg.model.allow_random_init = True
    r3d = 'r3d_18' in sys.argv[1:]
    S = 224
    if r3d:
        cfg.model.video_backbone = 'r3d_18'
        cfg.data.video_resize = (112, 112)
        S = 112
    torch.manual_seed(0)
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        model = CrossModalModel(cfg).to(dev).train()
    lf = SigmoidContrastiveLoss().to(dev)
    opt = FusedAdamW(model.parameters(), lr=1e-5, weight_decay=0.01,
                     shadow_sources=[] if r3d else [model.video_encoder.backbone])
    B = 32
    video = torch.randn(B, 16, 3, S, S, device=dev)
    imu = torch.randn(B, 6, 200, device=dev)
    params = list(model.parameters())
    stub = torch.nn.Parameter(torch.randn(B, 128, device=dev))
    real = model.imu_encoder.forward

    def step():
        a, b = model(imu, video)
        loss = lf(a, b)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        clip_grad_norm_(params, 1.0)
        opt.step()

    for name, side, use_stub in [('side stream', True, False), ('main stream', False, False), ('stub', True, True)]:
        model.overlap_imu = side
        model.imu_encoder.forward = (lambda x: (stub * 1.0, None)) if use_stub else real
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 10
        print(f'{name:12s} {dt * 1e3:7.2f} ms/step  {B / dt:7.1f} clips/s', flush=True)


if __name__ == '__main__':
    main()
