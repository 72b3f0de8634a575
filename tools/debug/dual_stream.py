"""Would two half-batch VideoMAE-B backbone passes on two HIP streams beat one full-batch pass?  (micro-batch
interleaving experiment).  Times fwd+bwd of: one B=32 pass; two B=16 passes back to back on one stream; two B=16
passes on two streams (forward of each half on its own stream; autograd runs each backward node on its forward's
stream).  python tools/debug/dual_stream.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..',
                                'crossmodal-imu-video-ood-har_amd'))
from cmhar.config import Config  # noqa: E402
from cmhar.models import CrossModalModel  # noqa: E402
from cmhar.videomae import run_backbone  # noqa: E402


def main():
    dev = torch.device('cuda')
    cfg = Config()
    cfg.model.allow_random_init = True
    cfg.data.video_frames_per_window = 16
    cfg.data.video_resize = (224, 224)
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        model = CrossModalModel(cfg).to(dev).train()
    bb = model.video_encoder.backbone
    g = torch.Generator(device=dev).manual_seed(0)
    video = torch.randn(32, 16, 3, 224, 224, device=dev, generator=g)
    halves = [video[:16].contiguous(), video[16:].contiguous()]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def full():
        out = run_backbone(bb, video, True)
        out.float().sum().backward()

    def seq():
        outs = [run_backbone(bb, h, True) for h in halves]
        torch.autograd.backward([o.float().sum() for o in outs])

    def dual():
        cur = torch.cuda.current_stream()
        outs = []
        for h, s in zip(halves, (s1, s2)):
            s.wait_stream(cur)
            with torch.cuda.stream(s):
                outs.append(run_backbone(bb, h, True).float().sum())
        for s in (s1, s2):
            cur.wait_stream(s)
        torch.autograd.backward(outs)

    for name, fn in (('full B=32', full), ('2x B=16 one stream', seq), ('2x B=16 two streams', dual),
                     ('full B=32', full), ('2x B=16 two streams', dual)):
        for _ in range(3):
            fn()
            bb.zero_grad(set_to_none=True)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(10):
            fn()
            bb.zero_grad(set_to_none=True)
        torch.cuda.synchronize()
        print(f'{name:24s} {(time.perf_counter() - t) / 10 * 1e3:7.2f} ms', flush=True)


if __name__ == '__main__':
    main()
