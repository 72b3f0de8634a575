"""Time the fp32 GEMMs of the projection heads and the video projection (M = batch rows) on the product entry
(cmhar.kernels.gemm), per layout: python tools/debug/head_gemms.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..',
                                'crossmodal-imu-video-ood-har_amd'))
from cmhar import kernels as K  # noqa: E402


def timed(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    B = 32
    tot = 0.0
    for name, n_in, n_out in [('video_projection', 768, 768), ('video_head.0', 768, 512), ('video_head.3', 512, 256),
                              ('imu_head.0', 128, 512), ('imu_head.3', 512, 256)]:
        x = torch.randn(B, n_in, device='cuda')
        w = torch.randn(n_out, n_in, device='cuda')
        dy = torch.randn(B, n_out, device='cuda')
        y = torch.empty(B, n_out, device='cuda')
        dx = torch.empty(B, n_in, device='cuda')
        dw = torch.empty(n_out, n_in, device='cuda')
        for tag, fn in (('fwd', lambda: K.gemm(0, x, w, y)), ('dgrad', lambda: K.gemm(1, dy, w, dx)),
                        ('wgrad', lambda: K.gemm(2, dy, x, dw))):
            t = timed(fn)
            tot += t
            print(f'{name:18s} {tag:6s} {t:8.1f} us', flush=True)
    print(f'total {tot:.1f} us')


if __name__ == '__main__':
    main()
