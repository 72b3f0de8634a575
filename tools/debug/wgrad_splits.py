"""Old 256² wgrad GEMM vs split count (B=32, 16x224² shapes).  python tools/debug/wgrad_splits.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..',
                                'crossmodal-imu-video-ood-har_amd'))
from cmhar import kernels as K  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_pp_bench import run  # noqa: E402


def main():
    dev = 'cuda'
    T = 50176
    for name, n, k in (('fc1', 3072, 768), ('fc2', 768, 3072), ('qkv', 2304, 768), ('out', 768, 768)):
        d = torch.randn(T, n, device=dev).bfloat16()
        x = torch.randn(T, k, device=dev).bfloat16()
        dw = torch.empty(n, k, device=dev)
        fl = 2 * T * n * k
        res = []
        for s in (1, 4, 7, 8, 12, 16, 24):
            t = run(lambda: K.gemm(2, d, x, dw, splits=s))
            res.append(f's{s} {t * 1e3:6.1f}us {fl / t / 1e9:5.0f}TF')
        print(name, ' | '.join(res), flush=True)


if __name__ == '__main__':
    main()
