"""One fp32 VideoMAE GEMM shape on the f32 MFMA kernel, repeated (for rocprofv3 --pmc passes / kernel traces).
    python tools/debug/f32_gemm_bench.py [layout M N K] [--reps R]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..',
                                'crossmodal-imu-video-ood-har_amd'))
from cmhar import kernels as K  # noqa: E402


def main():
    a = [x for x in sys.argv[1:] if not x.startswith('--')]
    reps = int(sys.argv[sys.argv.index('--reps') + 1]) if '--reps' in sys.argv else 20
    lay, M, N, Kd = (int(x) for x in a[:4]) if len(a) >= 4 else (0, 12544, 3072, 768)
    g = torch.Generator(device='cuda').manual_seed(0)
    A = torch.randn((M, Kd) if lay < 2 else (Kd, M), device='cuda', generator=g)
    B = torch.randn((N, Kd) if lay == 0 else (Kd, N), device='cuda', generator=g)
    C = torch.empty(M, N, device='cuda')
    for _ in range(reps):
        K.gemm(lay, A, B, C)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        K.gemm(lay, A, B, C)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(f'layout {lay} {M}x{N}x{Kd}: {ms * 1e3:.1f} us  {2 * M * N * Kd / ms / 1e9:.1f} TF/s')


if __name__ == '__main__':
    main()
