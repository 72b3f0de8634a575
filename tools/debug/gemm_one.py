"""Run one product GEMM shape repeatedly (for rocprofv3 counter passes).
python tools/debug/gemm_one.py NAME LAYOUT [reps]   NAME in qkv/out/fc1/fc2/embed, LAYOUT fwd/dgrad/wgrad"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..',
                                'crossmodal-imu-video-ood-har_amd'))
from cmhar import kernels as K  # noqa: E402

SHAPES = {'qkv': (2304, 768), 'out': (768, 768), 'fc1': (3072, 768), 'fc2': (768, 3072), 'embed': (768, 1536)}


def main():
    name, lay = sys.argv[1], sys.argv[2]
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    T = 50176
    n_out, n_in = SHAPES[name]
    g = torch.Generator(device='cuda').manual_seed(0)
    x = torch.randn(T, n_in, device='cuda', generator=g).bfloat16()
    w = torch.randn(n_out, n_in, device='cuda', generator=g).bfloat16()
    dy = torch.randn(T, n_out, device='cuda', generator=g).bfloat16()
    if lay == 'fwd':
        y = torch.empty(T, n_out, device='cuda', dtype=torch.bfloat16)
        fn = lambda: K.gemm(0, x, w, y)   # noqa: E731
    elif lay == 'dgrad':
        dx = torch.empty(T, n_in, device='cuda', dtype=torch.bfloat16)
        fn = lambda: K.gemm(1, dy, w, dx)   # noqa: E731
    else:
        dw = torch.empty(n_out, n_in, device='cuda', dtype=torch.float32)
        fn = lambda: K.gemm(2, dy, x, dw)   # noqa: E731
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(f'{name} {lay}: {ms * 1e3:.1f} us/call (incl. reduce), {2 * T * n_out * n_in / ms / 1e9:.0f} TF')


if __name__ == '__main__':
    main()
