"""Square bf16 GEMMs (4096³, 8192³) through the product library, every layout, random [-1, 1) operands: how the
product kernels compare with the guide's 256² 8-phase template figures (1320-1340 TF @4k, ~1470 @8k, random).
python tools/debug/gemm_square.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..',
                                'crossmodal-imu-video-ood-har_amd'))
from cmhar import _lib  # noqa: E402
from cmhar import kernels as K  # noqa: E402


def bench(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    for n in (4096, 8192):
        g = torch.Generator(device='cuda').manual_seed(0)
        a = (torch.rand(n, n, device='cuda', generator=g) * 2 - 1).bfloat16()
        b = (torch.rand(n, n, device='cuda', generator=g) * 2 - 1).bfloat16()
        for lay, name in ((0, 'fwd NT'), (1, 'dgrad NN'), (2, 'wgrad TN')):
            for odt in (torch.bfloat16, torch.float32):
                if lay == 2 and odt == torch.bfloat16:
                    continue
                c = torch.empty(n, n, device='cuda', dtype=odt)
                plan = _lib.lib().cmhar_gemm_bf16_plan(lay, n, n, n, 1, 0, 0)
                ms = bench(lambda: K.gemm(lay, a, b, c, splits=1))
                print(f'{n}^3 {name:9s} out={str(odt)[6:]:9s} plan={plan}: {ms * 1e3:8.1f} us  '
                      f'{2 * n ** 3 / ms / 1e9:6.0f} TF', flush=True)
        ref = bench(lambda: torch.matmul(a, b.T))
        print(f'{n}^3 torch.matmul (hipBLASLt) NT bf16: {ref * 1e3:8.1f} us  {2 * n ** 3 / ref / 1e9:6.0f} TF', flush=True)


if __name__ == '__main__':
    main()
