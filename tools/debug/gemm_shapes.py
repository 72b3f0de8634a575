"""Time the product GEMM entry (cmhar.kernels.gemm) on every GEMM shape of the VideoMAE-B step at B=32, 16x224²,
against torch.matmul (hipBLASLt).  python tools/debug/gemm_shapes.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..',
                                'crossmodal-imu-video-ood-har_amd'))
from cmhar import kernels as K  # noqa: E402


def run(fn, reps=20):
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
    dev = 'cuda'
    T = 50176
    lin = [('qkv', 2304, 768), ('out', 768, 768), ('fc1', 3072, 768), ('fc2', 768, 3072), ('embed', 768, 1536)]
    tot_ours = tot_ref = 0.0
    for name, n_out, n_in in lin:
        x = torch.randn(T, n_in, device=dev).bfloat16()
        w = torch.randn(n_out, n_in, device=dev).bfloat16()
        dy = torch.randn(T, n_out, device=dev).bfloat16()
        y = torch.empty(T, n_out, device=dev, dtype=torch.bfloat16)
        dx = torch.empty(T, n_in, device=dev, dtype=torch.bfloat16)
        dw = torch.empty(n_out, n_in, device=dev, dtype=torch.float32)
        fl = 2 * T * n_out * n_in
        cases = [('fwd', lambda: K.gemm(0, x, w, y), lambda: torch.matmul(x, w.T)),
                 ('dgrad', lambda: K.gemm(1, dy, w, dx), lambda: torch.matmul(dy, w)),
                 ('wgrad', lambda: K.gemm(2, dy, x, dw), lambda: torch.matmul(dy.T, x, out=None).float())]
        for tag, ours, ref in cases:
            if name == 'embed' and tag == 'dgrad':
                continue
            a, b = run(ours), run(ref)
            mult = 1 if name == 'embed' else 12
            tot_ours += a * mult
            tot_ref += b * mult
            print(f'{name:6s} {tag:6s} ours {a * 1e3:8.1f} us {fl / a / 1e9:6.0f} TF | torch {b * 1e3:8.1f} us '
                  f'{fl / b / 1e9:6.0f} TF', flush=True)
    print(f'per-step GEMM total: ours {tot_ours:.2f} ms  torch {tot_ref:.2f} ms')


if __name__ == '__main__':
    main()
