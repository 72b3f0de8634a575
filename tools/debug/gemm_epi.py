"""Time the product GEMMs of one VideoMAE-B layer (B=32, 16x224²) WITH their fused epilogues, in isolation, against
the same GEMM with no epilogue.  python tools/debug/gemm_epi.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..',
                                'crossmodal-imu-video-ood-har_amd'))
from cmhar import _lib as L  # noqa: E402
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
    T, H, F = 50176, 768, 3072
    bf = torch.bfloat16
    r = lambda *s: torch.randn(*s, device=dev).to(bf)  # noqa: E731
    x, h, g, pre = r(T, H), r(T, H), r(T, F), r(T, F)
    wqkv, wo, w1, w2 = r(3 * H, H), r(H, H), r(F, H), r(H, F)
    bqkv, bo, b1, b2 = (torch.randn(n, device=dev) for n in (3 * H, H, F, H))
    dy = r(T, H)
    cases = [
        ('qkv fwd +bias', lambda: K.linear(h, wqkv, bqkv), lambda: K.linear(h, wqkv), 3 * H, H),
        ('out fwd +bias+res', lambda: K.linear(h, wo, bo, residual=x), lambda: K.linear(h, wo), H, H),
        ('fc1 fwd +bias+gelu+aux', lambda: K.linear(h, w1, b1, act=L.ACT_GELU, aux_out=pre),
         lambda: K.linear(h, w1), F, H),
        ('fc2 fwd +bias+res', lambda: K.linear(g, w2, b2, residual=x), lambda: K.linear(g, w2), H, F),
        ('fc2 dgrad +dgelu', lambda: K.linear_dgrad(dy, w2, act=L.ACT_DGELU, aux_in=pre),
         lambda: K.linear_dgrad(dy, w2), F, H),
        ('fc1 fwd +bias+gelu+gelu\'', lambda: K.linear(h, w1, b1, act=L.ACT_GELU_SAVEGRAD, aux_out=pre),
         lambda: K.linear(h, w1), F, H),
        ('fc2 dgrad *aux', lambda: K.linear_dgrad(dy, w2, act=L.ACT_MULAUX, aux_in=pre),
         lambda: K.linear_dgrad(dy, w2), F, H),
    ]
    # weight gradients with / without the fused bias row sums
    for name, n, k, a_ in (('fc1', F, H, h), ('fc2', H, F, g), ('qkv', 3 * H, H, h)):
        d = r(T, n)
        db = torch.empty(n, device=dev)
        a = run(lambda: K.linear_wgrad(d, a_, bias_out=db))
        b = run(lambda: K.linear_wgrad(d, a_))
        c = run(lambda: K.colsum(d, db))
        fl = 2 * T * n * k
        print(f'{name} wgrad+bias {a * 1e3:7.1f} us | wgrad {b * 1e3:7.1f} us {fl / b / 1e9:5.0f} TF | '
              f'separate colsum {c * 1e3:6.1f} us', flush=True)
    for name, epi, plain, n, k in cases:
        a, b = run(epi), run(plain)
        fl = 2 * T * n * k
        print(f'{name:26s} epi {a * 1e3:7.1f} us {fl / a / 1e9:5.0f} TF | plain {b * 1e3:7.1f} us {fl / b / 1e9:5.0f} TF'
              f' | epilogue cost {100 * (a / b - 1):5.1f} %', flush=True)


if __name__ == '__main__':
    main()
