"""A/B two (or more) builds of libcmhar.so on every GEMM shape of the VideoMAE-B step in ONE process (interleaved rounds,
median per variant), so device/clock differences between boxes do not enter the comparison.

    python tools/debug/gemm_ab.py libA.so libB.so [libC.so ...] [--rounds R]
"""
import ctypes as C
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..',
                                'crossmodal-imu-video-ood-har_amd'))
from cmhar import _lib  # noqa: E402
from cmhar import kernels as K  # noqa: E402


def load(path):
    L = C.CDLL(os.path.abspath(path))
    for name, (res, args) in _lib._SIGS.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    return L


def timed(fn, reps=10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    args = sys.argv[1:]
    rounds = 7
    if '--rounds' in args:
        i = args.index('--rounds')
        rounds = int(args[i + 1])
        del args[i:i + 2]
    libs = [load(a) for a in args]
    nv = len(libs)
    T = 50176
    lin = [('qkv', 2304, 768), ('out', 768, 768), ('fc1', 3072, 768), ('fc2', 768, 3072), ('embed', 768, 1536)]
    tot = [0.0] * nv
    for name, n_out, n_in in lin:
        x = torch.randn(T, n_in, device='cuda').bfloat16()
        w = torch.randn(n_out, n_in, device='cuda').bfloat16()
        dy = torch.randn(T, n_out, device='cuda').bfloat16()
        y = torch.empty(T, n_out, device='cuda', dtype=torch.bfloat16)
        dx = torch.empty(T, n_in, device='cuda', dtype=torch.bfloat16)
        dw = torch.empty(n_out, n_in, device='cuda', dtype=torch.float32)
        fl = 2 * T * n_out * n_in
        cases = [('fwd', lambda: K.gemm(0, x, w, y)), ('dgrad', lambda: K.gemm(1, dy, w, dx)),
                 ('wgrad', lambda: K.gemm(2, dy, x, dw))]
        for tag, fn in cases:
            if name == 'embed' and tag == 'dgrad':
                continue
            outs = []
            for v in range(nv):
                _lib._lib = libs[v]
                for _ in range(3):
                    fn()
                torch.cuda.synchronize()
                outs.append(y.clone() if tag == 'fwd' else dx.clone() if tag == 'dgrad' else dw.clone())
            same = all(torch.equal(outs[0], o) for o in outs[1:])
            ts = [[] for _ in range(nv)]
            for _ in range(rounds):
                for v in range(nv):
                    _lib._lib = libs[v]
                    ts[v].append(timed(fn))
            med = [statistics.median(t) for t in ts]
            mult = 1 if name == 'embed' else 12
            for v in range(nv):
                tot[v] += med[v] * mult
            cols = ' | '.join(f'{chr(65 + v)} {med[v] * 1e3:7.1f} us {fl / med[v] / 1e9:5.0f} TF' for v in range(nv))
            print(f'{name:6s} {tag:6s} {cols} | bitwise-equal={same}', flush=True)
    print('per-step GEMM total: ' + '  '.join(f'{chr(65 + v)} {tot[v]:.2f} ms' for v in range(nv)))


if __name__ == '__main__':
    main()
