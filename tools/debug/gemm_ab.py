"""A/B two (or more) builds of libcmhar.so on every GEMM shape of the VideoMAE-B step in ONE process (interleaved rounds,
median per variant), so device/clock differences between boxes do not enter the comparison.

    python tools/debug/gemm_ab.py libA.so libB.so [libC.so ...] [--rounds R] [--dtype bf16|fp32] [--tokens T]
              [--torch]     (--torch: also time torch.matmul on the same operands, as variant 'T')
              [--epi]       (--epi: the bench step's epilogues — QKV bias + key colscale, out-proj / FC2 bias +
                             residual, FC1 bias + GELU with GELU' saved, FC2 dgrad × GELU'; bf16 only)
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
        if not hasattr(L, name):   # an older build without this entry point
            continue
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
    dt, T, with_torch = torch.bfloat16, 50176, False
    if '--dtype' in args:
        i = args.index('--dtype')
        dt = {'bf16': torch.bfloat16, 'fp32': torch.float32}[args[i + 1]]
        del args[i:i + 2]
    if '--tokens' in args:
        i = args.index('--tokens')
        T = int(args[i + 1])
        del args[i:i + 2]
    if '--torch' in args:
        args.remove('--torch')
        with_torch = True
    epi = '--epi' in args
    if epi:
        args.remove('--epi')
    libs = [load(a) for a in args]
    if with_torch:
        libs.append(None)
    nv = len(libs)
    lin = [('qkv', 2304, 768), ('out', 768, 768), ('fc1', 3072, 768), ('fc2', 768, 3072), ('embed', 768, 1536)]
    tot = [0.0] * nv
    for name, n_out, n_in in lin:
        x = torch.randn(T, n_in, device='cuda').to(dt)
        w = torch.randn(n_out, n_in, device='cuda').to(dt)
        dy = torch.randn(T, n_out, device='cuda').to(dt)
        y = torch.empty(T, n_out, device='cuda', dtype=dt)
        dx = torch.empty(T, n_in, device='cuda', dtype=dt)
        dw = torch.empty(n_out, n_in, device='cuda', dtype=torch.float32)
        fl = 2 * T * n_out * n_in
        fkw, dkw = {}, {}
        if epi:
            b = torch.randn(n_out, device='cuda') * 0.1
            fkw = {'bias': b}
            if name == 'qkv':
                fkw['colscale'] = (768, 1536, 0.125 * K.LOG2E)
            if name in ('out', 'fc2'):
                fkw['residual'] = torch.randn(T, n_out, device='cuda').to(dt)
            if name == 'fc1':
                fkw['act'] = _lib.ACT_GELU_SAVEGRAD
                fkw['aux_out'] = torch.empty(T, n_out, device='cuda', dtype=dt)
            if name == 'fc2':
                dkw = {'act': _lib.ACT_MULAUX, 'aux_in': torch.rand(T, n_in, device='cuda').to(dt)}
        cases = [('fwd', lambda: K.gemm(0, x, w, y, **fkw), lambda: torch.matmul(x, w.t(), out=y)),
                 ('dgrad', lambda: K.gemm(1, dy, w, dx, **dkw), lambda: torch.matmul(dy, w, out=dx)),
                 ('wgrad', lambda: K.gemm(2, dy, x, dw), lambda: torch.matmul(dy.t(), x, out=dw) if dt == torch.float32
                  else dw.copy_(dy.t() @ x))]
        if epi and name == 'fc2':   # the step's FC2 input gradient: layout 0 over the transposed weight copy
            wt = w.t().contiguous()
            cases.append(('dgradT', lambda: K.gemm(0, dy, wt, dx, **dkw), lambda: torch.matmul(dy, w, out=dx)))
        for tag, fn0, tfn in cases:
            if name == 'embed' and tag == 'dgrad':
                continue
            outs = []

            def fn_of(v):
                return tfn if libs[v] is None else fn0
            for v in range(nv):
                _lib._lib = libs[v]
                fn = fn_of(v)
                for _ in range(3):
                    fn()
                torch.cuda.synchronize()
                outs.append(y.clone() if tag == 'fwd' else dx.clone() if tag.startswith('dgrad') else dw.clone())
            same = all(torch.equal(outs[0], o) for o, lb in zip(outs[1:], libs[1:]) if lb is not None)
            ts = [[] for _ in range(nv)]
            for _ in range(rounds):
                for v in range(nv):
                    _lib._lib = libs[v]
                    ts[v].append(timed(fn_of(v)))
            med = [statistics.median(t) for t in ts]
            mult = 1 if name == 'embed' else 0 if tag == 'dgradT' else 12
            for v in range(nv):
                tot[v] += med[v] * mult
            cols = ' | '.join(f'{"T" if libs[v] is None else chr(65 + v)} {med[v] * 1e3:7.1f} us {fl / med[v] / 1e9:5.0f} TF' for v in range(nv))
            print(f'{name:6s} {tag:6s} {cols} | bitwise-equal={same}', flush=True)
    print('per-step GEMM total: ' + '  '.join(f'{chr(65 + v)} {tot[v]:.2f} ms' for v in range(nv)))


if __name__ == '__main__':
    main()
