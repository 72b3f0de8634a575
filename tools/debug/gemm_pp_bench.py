"""Ping-pong GEMM (cmhar_gemm_pp) vs the 256² GEMM (cmhar_gemm_bf16): exactness on integer operands, then the
product GEMMs of one VideoMAE-B layer (B=32, 16x224²) with their real epilogues.  python tools/debug/gemm_pp_bench.py"""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..',
                                'crossmodal-imu-video-ood-har_amd'))
from cmhar import _lib as L  # noqa: E402
from cmhar import kernels as K  # noqa: E402

_PP = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'libablate_pp.so'))
_PP.cmhar_gemm_pp.argtypes = [C.c_int] * 5 + [C.c_void_p, C.c_long, C.c_void_p, C.c_long, C.c_void_p, C.c_long,
                                             C.POINTER(L.Epilogue), C.c_int, C.c_void_p, C.c_int, C.c_void_p]


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


def pp(layout, a, b, out, delay, splits=1, **kw):
    if layout == 0:
        M, Kd = a.shape; N = b.shape[0]
    elif layout == 1:
        M, Kd = a.shape; N = b.shape[1]
    else:
        Kd, M = a.shape; N = b.shape[1]
    epi = L.epilogue(kw.get('bias'), kw.get('residual'), kw.get('aux_in'), kw.get('aux_out'), None, 1,
                     kw.get('act', 0), 1.0, kw.get('beta', 0.0), 0.0, 0, kw.get('rowsum'), kw.get('rowsum_beta', 0.0))
    ws = K.workspace(splits * M * N + splits * M, out.device) if splits > 1 else None
    rc = _PP.cmhar_gemm_pp(layout, L.dtype_code(out.dtype), M, N, Kd, a.data_ptr(), a.stride(0), b.data_ptr(),
                               b.stride(0), out.data_ptr(), out.stride(0), C.byref(epi), splits, L.ptr(ws), delay,
                               L.stream(out.device))
    assert rc == 1, rc
    return out


def ints(shape, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(-3, 4, shape, generator=g).float()


def exactness():
    dev = 'cuda'
    for layout, (M, N, Kd) in [(0, (512, 384, 1024)), (1, (512, 384, 1024)), (2, (768, 512, 1024))]:
        if layout == 0:
            a, b = ints((M, Kd), 1), ints((N, Kd), 2); ref = a @ b.T
        elif layout == 1:
            a, b = ints((M, Kd), 1), ints((Kd, N), 2); ref = a @ b
        else:
            a, b = ints((Kd, M), 1), ints((Kd, N), 2); ref = a.T @ b
        a, b, ref = a.to(dev).bfloat16(), b.to(dev).bfloat16(), ref.to(dev)
        for splits in (1, 3):
            out = torch.empty(M, N, device=dev)
            rs = torch.empty(M, device=dev) if layout == 2 else None
            pp(layout, a, b, out, 0, splits=splits, rowsum=rs)
            ok = torch.equal(out, ref)
            if rs is not None:
                ok = ok and torch.equal(rs, a.float().sum(0))
            print(f'exact layout {layout} splits {splits}: {ok}', flush=True)


def main():
    exactness()
    dev = 'cuda'
    T, H, F = 50176, 768, 3072
    bf = torch.bfloat16
    r = lambda *s: torch.randn(*s, device=dev).to(bf)  # noqa: E731
    h, g, x = r(T, H), r(T, F), r(T, H)
    wqkv, wo, w1, w2 = r(3 * H, H), r(H, H), r(F, H), r(H, F)
    bqkv, bo, b1, b2 = (torch.randn(n, device=dev) for n in (3 * H, H, F, H))
    gp = r(T, F)
    dy, dF = r(T, H), r(T, F)
    outs = {n: torch.empty(T, n, device=dev, dtype=bf) for n in (H, 3 * H, F)}
    cases = [
        ('qkv fwd', 0, h, wqkv, 3 * H, dict(bias=bqkv)),
        ('out fwd +res', 0, h, wo, H, dict(bias=bo, residual=x)),
        ('fc1 fwd gelu2', 0, h, w1, F, dict(bias=b1, act=L.ACT_GELU_SAVEGRAD, aux_out=gp)),
        ('fc2 fwd +res', 0, g, w2, H, dict(bias=b2, residual=x)),
        ('fc2 dgrad *aux', 1, dy, w2, F, dict(act=L.ACT_MULAUX, aux_in=gp)),
        ('fc1 dgrad', 1, dF, w1, H, {}),
        ('out dgrad', 1, dy, wo, H, {}),
        ('qkv dgrad', 1, r(T, 3 * H), wqkv, H, {}),
    ]
    for name, layout, a, w, n, kw in cases:
        out = outs[n]
        Kd = a.shape[1]
        fl = 2 * T * n * Kd
        t_old = run(lambda: K.gemm(layout, a, w, out, **kw))
        ref = out.float().clone()
        res = [f'old {t_old * 1e3:6.1f}us {fl / t_old / 1e9:5.0f}TF']
        for delay in (0, Kd // 32 * 256, Kd // 32 * 512):
            t = run(lambda: pp(layout, a, w, out, delay, **kw))
            err = ((out.float() - ref).norm() / ref.norm()).item()
            res.append(f'pp[d={delay}] {t * 1e3:6.1f}us {fl / t / 1e9:5.0f}TF err {err:.1e}')
        print(f'{name:15s} ' + ' | '.join(res), flush=True)
    # weight gradients with bias row sums
    for name, n, k, a_ in (('fc1 wgrad', F, H, h), ('fc2 wgrad', H, F, g), ('qkv wgrad', 3 * H, H, h),
                           ('out wgrad', H, H, h)):
        d = r(T, n)
        dw = torch.empty(n, k, device=dev)
        db = torch.empty(n, device=dev)
        fl = 2 * T * n * k
        t_old = run(lambda: K.linear_wgrad(d, a_, out=dw, bias_out=db))
        ref = dw.clone()
        res = [f'old {t_old * 1e3:6.1f}us {fl / t_old / 1e9:5.0f}TF']
        tiles = (n // 256) * (k // 128)
        for splits in (max(1, 512 // tiles), max(1, 1024 // tiles)):
            t = run(lambda: pp(2, d, a_, dw, 0, splits=splits, rowsum=db))
            err = ((dw - ref).norm() / ref.norm()).item()
            res.append(f'pp[s={splits}] {t * 1e3:6.1f}us {fl / t / 1e9:5.0f}TF err {err:.1e}')
        print(f'{name:15s} ' + ' | '.join(res), flush=True)


if __name__ == '__main__':
    main()
