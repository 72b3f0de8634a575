"""A/B two (or more) builds of libcmhar.so on the bf16 flash attention kernels at the VideoMAE-B step shape
(B=32, H=12, L=1568, D=64) in ONE process: interleaved rounds, median per variant, outputs compared bitwise.

    python tools/debug/attn_ab.py libA.so libB.so [...] [--rounds R]
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..',
                                'crossmodal-imu-video-ood-har_amd'))
from cmhar import _lib  # noqa: E402
from cmhar import kernels as K  # noqa: E402
from gemm_ab import load, timed  # noqa: E402


def main():
    args = sys.argv[1:]
    rounds = 7
    prescaled = '--prescaled' in args      # the bf16 training path's scale (c = scale·log2e = 1, pre-scaled keys)
    if prescaled:
        args.remove('--prescaled')
    if '--rounds' in args:
        i = args.index('--rounds')
        rounds = int(args[i + 1])
        del args[i:i + 2]
    libs = [load(a) for a in args]
    nv = len(libs)
    B, H, L, D = 32, 12, 1568, 64
    g = torch.Generator(device='cuda').manual_seed(0)
    qkv = torch.randn(B * L, 3 * H * D, device='cuda', generator=g).bfloat16()
    q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
    o = torch.empty(B * L, H * D, device='cuda', dtype=torch.bfloat16)
    lse = torch.empty(B * H * L, device='cuda')
    do = torch.randn(B * L, H * D, device='cuda', generator=g).bfloat16()
    dqkv = torch.empty_like(qkv)
    dq, dk, dv = dqkv[:, :H * D], dqkv[:, H * D:2 * H * D], dqkv[:, 2 * H * D:]
    sc = 1.0 / K.LOG2E if prescaled else D ** -0.5
    fl = 4 * B * H * L * L * D
    cases = [('fwd', 1.0, lambda: K.attention_fwd(q, k, v, o, lse, B=B, H=H, Lq=L, Lk=L, D=D, scale=sc), lambda: o),
             ('bwd', 2.5, (lambda: K.attention_bwd_prescaled(q, k, v, o, do, lse, dq, dk, dv, B=B, H=H, Lq=L, Lk=L,
                                                             D=D, scale=D ** -0.5)) if prescaled else
              (lambda: K.attention_bwd(q, k, v, o, do, lse, dq, dk, dv, B=B, H=H, Lq=L, Lk=L, D=D, scale=sc)),
              lambda: dqkv)]
    _lib._lib = libs[0]
    K.attention_fwd(q, k, v, o, lse, B=B, H=H, Lq=L, Lk=L, D=D, scale=sc)
    for tag, mult, fn, res in cases:
        outs = []
        for lb in libs:
            _lib._lib = lb
            if tag == 'bwd':   # every variant's backward from the same forward output
                _lib._lib = libs[0]
                K.attention_fwd(q, k, v, o, lse, B=B, H=H, Lq=L, Lk=L, D=D, scale=sc)
                _lib._lib = lb
            fn()
            torch.cuda.synchronize()
            outs.append(res().clone())
        same = [torch.equal(outs[0], x) for x in outs[1:]]
        diff = [((outs[0].float() - x.float()).norm() / outs[0].float().norm()).item() for x in outs[1:]]
        ts = [[] for _ in range(nv)]
        for _ in range(rounds):
            for vi in range(nv):
                _lib._lib = libs[vi]
                ts[vi].append(timed(fn, 5))
        med = [statistics.median(t) for t in ts]
        cols = ' | '.join(f'{chr(65 + vi)} {med[vi] * 1e3:7.1f} us {mult * fl / med[vi] / 1e9:5.0f} TF'
                          for vi in range(nv))
        print(f'{tag} {cols} | bitwise-equal-to-A={same} rel-diff-to-A={["%.2e" % d for d in diff]}', flush=True)


if __name__ == '__main__':
    main()
