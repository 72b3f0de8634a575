"""A/B two (or more) builds of libcmhar.so on the VideoMAE-B LayerNorm forward (M = 50 176 tokens, N = 768, bf16) in
ONE process: interleaved rounds, median per variant, outputs (y, mean, rstd) compared bitwise with the first.

    python tools/debug/ln_ab.py libA.so libB.so [...] [--rounds R]
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..',
                                'crossmodal-imu-video-ood-har_amd'))
from cmhar import _lib  # noqa: E402
from gemm_ab import load, timed  # noqa: E402


def main():
    args = sys.argv[1:]
    rounds = 9
    if '--rounds' in args:
        i = args.index('--rounds')
        rounds = int(args[i + 1])
        del args[i:i + 2]
    libs = [load(a) for a in args]
    M, N = 50176, 768
    g = torch.Generator(device='cuda').manual_seed(0)
    x = (torch.randn(M, N, device='cuda', generator=g) * 2 + 0.5).bfloat16()
    gamma = torch.rand(N, device='cuda', generator=g) + 0.5
    beta = torch.randn(N, device='cuda', generator=g)
    st = torch.cuda.current_stream().cuda_stream
    outs = []
    for L in libs:
        y = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)
        mu = torch.empty(M, device='cuda')
        rs = torch.empty(M, device='cuda')
        outs.append((y, mu, rs))

    def run(k):
        y, mu, rs = outs[k]
        rc = libs[k].cmhar_layernorm_fwd(_lib.BF16, M, N, x.data_ptr(), N, None, 0, 0.0, 0, None, 0, y.data_ptr(), N,
                                         gamma.data_ptr(), beta.data_ptr(), mu.data_ptr(), rs.data_ptr(), 1e-6, st)
        assert rc == 0
    times = [[] for _ in libs]
    for k in range(len(libs)):
        run(k)
    torch.cuda.synchronize()
    for _ in range(rounds):
        for k in range(len(libs)):
            times[k].append(timed(lambda: run(k), reps=20) * 1e3)
    same = [all(torch.equal(a.view(torch.int16) if a.dtype == torch.bfloat16 else a, b.view(torch.int16)
                            if b.dtype == torch.bfloat16 else b) for a, b in zip(outs[0], o)) for o in outs[1:]]
    med = [statistics.median(t) for t in times]
    gbs = [(2 * M * N * 2) / (m * 1e-6) / 1e9 for m in med]
    print('ln_fwd ' + ' | '.join(f'{chr(65 + k)} {m:7.1f} us {b:6.0f} GB/s' for k, (m, b) in enumerate(zip(med, gbs)))
          + f' | bitwise-equal-to-A={same}')

    # backward (dy, h, residual gradient in; dh out; dγ / dβ through the partial-row reduction)
    dy = torch.randn(M, N, device='cuda', generator=g).bfloat16()
    dres = torch.randn(M, N, device='cuda', generator=g).bfloat16()
    mu, rs = outs[0][1], outs[0][2]
    nws = int(libs[0].cmhar_layernorm_bwd_ws(M, N))
    bouts = []
    for L in libs:
        bouts.append((torch.empty(M, N, device='cuda', dtype=torch.bfloat16), torch.empty(N, device='cuda'),
                      torch.empty(N, device='cuda'), torch.empty(nws, device='cuda')))

    def runb(k):
        dh, dg, db, ws = bouts[k]
        rc = libs[k].cmhar_layernorm_bwd(_lib.BF16, M, N, dy.data_ptr(), N, x.data_ptr(), N, gamma.data_ptr(),
                                         mu.data_ptr(), rs.data_ptr(), dres.data_ptr(), N, dh.data_ptr(), N, None, 0,
                                         0.0, 0, dg.data_ptr(), db.data_ptr(), 0.0, ws.data_ptr(), st)
        assert rc == 0
    bt = [[] for _ in libs]
    for k in range(len(libs)):
        runb(k)
    torch.cuda.synchronize()
    for _ in range(rounds):
        for k in range(len(libs)):
            bt[k].append(timed(lambda: runb(k), reps=20) * 1e3)
    bmed = [statistics.median(t) for t in bt]
    dh_same = [torch.equal(bouts[0][0].view(torch.int16), o[0].view(torch.int16)) for o in bouts[1:]]
    rel = [max(float((o[i] - bouts[0][i]).abs().max() / bouts[0][i].abs().max()) for i in (1, 2)) for o in bouts[1:]]
    print('ln_bwd ' + ' | '.join(f'{chr(65 + k)} {m:7.1f} us' for k, m in enumerate(bmed))
          + f' | dh bitwise-equal-to-A={dh_same} | dgamma/dbeta max rel diff to A={rel}')


if __name__ == '__main__':
    main()
