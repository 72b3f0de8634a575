"""Ablation of the ping-pong GEMM (layout 0): 0 full, 1 no epilogue, 3 no DMA; and a stamped run (mode 4) that
shows whether a CU's two workgroups really alternate K loop and epilogue."""
import ctypes as C
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gemm_pp_bench import run  # noqa: E402

lib = C.CDLL(os.path.join(HERE, 'libablate_pp.so'))
vp, i32, i64 = C.c_void_p, C.c_int, C.c_long
lib.ablate_pp.argtypes = [i32, i32, i32, i32, i32, vp, i64, vp, i64, vp, i64, vp, vp, i32, vp]


def stamps_report(st, G=512):
    s = st.view(G, 64, 3).cpu().numpy().astype(np.int64)
    valid = s[:, :, 2] > 0
    t0 = s[:, :, 0][valid].min()
    main = (s[:, :, 1] - s[:, :, 0])[valid]
    epi = (s[:, :, 2] - s[:, :, 1])[valid]
    print(f'   units {valid.sum()}  K-loop cycles median {np.median(main):.0f}  epilogue median {np.median(epi):.0f}'
          f'  span {(s[:, :, 2][valid].max() - t0)}')
    # overlap of the partner's epilogue with my K loop, CU pairs (b, b+256)
    fr = []
    for b in range(256):
        a_ep = [(s[b, u, 1], s[b, u, 2]) for u in range(64) if s[b, u, 2] > 0]
        b_ml = [(s[b + 256, u, 0], s[b + 256, u, 1]) for u in range(64) if s[b + 256, u, 2] > 0]
        tot = sum(e - s_ for s_, e in a_ep)
        ov = 0
        for s1, e1 in a_ep:
            for s2, e2 in b_ml:
                ov += max(0, min(e1, e2) - max(s1, s2))
        if tot:
            fr.append(ov / tot)
    print(f'   fraction of slot-0 epilogue time overlapped by the partner K loop: mean {np.mean(fr):.2f}')
    first = s[:, 0, 0] - t0
    print(f'   first-unit start offset slot0 median {np.median(first[:256]):.0f} slot1 {np.median(first[256:]):.0f}')


def main():
    dev = 'cuda'
    T = 50176
    bf = torch.bfloat16
    st = torch.cuda.current_stream().cuda_stream
    stamps = torch.zeros(512 * 64 * 3, dtype=torch.int64, device=dev)
    for name, N, Kd, act in (('qkv', 2304, 768, 0), ('fc1', 3072, 768, 5), ('fc2', 768, 3072, 0)):
        a = torch.randn(T, Kd, device=dev).to(bf)
        w = torch.randn(N, Kd, device=dev).to(bf)
        out = torch.empty(T, N, device=dev, dtype=bf)
        aux = torch.empty(T, N, device=dev, dtype=bf)
        fl = 2 * T * N * Kd
        res = []
        for mode in (0, 1, 3):
            for delay in ((0, Kd * 16) if mode == 0 else (0,)):
                t = run(lambda: lib.ablate_pp(mode, act, T, N, Kd, a.data_ptr(), a.stride(0), w.data_ptr(),
                                              w.stride(0), out.data_ptr(), out.stride(0), aux.data_ptr(),
                                              stamps.data_ptr(), delay, st))
                res.append(f'm{mode}d{delay} {t * 1e3:6.1f}us {fl / t / 1e9:5.0f}TF')
        print(name, ' | '.join(res), flush=True)
        for delay in (0, Kd * 16):
            stamps.zero_()
            lib.ablate_pp(4, act, T, N, Kd, a.data_ptr(), a.stride(0), w.data_ptr(), w.stride(0), out.data_ptr(),
                          out.stride(0), aux.data_ptr(), stamps.data_ptr(), delay, st)
            torch.cuda.synchronize()
            print(f'  stamped, delay {delay}:')
            stamps_report(stamps)


if __name__ == '__main__':
    main()
