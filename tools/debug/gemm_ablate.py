"""Time GEMM ablation variants on the GPU (HIP events, same stream).  python tools/debug/gemm_ablate.py"""
import ctypes as C
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = C.CDLL(os.path.join(HERE, 'libablate.so'))
vp, i32, i64 = C.c_void_p, C.c_int, C.c_long
lib.ablate_gemm256.argtypes = [i32, i32, i32, i32, i32, vp, i64, vp, i64, vp, i64, vp]
lib.ablate_gemm128.argtypes = [i32, i32, i32, i32, vp, i64, vp, i64, vp, i64, vp]
lib.ablate_gemm256p.argtypes = [i32, i32, i32, i32, vp, i64, vp, i64, vp, i64, vp]


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
    st = torch.cuda.current_stream().cuda_stream
    shapes = [('qkv', 0, 50176, 2304, 768), ('fc1', 0, 50176, 3072, 768), ('fc2', 0, 50176, 768, 3072),
              ('dgrad_fc1', 1, 50176, 768, 3072), ('wgrad_fc1', 2, 3072, 768, 50176)]
    only = sys.argv[1].split(',') if len(sys.argv) > 1 else None
    modes = [int(x) for x in sys.argv[2].split(',')] if len(sys.argv) > 2 else [0, 3, 4, 5, 6]
    tags = {0: 'full', 1: 'dma_only', 2: 'mfma_only', 3: 'epi_only', 4: 'no_epi', 5: 'stage_only', 6: 'plain_store',
            7: 'no_dma', 8: 'spread_no_epi', 9: 'A3_full', 10: 'A3_no_epi'}
    for name, layout, M, N, K in shapes:
        if only and name not in only:
            continue
        if layout == 0:
            a = torch.randn(M, K, device=dev).bfloat16(); b = torch.randn(N, K, device=dev).bfloat16()
        elif layout == 1:
            a = torch.randn(M, K, device=dev).bfloat16(); b = torch.randn(K, N, device=dev).bfloat16()
        else:
            a = torch.randn(K, M, device=dev).bfloat16(); b = torch.randn(K, N, device=dev).bfloat16()
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        fl = 2 * M * N * K
        res = {}
        for mode, tag in ((m, tags[m]) for m in modes):
            ms = run(lambda: lib.ablate_gemm256(mode, layout, M, N, K, a.data_ptr(), a.stride(0), b.data_ptr(),
                                                b.stride(0), c.data_ptr(), c.stride(0), st))
            res[tag] = (ms, fl / ms / 1e9)
        ms = run(lambda: lib.ablate_gemm256p(layout, M, N, K, a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0),
                                             c.data_ptr(), c.stride(0), st))
        res['gemm256p'] = (ms, fl / ms / 1e9)
        ms = run(lambda: lib.ablate_gemm128(layout, M, N, K, a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0),
                                            c.data_ptr(), c.stride(0), st))
        res['gemm128'] = (ms, fl / ms / 1e9)
        ms = run(lambda: torch.matmul(a.T if layout == 2 else a, b.T if layout == 0 else b, out=None))
        res['torch(hipblaslt)'] = (ms, fl / ms / 1e9)
        ms = run(lambda: c.zero_())
        res['zero_'] = (ms, c.numel() * 2 / ms / 1e6)   # GB/s in the TF slot
        print(name, M, N, K, ' '.join(f'{k}={v[0]:.3f}ms/{v[1]:.0f}TF' for k, v in res.items()), flush=True)


if __name__ == '__main__':
    main()
