"""Forward-attention tail kernel time vs key count: Lq = 32 queries (the whole sequence is one tail group, so only
attn_fwd_tail_bf16 runs) at B·H = 384 (the VideoMAE-B step's heads), Lk = 128 … 1568.
    python tools/debug/attn_tail_scan.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..',
                                'crossmodal-imu-video-ood-har_amd'))
from cmhar import kernels as K  # noqa: E402
from gemm_ab import timed  # noqa: E402


def main():
    B, H, D = 32, 12, 64
    g = torch.Generator(device='cuda').manual_seed(0)
    for Lk in (128, 256, 512, 1024, 1568, 3136):
        q = torch.randn(B * 32, H * D, device='cuda', generator=g).bfloat16()
        kv = torch.randn(B * Lk, 2 * H * D, device='cuda', generator=g).bfloat16()
        k, v = kv[:, :H * D], kv[:, H * D:]
        o = torch.empty(B * 32, H * D, device='cuda', dtype=torch.bfloat16)
        lse = torch.empty(B * H * 32, device='cuda')
        fn = lambda: K.attention_fwd(q, k, v, o, lse, B=B, H=H, Lq=32, Lk=Lk, D=D, scale=1.0 / K.LOG2E)  # noqa: E731
        fn()
        torch.cuda.synchronize()
        t = sorted(timed(fn, 20) for _ in range(5))[2]
        print(f'Lk {Lk:5d}  {t * 1e3:7.1f} us  ({(Lk + 127) // 128} stages)', flush=True)


if __name__ == '__main__':
    main()
