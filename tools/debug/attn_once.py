"""Run the bf16 flash attention forward + pre-scaled backward of the VideoMAE-B step shape (B=32, H=12, L=1568,
D=64) a few times with one libcmhar.so build — the workload of the attention PMC passes (tools/debug/pmc_attn2.sh).

    python tools/debug/attn_once.py [LIB.so] [--reps N]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..',
                                'crossmodal-imu-video-ood-har_amd'))
from cmhar import _lib  # noqa: E402
from cmhar import kernels as K  # noqa: E402


def main():
    args = sys.argv[1:]
    reps = 3
    if '--reps' in args:
        i = args.index('--reps')
        reps = int(args[i + 1])
        del args[i:i + 2]
    if args:
        from gemm_ab import load
        _lib._lib = load(args[0])
    B, H, L, D = 32, 12, 1568, 64
    g = torch.Generator(device='cuda').manual_seed(0)
    qkv = torch.randn(B * L, 3 * H * D, device='cuda', generator=g).bfloat16()
    q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
    o = torch.empty(B * L, H * D, device='cuda', dtype=torch.bfloat16)
    lse = torch.empty(B * H * L, device='cuda')
    do = torch.randn(B * L, H * D, device='cuda', generator=g).bfloat16()
    dqkv = torch.empty_like(qkv)
    dq, dk, dv = dqkv[:, :H * D], dqkv[:, H * D:2 * H * D], dqkv[:, 2 * H * D:]
    for _ in range(reps):
        K.attention_fwd(q, k, v, o, lse, B=B, H=H, Lq=L, Lk=L, D=D, scale=1.0 / K.LOG2E)
        K.attention_bwd_prescaled(q, k, v, o, do, lse, dq, dk, dv, B=B, H=H, Lq=L, Lk=L, D=D, scale=D ** -0.5)
    torch.cuda.synchronize()
    print('ok', flush=True)


if __name__ == '__main__':
    main()
