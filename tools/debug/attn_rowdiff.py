"""Where do two libcmhar.so builds' flash attention outputs differ?  Runs the VideoMAE-B step shape (B=32, H=12,
L=1568, D=64, pre-scaled keys) through lib A and lib B (each twice: run-to-run determinism) and prints, per output,
the differing rows (row index mod L) and the largest difference.

    python tools/debug/attn_rowdiff.py libA.so libB.so
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..',
                                'crossmodal-imu-video-ood-har_amd'))
from cmhar import _lib  # noqa: E402
from cmhar import kernels as K  # noqa: E402
from gemm_ab import load  # noqa: E402


def run(lib, q, k, v, do, B, H, L, D):
    _lib._lib = lib
    o = torch.empty(B * L, H * D, device='cuda', dtype=torch.bfloat16)
    lse = torch.empty(B * H * L, device='cuda')
    K.attention_fwd(q, k, v, o, lse, B=B, H=H, Lq=L, Lk=L, D=D, scale=1.0 / K.LOG2E)
    dqkv = torch.empty(B * L, 3 * H * D, device='cuda', dtype=torch.bfloat16)
    dq, dk, dv = dqkv[:, :H * D], dqkv[:, H * D:2 * H * D], dqkv[:, 2 * H * D:]
    K.attention_bwd_prescaled(q, k, v, o, do, lse, dq, dk, dv, B=B, H=H, Lq=L, Lk=L, D=D, scale=D ** -0.5)
    torch.cuda.synchronize()
    return {'o': o, 'lse': lse.view(B, H, L).permute(0, 2, 1).reshape(B * L, H), 'dq': dq, 'dk': dk, 'dv': dv}


def report(tag, a, b, L):
    for name in a:
        x, y = a[name].float(), b[name].float()
        bad = (x != y).any(dim=1).nonzero().flatten()
        if bad.numel() == 0:
            print(f'{tag} {name}: identical', flush=True)
            continue
        rows = sorted(set((bad % L).tolist()))
        print(f'{tag} {name}: {bad.numel()} rows differ, max |d| {(x - y).abs().max().item():.3e}, '
              f'rows mod L: {rows[:12]}{" ..." if len(rows) > 12 else ""} ({len(rows)} distinct)', flush=True)


def main():
    la, lb = load(sys.argv[1]), load(sys.argv[2])
    B, H, L, D = 32, 12, 1568, 64
    g = torch.Generator(device='cuda').manual_seed(0)
    qkv = torch.randn(B * L, 3 * H * D, device='cuda', generator=g).bfloat16()
    q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
    do = torch.randn(B * L, H * D, device='cuda', generator=g).bfloat16()
    a1, a2 = run(la, q, k, v, do, B, H, L, D), run(la, q, k, v, do, B, H, L, D)
    b1, b2 = run(lb, q, k, v, do, B, H, L, D), run(lb, q, k, v, do, B, H, L, D)
    report('A vs A', a1, a2, L)
    report('B vs B', b1, b2, L)
    report('A vs B', a1, b1, L)


if __name__ == '__main__':
    main()
