"""Time the bf16 flash attention kernels at the VideoMAE-B step shape (B=32, H=12, L=1568, D=64).
python tools/debug/attn_bench.py   (run under rocprofv3 --kernel-trace --stats for the per-kernel split)"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..',
                                'crossmodal-imu-video-ood-har_amd'))
from cmhar import kernels as K  # noqa: E402


def run(fn, reps=10):
    for _ in range(2):
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
    B, H, L, D = 32, 12, 1568, 64
    dev = 'cuda'
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = torch.randn(B * L, 3 * H * D, device=dev, generator=g).bfloat16()
    q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
    o = torch.empty(B * L, H * D, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B * H * L, device=dev)
    do = torch.randn(B * L, H * D, device=dev, generator=g).bfloat16()
    dqkv = torch.empty_like(qkv)
    dq, dk, dv = dqkv[:, :H * D], dqkv[:, H * D:2 * H * D], dqkv[:, 2 * H * D:]
    sc = D ** -0.5
    f = run(lambda: K.attention_fwd(q, k, v, o, lse, B=B, H=H, Lq=L, Lk=L, D=D, scale=sc))
    b = run(lambda: K.attention_bwd(q, k, v, o, do, lse, dq, dk, dv, B=B, H=H, Lq=L, Lk=L, D=D, scale=sc))
    fl = 4 * B * H * L * L * D
    print(f'fwd {f * 1e3:.1f} us {fl / f / 1e9:.0f} TF | bwd {b * 1e3:.1f} us {2.5 * fl / b / 1e9:.0f} TF(10N2D) '
          f'{3.5 * fl / b / 1e9:.0f} TF(14N2D executed)', flush=True)
    # numerics spot check against torch fp32 on 2 heads of batch 0
    qf = q[:L].float().view(L, H, D)[:, :2].transpose(0, 1)
    kf = k[:L].float().view(L, H, D)[:, :2].transpose(0, 1)
    vf = v[:L].float().view(L, H, D)[:, :2].transpose(0, 1)
    ref = torch.softmax(qf @ kf.transpose(1, 2) * sc, -1) @ vf
    got = o[:L].float().view(L, H, D)[:, :2].transpose(0, 1)
    print('fwd rel err', ((got - ref).norm() / ref.norm()).item())
    # torch SDPA (ROCm flash backend) at the same shape, for a ceiling reference
    import torch.nn.functional as F
    qt = q.reshape(B, L, H, D).transpose(1, 2).contiguous().requires_grad_(True)
    kt = k.reshape(B, L, H, D).transpose(1, 2).contiguous().requires_grad_(True)
    vt = v.reshape(B, L, H, D).transpose(1, 2).contiguous().requires_grad_(True)
    got = do.reshape(B, L, H, D).transpose(1, 2).contiguous()
    try:
        tf = run(lambda: F.scaled_dot_product_attention(qt, kt, vt))
        out = F.scaled_dot_product_attention(qt, kt, vt)
        tb = run(lambda: torch.autograd.grad(out, (qt, kt, vt), got, retain_graph=True))
        print(f'torch sdpa fwd {tf * 1e3:.1f} us {fl / tf / 1e9:.0f} TF | bwd {tb * 1e3:.1f} us '
              f'{2.5 * fl / tb / 1e9:.0f} TF', flush=True)
    except Exception as ex:  # noqa: BLE001
        print('torch sdpa unavailable:', ex)


if __name__ == '__main__':
    main()
