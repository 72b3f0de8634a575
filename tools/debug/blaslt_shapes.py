"""hipBLASLt (torch.matmul) on the VideoMAE-B step's forward / dgrad shapes, for kernel names and times under
rocprofv3 --kernel-trace --stats (reference point for the hand GEMMs; not on the product path)."""
import torch

T = 50176
dt = torch.bfloat16
shapes = [('qkv', 2304, 768), ('out', 768, 768), ('fc1', 3072, 768), ('fc2', 768, 3072), ('embed', 768, 1536)]
for name, n_out, n_in in shapes:
    x = torch.randn(T, n_in, device='cuda', dtype=dt)
    w = torch.randn(n_out, n_in, device='cuda', dtype=dt)
    b = torch.randn(n_out, device='cuda', dtype=dt)
    for _ in range(20):
        torch.nn.functional.linear(x, w, b)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        torch.nn.functional.linear(x, w, b)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    print(f'{name:6s} fwd {us:7.1f} us {2 * T * n_out * n_in / us / 1e6:6.0f} TF', flush=True)
