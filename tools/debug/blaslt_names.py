"""Print which hipBLASLt kernels torch.matmul picks for the VideoMAE forward GEMM shapes (run under rocprofv3)."""
import torch
T = 50176
for n_out, n_in in [(2304, 768), (768, 768), (3072, 768), (768, 3072)]:
    x = torch.randn(T, n_in, device='cuda').bfloat16()
    w = torch.randn(n_out, n_in, device='cuda').bfloat16()
    for _ in range(3):
        torch.matmul(x, w.T)
torch.cuda.synchronize()
