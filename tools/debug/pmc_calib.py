"""Calibration of the FETCH_SIZE / WRITE_SIZE traffic figures (tools/pmc_traffic.py doubles FETCH_SIZE, the guide's
gfx950 correction for 128-B requests) on launches whose HBM bytes are known exactly:
  copy     torch copy of a 154 MB bf16 tensor (global loads / stores): reads 154 MB, writes 154 MB
  gemm_n1  the library GEMM, M = 50176, N = 256, K = 768 (one column tile: every A byte fetched once by LDS-DMA):
           reads A 77.1 MB + W 0.4 MB, writes C 25.7 MB
  gemm_n3  the same with N = 768 (three column tiles share each A panel): the same A bytes if the L2 serves the reuse
Run under rocprofv3 --pmc FETCH_SIZE (then WRITE_SIZE) and summarise with tools/pmc_traffic.py."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..', 'crossmodal-imu-video-ood-har_amd'))
from cmhar import kernels as K  # noqa: E402

T = 50176
a = torch.randn(T * 2, 768, device='cuda').bfloat16()
b = torch.empty_like(a)
x = torch.randn(T, 768, device='cuda').bfloat16()
for n in (256, 768):
    w = torch.randn(n, 768, device='cuda').bfloat16()
    y = torch.empty(T, n, device='cuda', dtype=torch.bfloat16)
    for _ in range(3):
        K.gemm(0, x, w, y)
for _ in range(3):
    b.copy_(a)
torch.cuda.synchronize()
print('done')
