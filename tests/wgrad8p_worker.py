"""Worker for tests/test_kernels_gpu.py::test_wgrad_8phase_bit_identical_to_two_phase: runs the VideoMAE weight-
gradient GEMM shapes (reduced token count) with random bf16 operands through `cmhar.kernels.gemm` layout 2 — split-K
and whole-K, with the fused bias gradient, overwrite and accumulate — and saves every output to $CMHAR_AB_OUT.  The
parent runs it with CMHAR_GEMM_8P_WGRAD=1 (8-phase kernel) and =0 (two-phase gemm256_kernel), read once per process;
both accumulate each output in the same (K-tile, kk) order, so the outputs must be bit-identical."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'crossmodal-imu-video-ood-har_amd'))
from cmhar import _lib as L  # noqa: E402
from cmhar import kernels as K  # noqa: E402

CASES = [  # (M = out features, N = in features, K = tokens, splits (None = library choice), beta)
    (2304, 768, 6272, None, 0.0),     # QKV
    (768, 768, 6272, None, 1.0),      # out-projection, accumulate
    (3072, 768, 4096, None, 0.0),     # FC1
    (768, 3072, 4096, None, 0.0),     # FC2
    (512, 768, 1024, 1, 0.0),         # whole-K
    (256, 512, 2112, 7, 1.0),         # short last split (2112 = 6·320 + 192)
]


def main():
    dev = torch.device('cuda')
    g = torch.Generator(device=dev).manual_seed(17)
    out = {}
    for i, (M, N, T, splits, beta) in enumerate(CASES):
        dy = torch.randn(T, M, device=dev, generator=g).bfloat16()
        x = torch.randn(T, N, device=dev, generator=g).bfloat16()
        dw = torch.randn(M, N, device=dev, generator=g)
        db = torch.randn(M, device=dev, generator=g)
        s = splits if splits is not None else K._splits_for(M, N, T)
        plan = L.lib().cmhar_gemm_bf16_plan(2, M, N, T, s, 0, 1)
        K.gemm(2, dy, x, dw, beta=beta, splits=splits, rowsum=db, rowsum_beta=beta)
        out[f'dw{i}'], out[f'db{i}'] = dw, db
        out[f'plan{i}'] = torch.tensor([plan])
    torch.cuda.synchronize()
    torch.save({k: v.cpu() for k, v in out.items()}, os.environ['CMHAR_AB_OUT'])


if __name__ == '__main__':
    main()
