"""Worker for tests/test_f32_mfma_gpu.py: runs a fixed set of exact-fp32 GEMMs through `cmhar.kernels.gemm` and
the batched `cmhar_gemm_generic` entry, and saves every output to $CMHAR_AB_OUT.  The parent runs it twice, with
CMHAR_F32_MFMA=1 (f32 MFMA kernel) and =0 (VALU kernel), and requires bit-identical outputs: both kernels are the
k-ordered fmaf chain from 0 (csrc/gemm_generic.hip)."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'crossmodal-imu-video-ood-har_amd'))
from cmhar import _lib as L  # noqa: E402
from cmhar import kernels as K  # noqa: E402

CASES = [  # (layout, M, N, K, epilogue)
    (0, 1568, 768, 768, 'bias'),
    (0, 1000, 900, 772, 'gelu'),          # ragged M / N / K (K % 32 != 0)
    (0, 2048, 3072, 768, 'gelu_aux'),
    (0, 1568, 768, 3072, 'residual'),
    (1, 1568, 768, 2304, 'none'),         # dgrad: B [K, N]
    (1, 1284, 772, 1000, 'dgelu'),
    (2, 768, 768, 12544, 'none'),         # wgrad: A [K, M], split-K
    (2, 3072, 768, 8192, 'beta'),
    (2, 772, 900, 5000, 'none'),          # ragged split-K tail slice
    (2, 1024, 1024, 1568, 'none'),        # single-pass layout 2
]


def main():
    dev = torch.device('cuda')
    g = torch.Generator(device=dev).manual_seed(7)
    out = {}
    for i, (lay, M, N, Kd, ep) in enumerate(CASES):
        a = torch.randn((M, Kd) if lay < 2 else (Kd, M), device=dev, generator=g)
        b = torch.randn((N, Kd) if lay == 0 else (Kd, N), device=dev, generator=g)
        c = torch.randn(M, N, device=dev, generator=g) if ep == 'beta' else torch.empty(M, N, device=dev)
        kw = {}
        if ep in ('bias', 'gelu', 'gelu_aux'):
            kw['bias'] = torch.randn(N, device=dev, generator=g)
        if ep in ('gelu', 'gelu_aux'):
            kw['act'] = L.ACT_GELU
        if ep == 'gelu_aux':
            kw['aux_out'] = torch.empty(M, N, device=dev)
        if ep == 'residual':
            kw['residual'] = torch.randn(M, N, device=dev, generator=g)
        if ep == 'dgelu':
            kw['act'] = L.ACT_DGELU
            kw['aux_in'] = torch.randn(M, N, device=dev, generator=g)
        if ep == 'beta':
            kw['beta'] = 1.0
        K.gemm(lay, a, b, c, **kw)
        out[f'case{i}'] = c
        if 'aux_out' in kw:
            out[f'case{i}_aux'] = kw['aux_out']
    # batched, strided (the attention-style z-batched entry) with bf16 output
    Bt, M, N, Kd = 3, 640, 520, 384
    a = torch.randn(Bt, M, Kd, device=dev, generator=g)
    b = torch.randn(Bt, N, Kd, device=dev, generator=g)
    c = torch.empty(Bt, M, N, device=dev, dtype=torch.bfloat16)
    rc = L.lib().cmhar_gemm_generic(L.F32, L.BF16, M, N, Kd, Bt, K.ptr(a), Kd, 1, M * Kd, K.ptr(b), 1, Kd, N * Kd,
                                    K.ptr(c), N, M * N, None, L.stream(dev))
    assert rc == 0, rc
    out['batched_bf16'] = c
    torch.cuda.synchronize()
    torch.save({k: v.cpu() for k, v in out.items()}, os.environ['CMHAR_AB_OUT'])


if __name__ == '__main__':
    main()
