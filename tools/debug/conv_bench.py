"""Per-layer timing of the R3D-18 implicit-GEMM conv kernels at the bench geometry (B clips of 16x112^2, NDHWC bf16):
forward (cmhar_conv3d_fwd: row-slab or generic kernel per the library's plan / CMHAR_FWD_ROWS) and weight gradient
(cmhar_conv3d_wgrad; CMHAR_WGRAD_ROWS), each layer's algorithmic TFLOP/s.
    python tools/debug/conv_bench.py [--batch 32] [--reps 10]"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..',
                                'crossmodal-imu-video-ood-har_amd'))
from cmhar import _lib as L  # noqa: E402
from cmhar import kernels as K  # noqa: E402

# (name, T, H=W, Cin, Cout, stride) of the input of each 3x3x3 conv shape in R3D-18 at 16x112^2
LAYERS = [('layer1', 16, 56, 64, 64, 1), ('layer2.0.conv1', 16, 56, 64, 128, 2), ('layer2', 8, 28, 128, 128, 1),
          ('layer3.0.conv1', 8, 28, 128, 256, 2), ('layer3', 4, 14, 256, 256, 1),
          ('layer4.0.conv1', 4, 14, 256, 512, 2), ('layer4', 2, 7, 512, 512, 1)]


def timed(fn, reps):
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
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=32)
    ap.add_argument('--reps', type=int, default=10)
    ap.add_argument('--layers', default='', help='comma-separated layer names (default: all)')
    a = ap.parse_args()
    dev = torch.device('cuda')
    st = L.stream(dev)
    keep = set(a.layers.split(',')) if a.layers else None
    if keep is None or 'stem' in keep:
        # the implicit stem: 3 -> 64, 3x7x7, stride (1, 2, 2), pad (1, 3, 3) on the 16x112^2 clips
        from cmhar import r3d
        N = a.batch
        conv = torch.nn.Conv3d(3, 64, (3, 7, 7), (1, 2, 2), (1, 3, 3), bias=False).to(dev)
        x = torch.randn(N, 16, 112, 112, 3, device=dev).bfloat16()
        shp = tuple(x.shape)
        dims = r3d._dims(shp, conv, r3d._stem_kp(conv))
        w4 = r3d._pack_stem(conv)
        M = N * 16 * 56 * 56
        z = torch.empty(M, 64, device=dev, dtype=torch.bfloat16)
        dz = torch.randn(M, 64, device=dev).bfloat16()
        dw4 = torch.empty(64, r3d._stem_kp(conv), device=dev)
        ws = K.workspace(L.lib().cmhar_conv3d_stem_wgrad_ws(dims, 64), dev)
        fl = 2 * M * 64 * 3 * 7 * 7 * 3
        tf = timed(lambda: L.call('cmhar_conv3d_stem_fwd', dims, 64, K.ptr(x), K.ptr(w4), K.ptr(z), None, st), a.reps)
        tw = timed(lambda: L.call('cmhar_conv3d_stem_wgrad', dims, 64, K.ptr(x), K.ptr(dz), K.ptr(dw4), K.ptr(ws), st),
                   a.reps)
        print(f'{"stem":15s} M={M:8d} K={441:6d} Cout={64:4d}  fwd {tf * 1e3:7.1f} us {fl / tf / 1e9:6.0f} TF   '
              f'wgrad {tw * 1e3:7.1f} us {fl / tw / 1e9:6.0f} TF', flush=True)
    for name, T, H, C, Co, s in LAYERS:
        if keep is not None and name not in keep:
            continue
        N = a.batch
        To, Ho = (T - 1) // s + 1, (H - 1) // s + 1
        Kd = 27 * C
        dims = (ctypes.c_int * 15)(N, T, H, H, C, 3, 3, 3, s, s, s, 1, 1, 1, Kd)
        x = torch.randn(N, T, H, H, C, device=dev).bfloat16()
        w = (torch.randn(Co, Kd, device=dev) * 0.05).bfloat16()
        M = N * To * Ho * Ho
        z = torch.empty(M, Co, device=dev, dtype=torch.bfloat16)
        dz = torch.randn(M, Co, device=dev).bfloat16()
        dw = torch.empty(Co, Kd, device=dev)
        n = L.lib().cmhar_conv3d_wgrad_ws(dims, Co)
        ws = K.workspace(max(n, 1), dev)
        fl = 2 * M * Co * Kd
        tf = timed(lambda: L.call('cmhar_conv3d_fwd', dims, Co, K.ptr(x), K.ptr(w), None, K.ptr(z), None, st), a.reps)
        tw = timed(lambda: L.call('cmhar_conv3d_wgrad', dims, Co, K.ptr(x), K.ptr(dz), K.ptr(dw), K.ptr(ws), st),
                   a.reps)
        print(f'{name:15s} M={M:8d} K={Kd:6d} Cout={Co:4d}  fwd {tf * 1e3:7.1f} us {fl / tf / 1e9:6.0f} TF   '
              f'wgrad {tw * 1e3:7.1f} us {fl / tw / 1e9:6.0f} TF', flush=True)


if __name__ == '__main__':
    main()
