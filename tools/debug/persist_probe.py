"""In-kernel timeline of the persistent 8-phase GEMM (a build with -DCMHAR_PERSIST_PROBE=1 via CMHAR_LIB): s_memtime
stamps of each workgroup's wave 0 (group 0) and wave 4 (group 1) at tile start (0), after K-tile 0 (1), after the last
K-tile (2), after the re-align barrier + boundary DMA (3), after the epilogue's stores are issued (4).
python tools/debug/persist_probe.py qkv|fc1"""
import ctypes as C
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..',
                                'crossmodal-imu-video-ood-har_amd'))
from cmhar import _lib, kernels as K  # noqa: E402

SH = {'qkv': (2304, 768), 'fc1': (3072, 768)}
name = sys.argv[1] if len(sys.argv) > 1 else 'qkv'
n_out, n_in = SH[name]
T = int(sys.argv[2]) if len(sys.argv) > 2 else 50176    # rows (a build with CMHAR_PERSIST_MIN_ROUNDS=0 for few tiles)
x = torch.randn(T, n_in, device='cuda').bfloat16()
w = torch.randn(n_out, n_in, device='cuda').bfloat16()
y = torch.empty(T, n_out, device='cuda', dtype=torch.bfloat16)
b = torch.randn(n_out, device='cuda')
kw = {'bias': b}
if name == 'fc1':
    kw.update(act=_lib.ACT_GELU_SAVEGRAD, aux_out=torch.empty_like(y))
for _ in range(5):
    K.gemm(0, x, w, y, **kw)
torch.cuda.synchronize()
lib = _lib.lib()
n = 256 * 12 * 2 * 6
buf = (C.c_ulonglong * n)()
f = lib.cmhar_debug_persist_probe
f.argtypes = [C.c_void_p, C.c_long]
assert f(buf, n) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(256, 12, 2, 6).astype(np.int64)
t0 = a[:, 0, 0, 0][a[:, 0, 0, 0] > 0].min()
ntile = (T // 256) * (n_out // 256)
for g in range(2):
    rows = []
    for s in range(12):
        v = a[:, s, g, :]
        ok = (v[:, 0] > 0) & (v[:, 4] > 0)
        if ok.sum() < 1:
            continue
        v = v[ok]
        d = lambda i, j: statistics.median((v[:, j] - v[:, i]).tolist())  # noqa: E731
        rows.append((s, ok.sum(), statistics.median((v[:, 0] - t0).tolist()), d(0, 1), d(1, 2), d(2, 3), d(3, 4)))
    print(f'group {g}: tile  wgs  start   K0   K1..last  align+dma  epilogue   (cycles, medians)')
    for r in rows:
        print('   %4d %4d %7d %6d %8d %8d %8d' % r)
    # epilogue cycles per quarter of each XCD's CUs (workgroup slot (blockIdx >> 3) & 3), tiles 1..
    qs = []
    for q in range(4):
        sel = [w for w in range(256) if (w >> 3) & 3 == q]
        v = a[sel, 1:, g, :]
        v = v[(v[:, :, 3] > 0) & (v[:, :, 4] > 0)]
        qs.append(statistics.median((v[:, 4] - v[:, 3]).tolist()) if len(v) else 0)
    print('   epilogue by quarter:', qs)
