"""Which fp32 generic-GEMM launches a bench step issues, with shape, split count, stream and HIP-event time each
(round 6: the gemm_generic_kernel rows of the step's kernel trace, ~0.5 ms/step).  Wraps cmhar.kernels.gemm for one
warm step of bench.py's headline workload; events on the launch stream."""
import collections
import os
import sys
import traceback

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'crossmodal-imu-video-ood-har_amd'))
import torch  # noqa: E402
import bench  # noqa: E402
from cmhar import kernels as K  # noqa: E402

sys.argv = ['bench.py', '--steps', '1', '--warmup', '2', '--no-cpu-baseline', '--no-trace']
args = bench.parse()
dev = torch.device('cuda', 0)
torch.cuda.set_device(0)
W = bench.build_workload(args, dev, 0, 1)
for _ in range(3):
    W.step()
torch.cuda.synchronize()

rec = []
orig = K.gemm


def wrapped(layout, a, b, out, **kw):
    if a.dtype != torch.float32:
        return orig(layout, a, b, out, **kw)
    if layout == 0:
        M, Kd = a.shape
        N = b.shape[0]
    elif layout == 1:
        M, Kd = a.shape
        N = b.shape[1]
    else:
        Kd, M = a.shape
        N = b.shape[1]
    s = kw.get('splits')
    s = K._generic_splits(M, N, Kd) if s is None else s
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    r = orig(layout, a, b, out, **kw)
    e1.record(st)
    site = [f'{os.path.basename(f.filename)}:{f.lineno}:{f.name}' for f in traceback.extract_stack()[-5:-1]]
    rec.append((layout, M, N, Kd, s, st.cuda_stream, e0, e1, ' <- '.join(reversed(site))))
    return r


K.gemm = wrapped
W.step()
torch.cuda.synchronize()
tot = collections.defaultdict(float)
for layout, M, N, Kd, s, stream, e0, e1, site in rec:
    us = e0.elapsed_time(e1) * 1e3
    tot[stream] += us
    print(f'layout {layout} M {M:6d} N {N:5d} K {Kd:6d} splits {s:2d} stream {stream:#x} {us:8.1f} us  {site}')
print({hex(k): round(v, 1) for k, v in tot.items()}, 'us per stream')
