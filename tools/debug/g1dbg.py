"""Debug: every fp32 GEMM of the g1 IMU encoder fwd+bwd run twice (split-K default vs splits=1), compare."""
import sys
sys.path[:0] = ['tests', 'tests/golden', 'crossmodal-imu-video-ood-har_amd']
import torch
import test_models_gpu as T
from fixtures import load
from cmhar import kernels as K

orig = K.gemm


def checked(layout, a, b, out, **kw):
    if a.dtype != torch.float32 or kw.get('splits') is not None:
        return orig(layout, a, b, out, **kw)
    ref = out.clone()
    kw1 = dict(kw)
    for key in ('aux_out',):
        if kw1.get(key) is not None:
            kw1[key] = kw1[key].clone()
    orig(layout, a, b, ref, splits=1, **kw1)
    r = orig(layout, a, b, out, **kw)
    torch.cuda.synchronize()
    d = ((out - ref).norm() / ref.norm().clamp_min(1e-30)).item()
    M, N = out.shape
    Kd = a.shape[1] if layout < 2 else a.shape[0]
    print(f'layout {layout} M {M} N {N} K {Kd} splits {K._generic_splits(M, N, Kd)} rel {d:.2e} '
          f'keys {[k for k, v in kw.items() if isinstance(v, torch.Tensor) or (v not in (None, 0, 0.0))]}')
    return r


K.gemm = checked
fx = load('g1_imu_encoder')
m, _ = T._build('IMUEncoder', fx)
m.train()
x = torch.tensor(fx['x'], device='cuda')
cls, tok = m(x)
r = torch.tensor(fx['r'], device='cuda')
((cls * r).sum() + 0.1 * tok.pow(2).sum()).backward()
errs = T._grad_errors(m, fx)
print('GRADERR', sorted(errs.items(), key=lambda kv: -kv[1])[:3])
