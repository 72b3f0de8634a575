"""Every convolution launch of the R3D-18 training step (BASELINE config 2 with the north_star's R3D backbone:
`bench.py --workload r3d` / tools/bench_r3d.py, B = 32 clips of 16 × 112², bf16) at its PRODUCTION geometry, through
the entry points the step itself calls (`cmhar/r3d.py` `_conv_fwd` / `_conv_wgrad` / `_conv_dgrad`, which `_unit_fwd` /
`_unit_bwd` run between the BatchNorms) — VERDICT r04 item 2.  Smaller-shape tests (tests/test_r3d_gpu.py) do not
reach these plans: the nine-tap kernels of layers 1–3 (layer 1 at 1.6 M output rows, layers 2–3 on 64-wide Cout
slices; forward and flipped-weight input gradient), layer 4's on the split-K slab, the stride-2 convs and the
downsamples on the generic 128×128 gather kernel (layer 4's stride-2 conv split over K) with their input gradients as dz·W on the GEMM + col2im (the
residual-branch gradient accumulated), every weight gradient on the row-slab / nine-tap / gather kernels with its
split reduce.

Two checks per geometry (forward z, weight gradient dW, input gradient dx):
* integer operands (x, W in [-2, 2], dz sparse in {-1, 0, 1}: every product and partial sum exact in fp32, dz·W
  columns exact in bf16): bit-exact against torch's fp64 convolution and its autograd (fp64 has no MIOpen kernel, so
  torch runs its own vol2col + GEMM) — bf16 outputs compared after the same round-to-nearest-even;
* random bf16 operands: against torch fp32 conv3d / autograd on the same operands: z and dx ≤ 5e-3 rel (bf16 output
  rounding), dW ≤ 1e-4 rel (fp32 output, summation order only).
`test_r3d_production_plans` pins the kernel each geometry takes (cmhar_conv3d_fwd_plan / _wgrad_plan, the split
plan), so the parity cases test the code the bench runs."""
import math

import pytest
import torch
import torch.nn.functional as F

DEV = 'cuda'
B, T, S = 32, 16, 112

# (name, cin, cout, k, stride, pad, input (N, T, H, W)) — every distinct conv of R3D-18 at B = 32, 16 × 112²
# (the stem has its own production test, tests/test_r3d_gpu.py::test_r3d_implicit_stem_production_geometry)
GEOMS = [
    ('layer1.conv', 64, 64, 3, 1, 1, (B, 16, 56, 56)),
    ('layer2.0.conv1', 64, 128, 3, 2, 1, (B, 16, 56, 56)),
    ('layer2.0.downsample', 64, 128, 1, 2, 0, (B, 16, 56, 56)),
    ('layer2.conv2', 128, 128, 3, 1, 1, (B, 8, 28, 28)),
    ('layer3.0.conv1', 128, 256, 3, 2, 1, (B, 8, 28, 28)),
    ('layer3.0.downsample', 128, 256, 1, 2, 0, (B, 8, 28, 28)),
    ('layer3.conv2', 256, 256, 3, 1, 1, (B, 4, 14, 14)),
    ('layer4.0.conv1', 256, 512, 3, 2, 1, (B, 4, 14, 14)),
    ('layer4.0.downsample', 256, 512, 1, 2, 0, (B, 4, 14, 14)),
    ('layer4.conv2', 512, 512, 3, 1, 1, (B, 2, 7, 7)),
]

# the plans of the step (fwd: 'split' or cmhar_conv3d_fwd_plan; dgrad: 'flip:<fwd plan of the flipped conv>' or
# 'col2im'; wgrad: cmhar_conv3d_wgrad_plan, '+r' = with the split reduce)
PLANS = {
    'layer1.conv': (1, 'flip:1', '1+r'),
    'layer2.0.conv1': (5, 'col2im', '2+r'),          # stride 2: the row slab does not fit, generic 128x128 gather
    'layer2.0.downsample': (5, 'col2im', '4+r'),
    'layer2.conv2': (1, 'flip:1', '1+r'),            # nine-tap slab fwd / wgrad, 7-row tiles x 64-wide Cout slices
    'layer3.0.conv1': (5, 'col2im', '2+r'),
    'layer3.0.downsample': (5, 'col2im', '4+r'),
    'layer3.conv2': (1, 'flip:1', '1+r'),            # nine-tap slab fwd / wgrad, one 14-row tile per frame
    'layer4.0.conv1': ('split', 'col2im', '2+r'),    # stride 2, 100 128x128 tiles: generic gather split over K
    'layer4.0.downsample': (5, 'col2im', '4+r'),
    'layer4.conv2': ('split', 'flip:split', '2'),    # one split of the weight gradient: no reduce
}


def _conv(cin, cout, k, s, p):
    return torch.nn.Conv3d(cin, cout, k, s, p, bias=False)


def _plans(cin, cout, k, s, p, shape):
    from cmhar import _lib as L
    from cmhar import r3d
    lib = L.lib()
    conv = _conv(cin, cout, k, s, p)
    shp = tuple(shape) + (cin,)
    Kp = r3d._r8(conv.weight[0].numel())
    dims = r3d._dims(shp, conv, Kp)
    fwd = 'split' if lib.cmhar_conv3d_fwd_split_ws(dims, cout) > 0 else lib.cmhar_conv3d_fwd_plan(dims, cout)
    if r3d._dgrad_igemm_ok(conv):
        N, To, Ho, Wo, _ = r3d._out_shape(shp, conv)
        kt, kh, kw = conv.kernel_size
        fd = r3d._dims((N, To, Ho, Wo, cout), _conv(cout, cin, k, 1, p), kt * kh * kw * cout)
        dg = 'flip:' + str('split' if lib.cmhar_conv3d_fwd_split_ws(fd, cin) > 0 else lib.cmhar_conv3d_fwd_plan(fd, cin))
    else:
        dg = 'col2im'
    wg = str(lib.cmhar_conv3d_wgrad_plan(dims, cout)) + ('+r' if lib.cmhar_conv3d_wgrad_ws(dims, cout) > 0 else '')
    return fwd, dg, wg


def test_r3d_production_plans():
    """The geometries above take the plans the step takes (host-side plan queries of the library; no GPU needed)."""
    got = {g[0]: _plans(*g[1:]) for g in GEOMS}
    assert got == PLANS, {k: (got[k], PLANS[k]) for k in got if got[k] != PLANS[k]}


def test_r3d_plans_past_buffer_range():
    """The row-slab / nine-tap kernels address x and dz through buffer resources with 32-bit offsets (padding = an
    out-of-range offset that reads zero), so their plans require x (and dz) within 1 GiB; past that, a geometry falls
    back to the generic implicit GEMM (its 64-bit instantiation beyond 2 GiB).  Host-side plan queries, no GPU."""
    from cmhar import _lib as L
    from cmhar import r3d
    lib = L.lib()
    conv = _conv(64, 64, 3, 1, 1)
    for n, fwd, wg in [(32, 1, 1), (160, 1, 1), (168, 4, 4)]:    # x = N·16·56²·64·2 B: 205 MB, 1.028 GB, 1.079 GB
        shp = (n, 16, 56, 56, 64)
        dims = r3d._dims(shp, conv, r3d._r8(conv.weight[0].numel()))
        assert lib.cmhar_conv3d_fwd_plan(dims, 64) == fwd, n
        assert lib.cmhar_conv3d_fwd_split_ws(dims, 64) == 0
        assert lib.cmhar_conv3d_wgrad_plan(dims, 64) == wg, n


@pytest.mark.gpu
def test_conv3d_generic_forward_past_2gib():
    """The generic implicit-GEMM forward keeps a 64-bit-address instantiation for inputs over 2 GiB (R3D-18's
    layer2.0.conv1 geometry at N = 336: x = 2.16 GB): its output on the first clips equals, bit for bit, the
    buffer-resource instantiation's on those clips alone (each clip's convolution is independent), and the last
    clips' too.  Slices of 8 clips (392 tiles): fewer would take the split-K plan, whose fp32 partial sums associate
    differently."""
    from cmhar import _lib as L
    from cmhar import r3d
    torch.manual_seed(11)
    conv = _conv(64, 128, 3, 2, 1).to(DEV)
    n_big = 336
    x = torch.randn(n_big, 16, 56, 56, 64, device=DEV, dtype=torch.bfloat16)
    assert x.numel() * 2 > (1 << 31)
    wp = r3d._pack(conv, torch.bfloat16)
    with torch.no_grad():
        z_big = r3d._conv_fwd(x, tuple(x.shape), conv, wp, stats=False)[0]
        for sl in (slice(0, 8), slice(n_big - 8, n_big)):
            xs = x[sl].contiguous()
            assert L.lib().cmhar_conv3d_fwd_split_ws(r3d._dims(tuple(xs.shape), conv, wp.shape[1]), 128) == 0
            z_s = r3d._conv_fwd(xs, tuple(xs.shape), conv, wp, stats=False)[0]
            per = z_s.shape[0] // xs.shape[0]
            assert torch.equal(z_big[sl.start * per:sl.stop * per], z_s)
    torch.cuda.synchronize()


def _operands(kind, cin, cout, k, s, p, shape, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    N, T_, H, W = shape
    conv = _conv(cin, cout, k, s, p).to(DEV)
    if kind == 'int':
        ri = lambda shp, lo=-2, hi=3: torch.randint(lo, hi, shp, generator=g, device=DEV).float()   # noqa: E731
        x = ri((N, T_, H, W, cin)).bfloat16()
        with torch.no_grad():
            conv.weight.copy_(ri(tuple(conv.weight.shape)))
        Ho = [(d + 2 * p - k) // s + 1 for d in (T_, H, W)]
        dz = ri((N, *Ho, cout), -1, 2) * (torch.rand((N, *Ho, cout), generator=g, device=DEV) < 1.0 / 32).float()
        dz = dz.bfloat16()
        acc = ri((N, T_, H, W, cin)).bfloat16()
    else:
        x = torch.randn(N, T_, H, W, cin, generator=g, device=DEV).bfloat16()
        with torch.no_grad():
            conv.weight.copy_(torch.randn(conv.weight.shape, generator=g, device=DEV) / math.sqrt(conv.weight[0].numel()))
        Ho = [(d + 2 * p - k) // s + 1 for d in (T_, H, W)]
        dz = torch.randn(N, *Ho, cout, generator=g, device=DEV).bfloat16()
        acc = torch.randn(N, T_, H, W, cin, generator=g, device=DEV).bfloat16()
    return conv, x, dz, acc


@pytest.mark.gpu
@pytest.mark.parametrize('kind', ['int', 'rand'])
@pytest.mark.parametrize('geom', GEOMS, ids=[g[0] for g in GEOMS])
def test_r3d_production_conv(geom, kind):
    from cmhar import r3d
    name, cin, cout, k, s, p, shape = geom
    conv, x, dz5, acc = _operands(kind, cin, cout, k, s, p, shape, seed=sum(map(ord, name)) + (7 if kind == 'rand' else 0))
    shp = tuple(x.shape)
    dt = torch.bfloat16
    flip = r3d._dgrad_igemm_ok(conv) and cin % 64 == 0
    packs = r3d._pack_all([(conv, flip)], dt, x.device)[conv]        # the step's one-launch weight pack
    wp, wf = packs if flip else (packs, None)
    # residual-branch gradient: the 3x3x3 convs' input gradients accumulate into it in the step (dres of the block or
    # the downsample's dx), the downsamples' do not
    dx_acc = acc.clone() if k == 3 else None
    with torch.no_grad():
        z, col, wp, stem, igemm, _, _ = r3d._conv_fwd(x, shp, conv, wp, stats=True)
        u = r3d._Unit()
        oshape = r3d._out_shape(shp, conv)
        M = math.prod(oshape[:4])
        u.conv, u.shape, u.oshape, u.Kp, u.rows, u.wp = conv, shp, oshape, r3d._r8(conv.weight[0].numel()), r3d._r8(M), wp
        u.x, u.col, u.igemm, u.wf, u.stem = x, col, igemm, wf, stem
        dz = torch.zeros(u.rows, cout, dtype=dt, device=DEV)
        dz[:M] = dz5.reshape(M, cout)
        dwp = r3d._conv_wgrad(u, dz)
        dx = r3d._conv_dgrad(u, dz, dx_acc)
        torch.cuda.synchronize()
    # reference: torch conv3d + autograd in fp64 (integers: exact) or fp32 (random)
    rd = torch.float64 if kind == 'int' else torch.float32
    xr = x.permute(0, 4, 1, 2, 3).to(rd).requires_grad_(True)
    wr = conv.weight.detach().bfloat16().to(rd).requires_grad_(True)
    zr = F.conv3d(xr, wr, stride=s, padding=p)
    gx, gw = torch.autograd.grad(zr, (xr, wr), dz5.permute(0, 4, 1, 2, 3).to(rd))
    z_want = zr.detach().permute(0, 2, 3, 4, 1).reshape(M, cout)
    dx_want = gx.permute(0, 2, 3, 4, 1) + (acc.to(rd) if dx_acc is not None else 0)
    kk = conv.weight[0].numel()
    dw_got = dwp[:, :kk].reshape(cout, k, k, k, cin).permute(0, 4, 1, 2, 3)
    del zr, xr
    if kind == 'int':
        for what, got, want in (('z', z, z_want), ('dx', dx.reshape(dx_want.shape), dx_want)):
            bad = int((got != want.to(dt)).sum())
            assert bad == 0, (name, what, bad, (got.double() - want).abs().max().item())
        bad = int((dw_got.double() != gw).sum())
        assert bad == 0, (name, 'dW', bad, (dw_got.double() - gw).abs().max().item())
    else:
        def rel(a, b):
            a, b = a.double(), b.double()
            return ((a - b).norm() / b.norm()).item()
        assert rel(z, z_want) < 5e-3, (name, 'z', rel(z, z_want))
        assert rel(dx.reshape(dx_want.shape), dx_want) < 5e-3, (name, 'dx', rel(dx.reshape(dx_want.shape), dx_want))
        assert rel(dw_got, gw) < 1e-4, (name, 'dW', rel(dw_got, gw))
    del z, dx, dwp, gx, gw
    torch.cuda.empty_cache()
