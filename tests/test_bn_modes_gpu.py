"""BatchNorm edge modes the reference's torch modules support: `momentum=None` (cumulative moving
average, factor 1 / num_batches_tracked) and eval mode with `track_running_stats=False` (batch statistics).
The heads are checked against the same nn.Sequential run by torch on the CPU; R3D-18 (no reference code) against
an identical model with momentum 1.0 and against the CPU restatement oracle/r3d_cpu.py with batch statistics."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def rel(a, b):
    a, b = torch.as_tensor(a).detach().double().cpu(), torch.as_tensor(b).detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def test_projection_head_momentum_none_matches_torch():
    from cmhar.heads import ProjectionHead
    torch.manual_seed(0)
    head = ProjectionHead(24, 32, 16)
    head.net[1].momentum = None
    ref = ProjectionHead(24, 32, 16)
    ref.load_state_dict(head.state_dict())
    ref.net[1].momentum = None
    head = head.to(DEV).train()
    ref.train()
    for i in range(3):
        x = torch.randn(10, 24) * (i + 1)
        out = head(x.to(DEV))
        rout = ref.net(x)
        assert rel(out, rout) < 1e-5
    bn, rbn = head.net[1], ref.net[1]
    assert int(bn.num_batches_tracked) == int(rbn.num_batches_tracked) == 3
    assert rel(bn.running_mean, rbn.running_mean) < 1e-6
    assert rel(bn.running_var, rbn.running_var) < 1e-6


def _r3d(momentum):
    from cmhar.r3d import R3D18
    torch.manual_seed(0)
    m = R3D18(None, compute_dtype='fp32')
    for mod in m.modules():
        if isinstance(mod, torch.nn.BatchNorm3d):
            mod.momentum = momentum
    return m


def test_r3d_momentum_none_is_cumulative_average():
    x = torch.randn(2, 3, 4, 32, 32)
    a = _r3d(None).to(DEV).train()
    b = _r3d(1.0).to(DEV).train()
    with torch.no_grad():
        a(x.to(DEV))
        a(x.to(DEV))          # same batch twice: the cumulative average equals the batch statistics
        b(x.to(DEV))          # momentum 1: running stats = the batch statistics
    sa, sb = a.state_dict(), b.state_dict()
    keys = [k for k in sa if k.endswith('running_mean') or k.endswith('running_var')]
    assert keys
    for k in keys:
        assert rel(sa[k], sb[k]) < 1e-5, k
        assert int(sa[k.rsplit('.', 1)[0] + '.num_batches_tracked']) == 2


def test_r3d_eval_without_running_stats_uses_batch_statistics():
    from oracle.r3d_cpu import r3d18_features
    m = _r3d(0.1)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    for mod in m.modules():
        if isinstance(mod, torch.nn.BatchNorm3d):
            mod.track_running_stats = False
            mod.running_mean = mod.running_var = mod.num_batches_tracked = None
    m = m.to(DEV).eval()
    x = torch.randn(2, 3, 4, 32, 32)
    with torch.no_grad():
        got = m(x.to(DEV))
    want = r3d18_features(sd, x, training=True)
    assert rel(got, want) < 1e-4
