"""Threading contract of the drop-in boundary (the reference's `nn.DataParallel` drives its replicas
from one Python thread per GPU — torch `parallel_apply`, `/root/reference/main.py:89-93` — so launches must be
thread-safe and stream-local).

Two model instances run forward + backward concurrently from two Python threads, each on its own HIP stream, three
steps each; every output and parameter gradient must be bit-identical to the same steps run sequentially on the
default stream.  This exercises the per-(device, stream) workspaces (`cmhar/kernels.py` `workspace`), the ctypes
calls (which release the GIL, so the two threads' launches interleave), each model's IMU side stream and the
autograd engine replaying each backward node on its forward stream.  The HIP library itself keeps no global state.
"""
import threading
import warnings

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _model(backbone, dtype, seed):
    from cmhar.config import Config
    from cmhar.models import CrossModalModel
    cfg = Config()
    cfg.data.imu_window_size = 64
    cfg.data.video_frames_per_window = 4
    cfg.data.video_resize = (32, 32)
    m = cfg.model
    m.video_pretrained = False
    m.compute_dtype = dtype
    m.imu_d_model, m.imu_nhead, m.imu_num_layers, m.imu_dropout = 32, 4, 2, 0.0
    m.video_d_model, m.projection_hidden_dim, m.projection_dim = 64, 64, 32
    m.video_backbone = '/nonexistent/videomae-thr' if backbone == 'videomae' else backbone
    m.videomae_hidden_size, m.videomae_num_layers, m.videomae_num_heads = 128, 2, 2
    m.videomae_intermediate_size, m.videomae_patch_size = 256, 16
    torch.manual_seed(seed)
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        return CrossModalModel(cfg).to(DEV).train()


def _steps(model, batches):
    """fwd + SigLIP loss + bwd per batch on the CURRENT stream; returns the outputs and gradients of every step."""
    from cmhar.losses import SigmoidContrastiveLoss
    lf = SigmoidContrastiveLoss(group=False).to(DEV)
    out = []
    for imu, video in batches:
        model.zero_grad(set_to_none=True)
        a, b = model(imu, video)
        lf(a, b).backward()
        out.append([a.detach().clone(), b.detach().clone()] +
                   [p.grad.detach().clone() for p in model.parameters() if p.grad is not None])
    torch.cuda.current_stream().synchronize()
    return out


@pytest.mark.parametrize('pair', [('videomae', 'videomae'), ('videomae', 'r3d_18')])
@pytest.mark.parametrize('dtype', ['bf16', 'fp32'])
def test_two_threads_two_streams_bit_identical(pair, dtype):
    models = [_model(bb, dtype, 10 + i) for i, bb in enumerate(pair)]
    g = torch.Generator().manual_seed(3)
    data = [[(torch.randn(6, 6, 64, generator=g).to(DEV), torch.randn(6, 4, 3, 32, 32, generator=g).to(DEV))
             for _ in range(3)] for _ in models]
    sequential = [_steps(m, d) for m, d in zip(models, data)]

    results, errors = [None, None], []
    barrier = threading.Barrier(2)
    streams = [torch.cuda.Stream(DEV) for _ in models]

    def run(i):
        try:
            with torch.cuda.stream(streams[i]):
                barrier.wait()
                results[i] = _steps(models[i], data[i])
        except BaseException as e:          # surfaced below: a thread's exception would otherwise be lost
            errors.append(e)

    for s in streams:
        s.wait_stream(torch.cuda.current_stream())
    threads = [threading.Thread(target=run, args=(i,)) for i in range(2)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=100)
    assert not any(t.is_alive() for t in threads), 'thread did not finish'
    assert not errors, errors
    torch.cuda.synchronize()
    for i in range(2):
        assert len(results[i]) == len(sequential[i])
        for step, (got, want) in enumerate(zip(results[i], sequential[i])):
            assert len(got) == len(want)
            for j, (x, y) in enumerate(zip(got, want)):
                assert torch.equal(x, y), (pair[i], step, j, (x - y).abs().max().item())


def test_single_device_dataparallel_wrapper_works():
    """`nn.DataParallel(model)` on one GPU calls the module directly (no replication): same outputs as the bare
    model; the multi-GPU case refuses to replicate (tests/test_api_cpu.py)."""
    m = _model('videomae', 'fp32', 5)
    imu = torch.randn(4, 6, 64, device=DEV)
    video = torch.randn(4, 4, 3, 32, 32, device=DEV)
    a, b = m(imu, video)
    dp = torch.nn.DataParallel(m, device_ids=[0])
    a2, b2 = dp(imu, video)
    assert torch.equal(a, a2) and torch.equal(b, b2)
