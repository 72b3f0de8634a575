"""The drop-in model at the other geometries the BASELINE configs name, against the CPU oracle (oracle/cpu_model.py,
pinned to the reference by g1-g9) on identical seeded weights and inputs:

* IMU windows of 250 (the reference default: 15 patches → CLS + 15 channel-0 tokens) and 400 (config 4: 25 → 26),
* 32-frame clips (config 4's VideoMAE `num_frames=32`: 16 tubelets in time), small spatial size to keep the oracle fast.

fp32 mode: projections ≤ 1e-4 relative, loss ≤ 1e-5, every parameter gradient ≤ 1e-3 relative (as g2); bf16 mode
(throughput): projections ≤ 3e-2."""
import numpy as np
import pytest
import torch

from fixtures import oracle_mcfg
from seeded import seeded_input, seeded_state_dict

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _cfg(imu_w, frames, image, dtype):
    from cmhar.config import Config
    cfg = Config()
    cfg.data.imu_window_size = imu_w
    cfg.data.video_frames_per_window = frames
    cfg.data.video_resize = (image, image)
    m = cfg.model
    m.video_backbone = '/nonexistent/videomae-geom'
    m.video_pretrained = False
    m.imu_dropout = 0.0
    m.videomae_hidden_size, m.videomae_num_layers, m.videomae_num_heads = 128, 2, 2
    m.videomae_intermediate_size, m.videomae_patch_size = 256, 16
    m.video_d_model, m.projection_hidden_dim, m.projection_dim = 96, 64, 32
    m.compute_dtype = dtype
    return cfg


def rel(a, b):
    a, b = torch.as_tensor(a).detach().float().cpu(), torch.as_tensor(b).detach().float().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize('imu_w,frames,image', [(250, 16, 32), (400, 32, 32)])
@pytest.mark.parametrize('dtype,tol', [('fp32', 1e-4), ('bf16', 3e-2)])
def test_crossmodal_geometry_vs_oracle(imu_w, frames, image, dtype, tol):
    import warnings
    from cmhar.losses import SigmoidContrastiveLoss
    from cmhar.models import CrossModalModel
    from oracle import cpu_model as O
    cfg = _cfg(imu_w, frames, image, dtype)
    torch.manual_seed(0)
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        m = CrossModalModel(cfg)
    sd = seeded_state_dict(m.state_dict(), seed=77)
    m.load_state_dict(sd, strict=True)
    m = m.to(DEV).train()
    B = 6
    imu = seeded_input(78, (B, 6, imu_w))
    video = seeded_input(79, (B, frames, 3, image, image))
    n_tok = (imu_w - 16) // 16 + 2
    assert m.imu_encoder.pos_encoding.shape[1] == n_tok
    a, b = m(imu.to(DEV), video.to(DEV))
    loss = SigmoidContrastiveLoss().to(DEV)(a, b)
    loss.backward()
    ref_sd = {k: (v.clone().requires_grad_(True) if v.is_floating_point() else v.clone()) for k, v in sd.items()}
    ra, rb = O.crossmodal(ref_sd, imu, video, oracle_mcfg(cfg), training=True)
    rloss = O.siglip_loss(ra, rb, torch.tensor(float(np.log(10.0))), torch.tensor(-10.0))
    rloss.backward()
    assert rel(a, ra) < tol and rel(b, rb) < tol
    assert abs(loss.item() - rloss.item()) < (1e-5 if dtype == 'fp32' else 1e-2) * abs(rloss.item())
    if dtype == 'fp32':
        gscale = max(float(v.grad.abs().max()) for v in ref_sd.values() if v.is_floating_point() and v.grad is not None)
        worst = {}
        for name, p in m.named_parameters():
            g = ref_sd[name].grad
            if g is None or float(g.abs().max()) < 1e-5 * gscale:   # mathematically-zero gradient: noise only
                continue
            worst[name] = rel(p.grad, g)
        assert max(worst.values()) < 1e-3, sorted(worst.items(), key=lambda kv: -kv[1])[:4]
