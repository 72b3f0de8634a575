"""Cross-attention fusion (north_star extension; parity unpinned w.r.t. the reference, which has no fusion module)
against the CPU restatement oracle/fusion_cpu.py on identical weights and inputs.

fp32 mode: logits / fused ≤ 1e-5 rel, every parameter and input gradient ≤ 1e-4 rel.  bf16 mode (K|V projection and
flash attention on MFMA): logits ≤ 2e-2 rel, gradients ≤ 5e-2 rel.  Ragged sizes: Lq = 13 IMU tokens (CLS + 12
patches of a 200-step window), Lk = 392 / 200 video tokens (not multiples of the attention tiles)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def rel(a, b):
    a, b = torch.as_tensor(a).detach().double().cpu(), torch.as_tensor(b).detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize('dtype,Lk,B', [('fp32', 392, 3), ('bf16', 392, 3), ('bf16', 200, 5)])
def test_fusion_matches_oracle(dtype, Lk, B):
    from cmhar.fusion import CrossAttentionFusion
    from oracle.fusion_cpu import fusion_forward
    torch.manual_seed(0)
    m = CrossAttentionFusion(128, 768, 256, 4, 32, compute_dtype=dtype)
    sd = {k: v.clone().requires_grad_(True) for k, v in m.state_dict().items()}
    imu = torch.randn(B, 13, 128, requires_grad=True)
    vid = torch.randn(B, Lk, 768, requires_grad=True)
    R = torch.randn(B, 32)
    logits_ref, fused_ref = fusion_forward(sd, imu, vid, 4)
    (logits_ref * R).sum().backward()
    m = m.to(DEV)
    imu_g = imu.detach().to(DEV).requires_grad_(True)
    vid_g = vid.detach().to(DEV).requires_grad_(True)
    logits, fused = m(imu_g, vid_g)
    (logits * R.to(DEV)).sum().backward()
    tol_f, tol_g = (1e-5, 1e-4) if dtype == 'fp32' else (2e-2, 5e-2)
    assert rel(logits, logits_ref) < tol_f
    assert rel(fused, fused_ref) < tol_f
    assert rel(imu_g.grad, imu.grad) < tol_g
    assert rel(vid_g.grad, vid.grad) < tol_g
    for k, p in m.named_parameters():
        assert rel(p.grad, sd[k].grad) < tol_g, (k, rel(p.grad, sd[k].grad))


def test_fusion_classifier_end_to_end():
    from cmhar.config import Config
    from cmhar.fusion import CrossModalFusionClassifier
    from cmhar.losses import cross_entropy
    cfg = Config()
    cfg.data.video_frames_per_window = 4
    cfg.data.video_resize = (32, 32)
    m = cfg.model
    m.video_backbone = '/nonexistent/videomae-fusion'
    m.video_pretrained = False
    m.videomae_hidden_size, m.videomae_num_layers, m.videomae_num_heads = 128, 2, 2
    m.videomae_intermediate_size = 256
    torch.manual_seed(1)
    model = CrossModalFusionClassifier(cfg).to(DEV).train()
    logits = model(torch.randn(4, 6, 200, device=DEV), torch.randn(4, 4, 3, 32, 32, device=DEV))
    assert logits.shape == (4, cfg.model.num_classes)
    loss = cross_entropy(logits, torch.randint(0, cfg.model.num_classes, (4,), device=DEV))
    loss.backward()
    assert torch.isfinite(loss)
    for k, p in model.named_parameters():
        if k.startswith('video_encoder.projection.'):      # the token path bypasses the CLS projection
            continue
        assert p.grad is not None and torch.isfinite(p.grad).all(), k


def test_ood_evaluator_on_fusion_logits():
    """Config 5 on the fused model: OODEvaluator over (imu, video) batches scores the fusion classifier's class
    logits; energies equal −logsumexp of the returned logits, predictions their argmax (torch reference)."""
    import numpy as np
    from cmhar.config import Config
    from cmhar.fusion import CrossModalFusionClassifier
    from cmhar.ood import OODEvaluator
    cfg = Config()
    cfg.data.video_frames_per_window = 4
    cfg.data.video_resize = (32, 32)
    m = cfg.model
    m.video_backbone = '/nonexistent/videomae-ood'
    m.video_pretrained = False
    m.videomae_hidden_size, m.videomae_num_layers, m.videomae_num_heads = 128, 2, 2
    m.videomae_intermediate_size = 256
    torch.manual_seed(2)
    model = CrossModalFusionClassifier(cfg)
    batches = [{'imu': torch.randn(4, 6, 200), 'video': torch.randn(4, 4, 3, 32, 32), 'label': np.arange(4)}
               for _ in range(3)]
    preds, labels, logits, energies = OODEvaluator(model, cfg, device=DEV).predict(batches)
    assert logits.shape == (12, cfg.model.num_classes) and labels.shape == (12,)
    lt = torch.from_numpy(logits).double()
    assert np.allclose(energies, (-torch.logsumexp(lt, 1)).numpy(), rtol=1e-5, atol=1e-5)
    assert (preds == lt.argmax(1).numpy()).all()
