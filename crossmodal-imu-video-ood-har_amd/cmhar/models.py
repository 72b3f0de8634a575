"""Drop-in replacements for the reference's `src/models/models.py` API, running on the cmhar HIP library.

    from cmhar.models import IMUEncoder, VideoEncoder, ProjectionHead, CrossModalModel, IMUClassifier

Constructor signatures, attributes, forward() outputs and state_dict() keys match the reference
(`models.py:16-348`), so `CrossModalTrainer` / `ClassificationTrainer` / `Evaluator` (src/train/trainer.py,
src/eval/evaluator.py) and checkpoints written by the reference work unchanged.  Compute runs in
`config.model.compute_dtype` ('bf16': MFMA bf16 with fp32 accumulation for the VideoMAE backbone — the FLOP-heavy
part; 'fp32': exact fp32 everywhere, the parity mode).  The IMU encoder, heads, normalisation and loss are always
fp32 (they are latency- not FLOP-bound).
"""
from __future__ import annotations

import math
import os
import warnings

import torch
import torch.nn as nn

from . import kernels as K
from .heads import ProjectionHead, l2_normalize, run_head, _Seeds
from .imu import IMUEncoder, PatchEmbedding
from .cnn2d import MobileNetV2Features, ResNet18Features, run_cnn2d
from .fusion import _TokenMeanFn
from .r3d import R3D18, run_r3d
from .videomae import VideoMAEBackbone, default_videomae_config, run_backbone

__all__ = ['PatchEmbedding', 'IMUEncoder', 'VideoEncoder', 'ProjectionHead', 'CrossModalModel', 'IMUClassifier']


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        return K.linear(x, weight.detach(), None if bias is None else bias.detach())

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.contiguous()
        dx = K.linear_dgrad(dy, w.detach()) if ctx.needs_input_grad[0] else None
        dw = K.linear_wgrad(dy, x) if ctx.needs_input_grad[1] else None
        db = K.colsum(dy) if ctx.has_bias and ctx.needs_input_grad[2] else None
        return dx, dw, db


def linear_fp32(x, lin: nn.Linear):
    x = x.contiguous().float()
    if torch.is_grad_enabled() and (x.requires_grad or lin.weight.requires_grad):
        return _LinearFn.apply(x, lin.weight, lin.bias)
    return K.linear(x, lin.weight.detach(), None if lin.bias is None else lin.bias.detach())


def _videomae_geometry(config):
    m, d = config.model, config.data
    frames = m.videomae_num_frames or d.video_frames_per_window
    image = m.videomae_image_size or (d.video_resize[0] if isinstance(d.video_resize, (tuple, list)) else d.video_resize)
    return default_videomae_config(image_size=image, patch_size=m.videomae_patch_size, num_frames=frames,
                                   tubelet_size=m.videomae_tubelet_size, hidden_size=m.videomae_hidden_size,
                                   num_hidden_layers=m.videomae_num_layers, num_attention_heads=m.videomae_num_heads,
                                   intermediate_size=m.videomae_intermediate_size,
                                   layer_norm_eps=m.videomae_layer_norm_eps, qkv_bias=m.videomae_qkv_bias,
                                   use_mean_pooling=m.videomae_use_mean_pooling)


class VideoEncoder(nn.Module):
    """models.py:137-216.  VideoMAE branch: a local HF-format directory is loaded (config.json + safetensors / .bin
    via weights-only loaders); a hub name cannot be fetched offline, so the VideoMAE architecture is built from
    `config.model.videomae_*` / the data geometry with HF's random init.  'resnet18' / 'mobilenet_v2': the per-frame
    torchvision CNNs (cmhar.cnn2d, torchvision state_dict names).  'r3d_18': the north_star R3D-18 extension."""

    def __init__(self, config):
        super().__init__()
        self.config = config
        model_cfg = config.model
        vb = model_cfg.video_backbone
        self.is_videomae = False
        dt = getattr(model_cfg, 'compute_dtype', 'bf16')
        if isinstance(vb, str) and ('videomae' in vb.lower() or '/' in vb):
            self.is_videomae = True
            if os.path.isdir(vb) and os.path.exists(os.path.join(vb, 'config.json')):
                self.backbone = VideoMAEBackbone.from_pretrained(vb, compute_dtype=dt)
            else:
                if model_cfg.video_pretrained:
                    allow = bool(getattr(model_cfg, 'allow_random_init', False)) or \
                        os.environ.get('CMHAR_ALLOW_RANDOM_INIT', '') == '1'
                    if not allow:   # VideoMAEModel.from_pretrained(vb) (models.py:157) would fail here too
                        raise OSError(f'VideoMAE checkpoint {vb!r} cannot be loaded (not a local HF directory '
                                      f'and no network); give a local directory, set video_pretrained=False, or '
                                      f'opt in to random weights with model.allow_random_init=True / '
                                      f'CMHAR_ALLOW_RANDOM_INIT=1')
                    warnings.warn(f'VideoMAE checkpoint {vb!r} is not available offline; using a randomly '
                                  f'initialised backbone of the configured geometry (allow_random_init)')
                self.backbone = VideoMAEBackbone(_videomae_geometry(config), compute_dtype=dt)
            self.feature_dim = self.backbone.config.hidden_size
        elif dt == 'fp16':
            raise ValueError("compute_dtype 'fp16' (inference path) covers the VideoMAE backbone only")
        elif vb == 'r3d_18':
            # north_star extension (no reference code): torchvision-layout R3D-18 on the HIP conv3d path
            self.backbone = R3D18(None, compute_dtype=dt)
            self.feature_dim = self.backbone.feature_dim
        elif vb in ('resnet18', 'mobilenet_v2'):
            # models.py:163-173: torchvision resnet18 children()[:-2] / mobilenet_v2 .features, run per frame
            if model_cfg.video_pretrained:
                allow = bool(getattr(model_cfg, 'allow_random_init', False)) or \
                    os.environ.get('CMHAR_ALLOW_RANDOM_INIT', '') == '1'
                if not allow:   # models.resnet18(pretrained=True) downloads ImageNet weights: not possible offline
                    raise OSError(f'{vb}: ImageNet weights cannot be fetched offline; set video_pretrained=False '
                                  f'(then load a torchvision state_dict into video_encoder.backbone), or opt in to '
                                  f'random weights with model.allow_random_init=True / CMHAR_ALLOW_RANDOM_INIT=1')
                warnings.warn(f'{vb}: pretrained ImageNet weights are not available offline; random init '
                              f'(allow_random_init)')
            self.backbone = (ResNet18Features if vb == 'resnet18' else MobileNetV2Features)(compute_dtype=dt)
            self.feature_dim = self.backbone.feature_dim
        else:
            raise ValueError(f'Backbone inconnu: {vb}')
        self.projection = nn.Linear(self.feature_dim, model_cfg.video_d_model)
        if vb in ('resnet18', 'mobilenet_v2'):
            self.temporal_pool = nn.AdaptiveAvgPool1d(1)            # models.py:182-183 (no parameters)

    def forward(self, x):
        """x (B, T, C, H, W) → (B, video_d_model)."""
        if x.dim() != 5:
            raise ValueError(f'expected (B, T, C, H, W) video, got {tuple(x.shape)}')
        if isinstance(self.backbone, (ResNet18Features, MobileNetV2Features)):
            # models.py:208-216: per-frame CNN + 2-D average pool → per-frame projection → mean over the T frames
            B, T = x.shape[:2]
            feats = linear_fp32(run_cnn2d(self.backbone, x, self.training), self.projection)   # (B·T, d)
            return _TokenMeanFn.apply(feats, B, T)
        if not self.is_videomae:                                  # r3d_18: pooled 3-D CNN features
            return linear_fp32(run_r3d(self.backbone, x, self.training), self.projection)
        feat = run_backbone(self.backbone, x, token0_only=True)   # last_hidden_state[:, 0]  (models.py:201)
        return linear_fp32(feat, self.projection)                 # models.py:202


class CrossModalModel(nn.Module):
    """models.py:239-291."""

    def __init__(self, config):
        super().__init__()
        self.config = config
        model_cfg = config.model
        self.imu_encoder = IMUEncoder(config)
        self.video_encoder = VideoEncoder(config)
        self.imu_proj = ProjectionHead(model_cfg.imu_d_model, model_cfg.projection_hidden_dim,
                                       model_cfg.projection_dim)
        self.video_proj = ProjectionHead(model_cfg.video_d_model, model_cfg.projection_hidden_dim,
                                         model_cfg.projection_dim)
        self.temperature = nn.Parameter(torch.ones([]) * math.log(10))
        self.bias = nn.Parameter(torch.ones([]) * -10)
        # The IMU branch (encoder + head, ~0.02 GFLOP/clip, launch/latency bound) runs on its own HIP stream,
        # concurrently with the VideoMAE backbone; autograd replays each node's backward on the stream its
        # forward ran on, so the IMU backward overlaps the video backward too.
        self.overlap_imu = True
        self._side = {}

    def _imu_branch(self, imu):
        imu_feat, _ = self.imu_encoder(imu)
        return l2_normalize(self.imu_proj(imu_feat))

    def forward(self, imu, video):
        if self.overlap_imu and imu.is_cuda:
            cur = torch.cuda.current_stream(imu.device)
            side = self._side.get(imu.device)
            if side is None:
                # CMHAR_IMU_STREAM_PRIORITY=-1: the side stream at high dispatch priority (A/B knob; default 0)
                side = self._side[imu.device] = torch.cuda.Stream(
                    imu.device, priority=int(os.environ.get('CMHAR_IMU_STREAM_PRIORITY', '0')))
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                imu_out = self._imu_branch(imu)
            video_out = l2_normalize(self.video_proj(self.video_encoder(video)))
            cur.wait_stream(side)
            imu_out.record_stream(cur)
            return imu_out, video_out
        imu_out = self._imu_branch(imu)
        return imu_out, l2_normalize(self.video_proj(self.video_encoder(video)))


class IMUClassifier(nn.Module):
    """models.py:296-348."""

    def __init__(self, imu_encoder, config, freeze_encoder=False):
        super().__init__()
        self.imu_encoder = imu_encoder
        self.config = config
        model_cfg = config.model
        if freeze_encoder:
            for param in self.imu_encoder.parameters():
                param.requires_grad = False
        layers = []
        in_dim = model_cfg.imu_d_model
        for hidden_dim in model_cfg.classifier_hidden_dims:
            layers.extend([nn.Linear(in_dim, hidden_dim), nn.BatchNorm1d(hidden_dim), nn.ReLU(inplace=True),
                           nn.Dropout(model_cfg.classifier_dropout)])
            in_dim = hidden_dim
        layers.append(nn.Linear(in_dim, model_cfg.num_classes))
        self.classifier = nn.Sequential(*layers)
        self._seeds = _Seeds()

    def forward(self, imu):
        with torch.set_grad_enabled(self.training or not self.freeze_encoder):
            imu_feat, _ = self.imu_encoder(imu)
        return run_head(self.classifier, imu_feat, self.training, self._seeds)

    @property
    def freeze_encoder(self):
        return not next(self.imu_encoder.parameters()).requires_grad

    def unfreeze_encoder(self):
        for param in self.imu_encoder.parameters():
            param.requires_grad = True
