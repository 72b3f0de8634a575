"""Fixture loading helpers (golden vectors produced by tests/golden/make_golden.py)."""
from __future__ import annotations

import json
import os

import numpy as np
import torch

from seeded import seeded_state_dict

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def load(name):
    return np.load(os.path.join(GOLDEN, name + '.npz'), allow_pickle=False)


def fixture_state_dict(fx, seed=None):
    keys = json.loads(str(fx['keys']))
    shapes = json.loads(str(fx['shapes']))
    tmpl = {}
    for k, s in zip(keys, shapes):
        dt = torch.int64 if k.endswith('num_batches_tracked') else torch.float32
        tmpl[k] = torch.empty(s, dtype=dt)
    return seeded_state_dict(tmpl, int(fx['seed']) if seed is None else seed)


def fixture_config(fx):
    from cmhar.config import Config
    cfg = Config()
    if 'config' in fx:
        for sect, kv in json.loads(str(fx['config'])).items():
            for k, v in kv.items():
                if isinstance(v, list) and k == 'video_resize':
                    v = tuple(v)
                if k == 'video_backbone':
                    v = '/nonexistent/videomae-fixture'     # the generator's temp dir; geometry comes from videomae_*
                setattr(getattr(cfg, sect), k, v)
    return cfg


def oracle_mcfg(cfg):
    m = cfg.model
    return {'imu_patch_size': m.imu_patch_size, 'imu_stride': m.imu_stride, 'imu_nhead': m.imu_nhead,
            'imu_num_layers': m.imu_num_layers, 'video_num_heads': m.videomae_num_heads,
            'video_patch_size': m.videomae_patch_size, 'video_tubelet': m.videomae_tubelet_size,
            'video_eps': m.videomae_layer_norm_eps, 'video_use_mean_pooling': m.videomae_use_mean_pooling,
            'classifier_hidden_dims': list(m.classifier_hidden_dims)}


def t(x):
    return torch.from_numpy(np.asarray(x)).clone()
