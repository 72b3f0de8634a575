"""Configuration dataclasses with the reference's field names.

Mirrors `configs/config.py:49-185` (DataConfig, ModelConfig, TrainingConfig, EvalConfig, Config) so that
`config.data.*`, `config.model.*` and `config.training.*` drive the drop-in modules exactly as they drive the
reference's.  Differences, all deliberate:

* no filesystem side effects at import (the reference's `PathConfig.__post_init__` mkdirs `./outputs/...`,
  `config.py:33-46`); `PathConfig` here only computes paths, `Config.make_dirs()` creates them on request;
* a few knobs the reference reads through `getattr(..., default)` are declared (`video_channel_first`,
  `trainer.py:108`);
* MI355X knobs live in `ModelConfig`: `compute_dtype` ("bf16" throughput mode / "fp32" parity mode) and
  the VideoMAE geometry used when `video_backbone` names a hub checkpoint that cannot be fetched offline.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from pathlib import Path
from typing import List, Optional


@dataclass
class PathConfig:
    """Paths (reference `config.py:9-46`), without the mkdir-on-construct side effect."""
    is_kaggle: bool = os.path.exists('/kaggle')
    base_input: Path = field(default_factory=lambda: Path('/kaggle/input/dataset-har/UESTC-MMEA-CL')
                             if os.path.exists('/kaggle') else Path('./data/UESTC-MMEA-CL'))
    base_output: Path = field(default_factory=lambda: Path('/kaggle/working')
                              if os.path.exists('/kaggle') else Path('./outputs'))
    train_file: str = 'train.txt'
    val_file: str = 'val.txt'
    test_file: str = 'test.txt'
    sensor_dir: str = 'sensor'
    video_dir: str = 'video'

    def __post_init__(self):
        self.base_input = Path(self.base_input)
        self.base_output = Path(self.base_output)
        self.preprocessed_dir = self.base_output / 'preprocessed'
        self.checkpoints_dir = self.base_output / 'checkpoints'
        self.logs_dir = self.base_output / 'logs'
        self.results_dir = self.base_output / 'results'

    def make_dirs(self):
        for d in [self.base_output, self.preprocessed_dir, self.checkpoints_dir, self.logs_dir, self.results_dir]:
            d.mkdir(parents=True, exist_ok=True)


@dataclass
class DataConfig:
    """Reference `config.py:49-70`."""
    imu_window_size: int = 250
    imu_stride: int = 125
    imu_sampling_rate: int = 50
    imu_channels: int = 6
    video_fps: int = 25
    video_frames_per_window: int = 16
    video_resize: tuple = (224, 224)
    normalize_imu: bool = True
    median_filter_kernel: int = 5
    use_augmentation: bool = False
    jitter_strength: float = 0.1
    time_warp_strength: float = 0.2
    video_channel_first: bool = False   # read via getattr in the reference (trainer.py:108, datasets.py:73)


@dataclass
class ModelConfig:
    """Reference `config.py:73-96` plus the MI355X build's compute-mode knobs."""
    imu_patch_size: int = 16
    imu_stride: int = 16
    imu_d_model: int = 128
    imu_nhead: int = 8
    imu_num_layers: int = 4
    imu_dropout: float = 0.1
    video_backbone: str = 'MCG-NJU/videomae-base-ssv2'
    video_pretrained: bool = True
    video_d_model: int = 768
    projection_dim: int = 256
    projection_hidden_dim: int = 512
    num_classes: int = 32
    classifier_hidden_dims: List[int] = field(default_factory=lambda: [256, 128])
    classifier_dropout: float = 0.3
    # ---- MI355X build knobs (not in the reference) ----
    compute_dtype: str = 'bf16'          # 'bf16' (MFMA bf16, fp32 accumulate), 'fp32' (exact-f32 parity mode) or
    #                                      'fp16' (MFMA fp16, fp32 accumulate; VideoMAE inference only — config 5)
    # video_pretrained=True with a hub name that cannot be loaded offline raises (as from_pretrained would);
    # True (or env CMHAR_ALLOW_RANDOM_INIT=1) builds the configured architecture with random weights instead
    # (benchmarks and tests, which use synthetic data)
    allow_random_init: bool = False
    # VideoMAE geometry used when the backbone cannot be loaded from a local directory.  None -> taken from
    # DataConfig (frames / resize) and the videomae-base defaults (hidden 768, 12 layers, 12 heads, 3072).
    videomae_hidden_size: int = 768
    videomae_num_layers: int = 12
    videomae_num_heads: int = 12
    videomae_intermediate_size: int = 3072
    videomae_patch_size: int = 16
    videomae_tubelet_size: int = 2
    videomae_layer_norm_eps: float = 1e-12
    videomae_use_mean_pooling: bool = True
    videomae_qkv_bias: bool = True
    videomae_num_frames: Optional[int] = None
    videomae_image_size: Optional[int] = None


@dataclass
class TrainingConfig:
    """Reference `config.py:99-130`."""
    seed: int = 42
    device: str = 'cuda'
    num_workers: int = 2
    pretrain_epochs: int = 10
    pretrain_batch_size: int = 16
    pretrain_lr: float = 1e-4
    pretrain_weight_decay: float = 0.01
    pretrain_warmup_epochs: int = 5
    temperature: float = 0.07
    use_sigmoid_loss: bool = True
    train_epochs: int = 100
    train_batch_size: int = 64
    train_lr_encoder: float = 1e-6
    train_lr_head: float = 1e-3
    patience: int = 15
    min_delta: float = 0.001
    save_every: int = 5
    save_best_only: bool = True


@dataclass
class EvalConfig:
    """Reference `config.py:133-146`."""
    metrics: List[str] = field(default_factory=lambda: [
        'accuracy', 'balanced_accuracy', 'f1_macro', 'precision_macro', 'recall_macro'])
    few_shot_samples: List[int] = field(default_factory=lambda: [10, 20, 50, 100])
    few_shot_runs: int = 5
    eval_modes: List[str] = field(default_factory=lambda: ['linear_probe', 'finetune'])


class Config:
    """Reference `config.py:149-181`."""

    def __init__(self):
        self.paths = PathConfig()
        self.data = DataConfig()
        self.model = ModelConfig()
        self.training = TrainingConfig()
        self.eval = EvalConfig()

    def to_dict(self):
        return {'paths': vars(self.paths), 'data': vars(self.data), 'model': vars(self.model),
                'training': vars(self.training), 'eval': vars(self.eval)}

    def save(self, path: str):
        import json
        with open(path, 'w') as f:
            json.dump(self.to_dict(), f, indent=2, default=str)

    def make_dirs(self):
        self.paths.make_dirs()


CONFIG = Config()
