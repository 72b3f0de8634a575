"""cmhar — MI355X-native (gfx950 HIP) implementation of the CrossModal-IMU-Video-OOD-HAR pretraining hot path.

Public surface mirrors the reference (`src/models/models.py`, `src/models/losses.py`, `configs/config.py`):

    from cmhar.config import Config, CONFIG
    from cmhar.models import IMUEncoder, VideoEncoder, ProjectionHead, CrossModalModel, IMUClassifier
    from cmhar.losses import SigmoidContrastiveLoss
    from cmhar.optim import FusedAdamW, clip_grad_norm_
    from cmhar import dist

All compute goes through the C-ABI HIP library `cmhar/libcmhar.so` (include/cmhar.h); importing a model module
does not require a GPU, running one does.
"""
__version__ = '0.1.0'
