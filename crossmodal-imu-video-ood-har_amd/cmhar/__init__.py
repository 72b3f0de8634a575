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

import os as _os

# Kernel arguments in device memory (read by the command processor from HBM at dispatch instead of from host memory
# over PCIe).  The step launches ~500 kernels, many with a by-value CmharEpilogue or a layer table; measured in the
# bench step on one MI355X (tools/debug/kernarg_ab.sh, alternated runs): 605.6 -> 609.7 clips/s.  Takes effect only
# if set before the HIP runtime initialises (importing cmhar before the first CUDA call does that); an explicit
# setting by the user wins.
_os.environ.setdefault('HIP_FORCE_DEV_KERNARG', '1')
