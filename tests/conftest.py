import os
import sys

import pytest

# tests build the VideoMAE architecture with random weights when the default hub checkpoint is named (no network)
os.environ.setdefault('CMHAR_ALLOW_RANDOM_INIT', '1')

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_ROOT = os.path.join(REPO, 'crossmodal-imu-video-ood-har_amd')
for p in (REPO, PKG_ROOT, os.path.join(REPO, 'tests', 'golden'), os.path.join(REPO, 'tests')):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (run with -m gpu on the GPU box)')
    config.addinivalue_line('markers', 'slow: long CPU test')


def _has_gpu():
    """Probe without initialising HIP (tests that launch their own GPU processes need a clean parent):
    torch.cuda.device_count() does not create a context on this image, torch.cuda.is_available() does."""
    try:
        import torch
        return torch.cuda.device_count() > 0
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason='no GPU in this container')
    for it in items:
        if 'gpu' in it.keywords:
            it.add_marker(skip)
