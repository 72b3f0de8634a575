"""Ingestion oracles (oracle/ingest.py) pinned on the CPU:

* Pillow BILINEAR restatement vs Pillow itself (the library under the reference's torchvision Resize on PIL images,
  src/data/datasets.py:51-57) — bit-exact uint8 on down-, up- and mixed-scale sizes incl. 1080p → 224²;
* IMU preprocessing restatement vs the reference's own MMEAPreprocessor output (fixture g8, preprocessing.py:176-243);
* the host-side frame selection of load_video_clip (datasets.py:180-211)."""
import numpy as np
import pytest

from fixtures import load
from oracle import ingest as I


@pytest.mark.parametrize('H0,W0,H,W', [(90, 160, 32, 40), (48, 64, 224, 224), (240, 320, 224, 224),
                                       (1080, 1920, 224, 224), (100, 100, 99, 101), (7, 500, 13, 40),
                                       (224, 224, 112, 112), (1, 1, 3, 5)])
def test_pil_bilinear_restatement_is_bit_exact(H0, W0, H, W):
    from PIL import Image
    img = np.random.default_rng(H0 * 7 + W).integers(0, 256, (H0, W0, 3), dtype=np.uint8)
    want = np.asarray(Image.fromarray(img).resize((W, H), Image.BILINEAR))
    assert np.array_equal(I.pil_bilinear_resize(img, (H, W)), want)


def test_imu_preprocessing_restatement_matches_reference():
    fx = load('g8_imu_preprocessing')
    for i, n in enumerate(fx['lengths']):
        proc = I.preprocess_imu(fx[f'conv{i}'], 5, True)
        np.testing.assert_allclose(proc, fx[f'proc{i}'], rtol=0, atol=2e-6)
        wins = np.stack(I.create_imu_windows(proc, 250, 125))
        assert wins.shape == fx[f'windows{i}'].shape
        np.testing.assert_allclose(wins, fx[f'windows{i}'], rtol=0, atol=2e-6)


def test_medfilt_restatement_matches_scipy():
    from scipy import signal
    x = np.random.default_rng(3).normal(size=301).astype(np.float32)
    x[50:80] = x[50]
    for k in (1, 3, 5, 9):
        assert np.array_equal(I.medfilt_zero_pad(x, k), signal.medfilt(x, k).astype(np.float32))


def test_clip_frame_indices_semantics():
    from cmhar.config import Config
    from cmhar.ingest import clip_frame_indices
    d = Config().data                       # 250-sample windows at 50 Hz = 5 s; 16 frames
    idx = clip_frame_indices(10, 1000, 25.0, d)
    assert list(idx) == list(np.linspace(10, 134, 16, dtype=int))
    assert list(clip_frame_indices(990, 1000, 25.0, d)) == list(np.linspace(990, 999, 16, dtype=int))
    assert (clip_frame_indices(-5, 100, 0.0, d) >= 0).all()          # unknown fps → video_fps (25)
    assert list(clip_frame_indices(5000, 50, 30.0, d)) == [49] * 16   # start past the end → last frame
