"""Ingestion kernels on the MI355X (csrc/ingest.hip) against the pinned oracles:

* video clip ingestion vs Pillow BILINEAR + ToTensor + Normalize (oracle/ingest.py, bit-exact vs Pillow): the fp32
  outputs must be IDENTICAL (integer resample, then the same fp32 division/normalisation);
* IMU preprocessing vs the reference's own MMEAPreprocessor outputs (fixture g8): median filter exact, z-score
  within 2e-6 absolute (the mean/std sums run in a different order than numpy's)."""
import numpy as np
import pytest
import torch

from fixtures import load
from oracle import ingest as I

pytestmark = pytest.mark.gpu
DEV = 'cuda'


@pytest.mark.parametrize('H0,W0,H,W,channel_first', [(240, 320, 224, 224, False), (1080, 1920, 224, 224, False),
                                                     (60, 80, 112, 112, True), (57, 91, 33, 47, False)])
def test_video_ingest_bit_exact_vs_pillow(H0, W0, H, W, channel_first):
    from cmhar.ingest import VideoClipIngest
    rng = np.random.default_rng(H0 + W)
    nf = 6
    frames = rng.integers(0, 256, (nf, H0, W0, 3), dtype=np.uint8)
    idx = np.array([[0, 2, 2, 5], [1, 3, 4, 5]])
    out = VideoClipIngest((H, W), channel_first=channel_first)(torch.from_numpy(frames).to(DEV), idx)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    for b in range(idx.shape[0]):
        want = I.clip_transform(frames[idx[b]], (H, W))            # (T, 3, H, W)
        g = got[b].transpose(1, 0, 2, 3) if channel_first else got[b]
        assert np.array_equal(g, want), (b, np.abs(g - want).max())


def test_video_ingest_rejects_bad_indices():
    from cmhar.ingest import VideoClipIngest
    frames = torch.zeros(3, 16, 16, 3, dtype=torch.uint8, device=DEV)
    with pytest.raises(IndexError):
        VideoClipIngest((8, 8))(frames, np.array([[0, 3]]))


def test_imu_preprocess_matches_reference():
    from cmhar.config import Config
    from cmhar.ingest import IMUPreprocessor
    fx = load('g8_imu_preprocessing')
    n = len(fx['lengths'])
    pre = IMUPreprocessor(Config())
    # raw sensor counts → unit conversion + filter + z-score + windows, whole ragged batch in one launch pair
    wins, recs, starts = pre.process([torch.tensor(fx[f'raw{i}']) for i in range(n)], raw_units=True)
    torch.cuda.synchronize()
    got = wins.cpu().numpy()
    for i in range(n):
        want = fx[f'windows{i}']                                   # (nw, 250, 6) from the reference
        sel = [j for j, r in enumerate(recs) if r == i]
        assert len(sel) == want.shape[0]
        np.testing.assert_allclose(got[sel].transpose(0, 2, 1), want, rtol=0, atol=2e-6)
    # preprocess_imu of a single already-converted recording
    proc = pre.preprocess_imu(torch.tensor(fx['conv2'])).cpu().numpy()
    np.testing.assert_allclose(proc, fx['proc2'], rtol=0, atol=2e-6)
