"""Ingestion throughput on one MI355X, with the reference's CPU path timed beside it.

Video: a pool of decoded 1080p RGB frames resident in HBM; every step ingests one batch of 32 clips × 16 frames
(frame indices from the reference's np.linspace selection over 5 s windows at 25 fps) → (32,16,3,224,224) fp32.
HBM roofline of the pair of kernels: algorithmic bytes per output frame = the source rows read once (H0·W0·3 B) +
the fp32 output (3·224·224·4 B); the RGBX intermediate of the two-pass resample (rows·224·4 B, written + read) is
implementation traffic and reported separately.
IMU: 256 recordings of 1000–3000 samples (20–60 s at 50 Hz) → 250/125 windows, one launch pair per batch.
CPU baseline: the reference's per-frame transform (Pillow resize + ToTensor/Normalize as numpy) and its IMU path
(scipy medfilt + numpy z-score + windows), single process, on a bounded sample.
    python tools/bench_ingest.py            → one JSON line
"""
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'crossmodal-imu-video-ood-har_amd'))
sys.path.insert(0, REPO)
from cmhar.config import Config  # noqa: E402
from cmhar.ingest import IMUPreprocessor, VideoClipIngest, clip_frame_indices  # noqa: E402

PEAK_HBM = 8000.0   # GB/s, MI355X_MICROARCH.md


def timed(fn, reps):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps / 1e3


def main():
    dev = torch.device('cuda')
    cfg = Config()
    cfg.model.allow_random_init = True   # synthetic benchmark: random-init weights
    H0, W0, H, W, B, T = 1080, 1920, 224, 224, 32, 16
    npool = 400                                       # 16 s of 25 fps video, 2.5 GB of decoded frames
    g = torch.Generator(device=dev).manual_seed(0)
    frames = torch.randint(0, 256, (npool, H0, W0, 3), dtype=torch.uint8, device=dev, generator=g)
    starts = np.linspace(0, npool - 126, B).astype(int)
    idx = np.stack([clip_frame_indices(s, npool, 25.0, cfg.data) for s in starts])
    ing = VideoClipIngest((H, W))
    out = torch.empty(B, T, 3, H, W, device=dev)
    sec = timed(lambda: ing(frames, idx, out=out), 20)
    nfr = B * T
    alg = nfr * (H0 * W0 * 3 + 3 * H * W * 4)
    inter = nfr * 2 * H0 * W * 4
    video = {'clips_per_s': round(B / sec, 1), 'frames_per_s': round(nfr / sec, 1), 'ms_per_batch': round(sec * 1e3, 3),
             'algorithmic_GBps': round(alg / sec / 1e9, 1), 'with_intermediate_GBps': round((alg + inter) / sec / 1e9, 1),
             'roofline_frac': round(alg / sec / 1e9 / PEAK_HBM, 4)}

    # IMU: ragged recordings
    rng = np.random.default_rng(1)
    recs = [torch.tensor(np.round(rng.normal(0, 9000, (int(n), 6))).astype(np.float32), device=dev)
            for n in rng.integers(1000, 3000, 256)]
    pre = IMUPreprocessor(cfg)
    res = {}

    def imu_step():
        res['w'] = pre.process(recs, raw_units=True)
    isec = timed(imu_step, 20)
    nwin = res['w'][0].shape[0]
    tot = sum(int(r.shape[0]) for r in recs)
    imu = {'recordings_per_s': round(256 / isec, 1), 'windows_per_s': round(nwin / isec, 1),
           'ms_per_batch': round(isec * 1e3, 3), 'samples': tot, 'windows': nwin}

    # CPU baselines (bounded samples)
    from PIL import Image
    from oracle import ingest as OI
    fr = frames[:8].cpu().numpy()
    m = np.asarray((0.485, 0.456, 0.406), np.float32).reshape(3, 1, 1)
    s = np.asarray((0.229, 0.224, 0.225), np.float32).reshape(3, 1, 1)
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < 10.0:
        f = fr[n % 8]
        r = np.asarray(Image.fromarray(f).resize((W, H), Image.BILINEAR)).transpose(2, 0, 1).astype(np.float32) / 255.0
        _ = (r - m) / s
        n += 1
    cpu_fps = n / (time.perf_counter() - t0)
    raw = [r.cpu().numpy() for r in recs[:64]]
    t0 = time.perf_counter()
    k = 0
    while time.perf_counter() - t0 < 10.0:
        x = raw[k % 64]
        conv = np.concatenate([x[:, :3] / 16384.0, x[:, 3:] / 16.4], axis=1).astype(np.float32)
        from scipy import signal
        flt = np.stack([signal.medfilt(conv[:, c], 5) for c in range(6)], axis=1).astype(np.float32)
        z = (flt - flt.mean(0, keepdims=True)) / (flt.std(0, keepdims=True) + 1e-8)
        _ = OI.create_imu_windows(z.astype(np.float32))
        k += 1
    cpu_rps = k / (time.perf_counter() - t0)
    print(json.dumps({'metric': 'ingestion throughput (video clips / IMU recordings per second)',
                      'video_1080p_to_224': video, 'imu_preprocess': imu,
                      'cpu_baseline': {'video_frames_per_s': round(cpu_fps, 1),
                                       'video_clips_per_s': round(cpu_fps / T, 2),
                                       'imu_recordings_per_s': round(cpu_rps, 1), 'cores': 1, 'kind': 'reference',
                                       'sample': 'Pillow BILINEAR resize + ToTensor/Normalize (numpy) of 1080p frames '
                                                 'for 10 s; scipy medfilt + numpy z-score + windows for 10 s'}}),
          flush=True)


if __name__ == '__main__':
    main()
