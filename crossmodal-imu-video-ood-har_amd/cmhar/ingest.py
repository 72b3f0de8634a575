"""Input ingestion on the GPU: the steps either side of the hot path's inputs.

* `clip_frame_indices` + `VideoClipIngest` replace `CrossModalDataset.load_video_clip` and its transform
  (src/data/datasets.py:49-58, 155-235): frame selection (host, the reference's np.linspace over the 5 s window)
  and ONE launch pair that resizes every selected decoded frame of a whole batch with Pillow's BILINEAR filter
  (bit-exact) and applies ToTensor + ImageNet Normalize, writing the (B,T,3,H,W) fp32 batch the model consumes.
  Decoding (cv2 in the reference) stays outside: frames arrive as RGB uint8 [n][H0][W0][3] in HBM.
* `IMUPreprocessor` replaces `MMEAPreprocessor.load_imu_data`'s unit conversion, `preprocess_imu` and
  `create_imu_windows` (src/data/preprocessing.py:176-183, 204-243) for a ragged batch of recordings in one
  launch pair: unit divisors, median filter (scipy.signal.medfilt semantics), per-recording z-score, windows.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np
import torch

from . import _lib as L
from ._lib import call, ptr

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def clip_frame_indices(start_frame: int, total_frames: int, fps: float, data_cfg) -> np.ndarray:
    """datasets.py:180-211: `video_frames_per_window` indices spread uniformly over the IMU window's duration."""
    if total_frames <= 0:
        raise ValueError('empty video (the reference returns a black clip)')
    if fps <= 1e-6:
        fps = float(getattr(data_cfg, 'video_fps', 25.0))
    window_sec = data_cfg.imu_window_size / float(data_cfg.imu_sampling_rate)
    window_frames = max(int(round(window_sec * fps)), 1)
    target = int(data_cfg.video_frames_per_window)
    start = int(start_frame)
    if start < 0:
        start = 0
    if start >= total_frames:
        start = max(total_frames - 1, 0)
    end = min(start + window_frames - 1, total_frames - 1)
    if end >= start:
        idx = np.linspace(start, end, target, dtype=int)
    else:
        idx = np.full((target,), start, dtype=int)
    return np.clip(idx, 0, total_frames - 1)


class VideoClipIngest:
    """(decoded frames, per-clip frame indices) → normalised clip batch, on the current HIP stream."""

    def __init__(self, size: Tuple[int, int] = (224, 224), mean=IMAGENET_MEAN, std=IMAGENET_STD,
                 channel_first: bool = False):
        self.H, self.W = int(size[0]), int(size[1])
        self.mean = (L.C.c_float * 3)(*mean)
        self.std = (L.C.c_float * 3)(*std)
        self.channel_first = channel_first

    def __call__(self, frames: torch.Tensor, frame_idx, out: torch.Tensor = None) -> torch.Tensor:
        if frames.dtype != torch.uint8 or frames.dim() != 4 or frames.shape[-1] != 3 or not frames.is_cuda:
            raise ValueError('frames: device uint8 [n][H0][W0][3] RGB expected')
        if frames.stride(3) != 1 or frames.stride(2) != 3 or frames.stride(1) != 3 * frames.shape[2]:
            raise ValueError('frames: each frame must be a dense H0 x W0 x 3 image')
        nf, H0, W0, _ = frames.shape
        idx = torch.as_tensor(frame_idx)
        if idx.dim() != 2:
            raise ValueError('frame_idx: (B, T) expected')
        if idx.numel() and (int(idx.min()) < 0 or int(idx.max()) >= nf):   # host check: no out-of-range gathers
            raise IndexError('frame index out of range')
        B, T = idx.shape
        idx = idx.to(device=frames.device, dtype=torch.int32).contiguous()
        shape = (B, 3, T, self.H, self.W) if self.channel_first else (B, T, 3, self.H, self.W)
        if out is None:
            out = torch.empty(shape, dtype=torch.float32, device=frames.device)
        elif tuple(out.shape) != shape or out.dtype != torch.float32 or not out.is_contiguous():
            raise ValueError(f'out: contiguous fp32 {shape} expected')
        nbytes = int(L.lib().cmhar_video_ingest_ws(B * T, H0, W0, self.H, self.W))
        ws = torch.empty(nbytes, dtype=torch.uint8, device=frames.device)
        call('cmhar_video_ingest', B, T, ptr(frames), frames.stride(0), H0, W0, ptr(idx), self.H, self.W, self.mean,
             self.std, int(self.channel_first), ptr(out), ptr(ws), nbytes, L.stream(frames.device))
        return out


class IMUPreprocessor:
    """GPU counterpart of MMEAPreprocessor's IMU path (preprocessing.py:156-243), driven by the same
    `config.data` fields (`median_filter_kernel`, `normalize_imu`, `imu_window_size`, `imu_stride`,
    `pad_short_sequences`, `Racc`, `Rgyro`)."""

    def __init__(self, config):
        self.data_cfg = config.data

    def _kernel(self):
        k = int(getattr(self.data_cfg, 'median_filter_kernel', 5))
        if k > 1 and k % 2 == 0:
            k += 1
        return max(k, 1)

    def unit_divisors(self, C: int, device) -> torch.Tensor:
        """load_imu_data's conversion (preprocessing.py:176-183): acc / Racc, gyro / Rgyro."""
        r = [float(getattr(self.data_cfg, 'Racc', 16384.0))] * 3 + [float(getattr(self.data_cfg, 'Rgyro', 16.4))] * 3
        return torch.tensor(r[:C] + [1.0] * max(0, C - 6), dtype=torch.float32, device=device)

    def window_plan(self, lengths: Sequence[int]) -> Tuple[List[int], List[int]]:
        """create_imu_windows (preprocessing.py:223-243): (recording, start) of every window."""
        win = int(getattr(self.data_cfg, 'imu_window_size', 250))
        stride = int(getattr(self.data_cfg, 'imu_stride', 125))
        pad = bool(getattr(self.data_cfg, 'pad_short_sequences', True))
        recs, starts = [], []
        for r, n in enumerate(lengths):
            if n < win:
                if not pad:
                    continue
                n = win
            for s in range(0, n - win + 1, stride):
                recs.append(r)
                starts.append(s)
        return recs, starts

    def process(self, recordings: Sequence[torch.Tensor], raw_units: bool = False, windows: bool = True):
        """recordings: list of (n_i, C) fp32 tensors (host or device).  raw_units: apply the Racc/Rgyro divisors
        first (load_imu_data).  Returns (windows [nW][C][win] fp32 device tensor, window recording ids, starts);
        windows=False returns the whole normalised series of each recording instead ([sum n_i][C] rows, like
        preprocess_imu's output stacked)."""
        if not recordings:
            raise ValueError('no recordings')
        C = int(recordings[0].shape[1])
        dev = torch.device('cuda', torch.cuda.current_device())
        lengths = [int(r.shape[0]) for r in recordings]
        if any(r.dim() != 2 or r.shape[1] != C for r in recordings):
            raise ValueError('recordings: (n_i, C) with a common C expected')
        raw = torch.cat([torch.as_tensor(r, dtype=torch.float32).to(dev) for r in recordings]).contiguous()
        offs = torch.tensor(np.concatenate([[0], np.cumsum(lengths)]), dtype=torch.int64, device=dev)
        total = int(raw.shape[0])
        if windows:
            recs, starts = self.window_plan(lengths)
            win = int(getattr(self.data_cfg, 'imu_window_size', 250))
        else:
            recs, starts = list(range(len(lengths))), [0] * len(lengths)
            win = max(lengths)
        wr = torch.tensor(recs, dtype=torch.int32, device=dev)
        ws_ = torch.tensor(starts, dtype=torch.int64, device=dev)
        out = torch.empty(len(recs), C, win, dtype=torch.float32, device=dev)
        scratch = torch.empty(int(L.lib().cmhar_imu_preprocess_ws(total, len(lengths), C)), dtype=torch.float32,
                              device=dev)
        div = self.unit_divisors(C, dev) if raw_units else None
        normalize = int(bool(getattr(self.data_cfg, 'normalize_imu', True)))
        call('cmhar_imu_preprocess', len(lengths), C, ptr(raw), ptr(offs), total, ptr(div), self._kernel(), normalize,
             len(recs), ptr(wr), ptr(ws_), win, ptr(out), ptr(scratch), L.stream(dev))
        if not windows:
            out = torch.cat([out[i, :, :n].t() for i, n in enumerate(lengths)])
        return out, recs, starts

    def preprocess_imu(self, imu) -> torch.Tensor:
        """preprocess_imu (preprocessing.py:204-221) of one (n, C) recording → (n, C) on the device."""
        out, _, _ = self.process([torch.as_tensor(imu)], windows=False)
        return out
