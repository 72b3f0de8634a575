"""ORACLE — test infrastructure only.  CPU restatements of the ingestion steps around the hot path's inputs.

* `pil_bilinear_resize`  — Pillow 12.2.0's BILINEAR resample of an RGB uint8 image (the engine under the
  reference's `transforms.Resize` on a PIL image, src/data/datasets.py:51-57), restated from Pillow's
  src/libImaging/Resample.c: `precompute_coeffs` (triangle filter, support widened by the downscale factor,
  bounds rounded by truncation of x + 0.5), `normalize_coeffs_8bpc` (22-bit fixed point), horizontal pass over
  the source rows the vertical pass needs, uint8 clip, vertical pass, uint8 clip.  Pinned against Pillow itself
  (tests/test_ingest_cpu.py).
* `clip_transform`       — ToTensor (÷255) + Normalize(ImageNet mean/std) in fp32 (datasets.py:52-58).
* `preprocess_imu` / `create_imu_windows` — src/data/preprocessing.py:204-243 (median filter with zero padding =
  scipy.signal.medfilt, per-channel z-score with population std + 1e-8, 250/125 windows with zero padding of short
  recordings).  Pinned against the reference's own functions (fixture g8, tests/golden/make_golden.py).
"""
from __future__ import annotations

import math

import numpy as np

PREC = 22


def _coeffs(in_size: int, out_size: int):
    scale = in_size / out_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), dtype=np.int64)
    kk = np.zeros((out_size, ksize), dtype=np.int64)
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        ss = 1.0 / filterscale
        xmin = max(int(center - support + 0.5), 0)          # C (int) cast: truncation toward zero
        xmax = min(int(center + support + 0.5), in_size) - xmin
        w = []
        for x in range(xmax):
            t = abs((x + xmin - center + 0.5) * ss)
            w.append(1.0 - t if t < 1.0 else 0.0)
        ww = 0.0
        for v in w:
            ww += v
        for x in range(xmax):
            k = w[x] / ww if ww != 0.0 else w[x]
            kk[xx, x] = int(-0.5 + k * (1 << PREC)) if k < 0 else int(0.5 + k * (1 << PREC))
        bounds[xx] = (xmin, xmax)
    return bounds, kk


def _clip8(v: np.ndarray) -> np.ndarray:
    return np.where(v >= (1 << PREC << 8), 255, np.where(v <= 0, 0, v >> PREC)).astype(np.uint8)


def pil_bilinear_resize(img: np.ndarray, size_hw) -> np.ndarray:
    """img: uint8 (H0, W0, 3) → uint8 (H, W, 3), Pillow BILINEAR semantics."""
    H0, W0, _ = img.shape
    H, W = size_hw
    bh, kh = _coeffs(W0, W)
    bv, kv = _coeffs(H0, H)
    y0 = int(bv[0, 0])
    y1 = int(bv[-1, 0] + bv[-1, 1])
    src = img[y0:y1].astype(np.int64)
    tmp = np.zeros((y1 - y0, W, 3), dtype=np.int64)
    for xx in range(W):
        xmin, n = bh[xx]
        acc = np.full((y1 - y0, 3), 1 << (PREC - 1), dtype=np.int64)
        acc += (src[:, xmin:xmin + n, :] * kh[xx, :n][None, :, None]).sum(axis=1)
        tmp[:, xx] = _clip8(acc)
    out = np.zeros((H, W, 3), dtype=np.uint8)
    for yy in range(H):
        ymin, n = bv[yy]
        ymin -= y0
        acc = np.full((W, 3), 1 << (PREC - 1), dtype=np.int64)
        acc += (tmp[ymin:ymin + n] * kv[yy, :n][:, None, None]).sum(axis=0)
        out[yy] = _clip8(acc)
    return out


def clip_transform(frames_u8: np.ndarray, size_hw, mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225)):
    """(T, H0, W0, 3) uint8 → (T, 3, H, W) fp32: Resize → ToTensor → Normalize."""
    outs = []
    m = np.asarray(mean, dtype=np.float32).reshape(3, 1, 1)
    s = np.asarray(std, dtype=np.float32).reshape(3, 1, 1)
    for f in frames_u8:
        r = pil_bilinear_resize(f, size_hw).transpose(2, 0, 1).astype(np.float32) / np.float32(255.0)
        outs.append((r - m) / s)
    return np.stack(outs)


def medfilt_zero_pad(x: np.ndarray, k: int) -> np.ndarray:
    """scipy.signal.medfilt(x, k) for 1-D x: median over a centred window, zeros outside."""
    h = k // 2
    p = np.concatenate([np.zeros(h, x.dtype), x, np.zeros(h, x.dtype)])
    win = np.lib.stride_tricks.sliding_window_view(p, k)
    return np.sort(win, axis=1)[:, h].astype(x.dtype)


def preprocess_imu(imu: np.ndarray, k: int = 5, normalize: bool = True) -> np.ndarray:
    """preprocessing.py:204-221 on an (n, C) float32 recording."""
    imu = np.asarray(imu, dtype=np.float32)
    if k > 1:
        if k % 2 == 0:
            k += 1
        imu = np.stack([medfilt_zero_pad(imu[:, c], k) for c in range(imu.shape[1])], axis=1)
    if normalize:
        mean = imu.mean(axis=0, keepdims=True)
        std = imu.std(axis=0, keepdims=True) + 1e-8
        imu = (imu - mean) / std
    return imu.astype(np.float32)


def create_imu_windows(imu: np.ndarray, window_size: int = 250, stride: int = 125, pad: bool = True):
    """preprocessing.py:223-243."""
    n = imu.shape[0]
    if n < window_size:
        if not pad:
            return []
        imu = np.vstack([imu, np.zeros((window_size - n, imu.shape[1]), dtype=np.float32)])
        n = window_size
    return [imu[s:s + window_size] for s in range(0, n - window_size + 1, stride)]
