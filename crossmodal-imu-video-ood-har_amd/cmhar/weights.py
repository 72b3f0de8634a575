"""Compute-dtype weight packs kept in HBM next to the fp32 master parameters.

A pack is one contiguous compute-dtype buffer holding one or more master parameters back to back (e.g. the
VideoMAE query/key/value weights → one [3·H, H] bf16 matrix, so QKV is a single GEMM) or an fp32 copy of several
biases.  Packs are refreshed by one multi-tensor HIP launch (cmhar_mt_cast_bf16) whenever a master parameter's
version counter moved (an in-place update by any torch optimizer), and are written directly by
`cmhar.optim.FusedAdamW` (which updates master and shadow in the same pass and then marks the pack fresh).

A weight pack may also keep a TRANSPOSED bf16 copy (`add_weight(..., transpose=True)`): the input-gradient GEMMs
dX = dY·W then run in the forward layout on Wᵀ [K, N] (K-contiguous operand reads) instead of the dgrad layout's
transposed LDS reads of W [N, K].  The copies are rebuilt by one multi-matrix transpose launch
(cmhar_mt_transpose_bf16) the first time `transposed()` is asked for after the shadows changed (once per training
step, right after AdamW rewrote them).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib as L

# struct MTTensor { float* p; const float* g; float* m; float* v; bf16* pbf; float* pcopy; long n; float wd;
#                   float lr_scale; }   (64 bytes)
MT_TENSOR = np.dtype([('p', '<u8'), ('g', '<u8'), ('m', '<u8'), ('v', '<u8'), ('pbf', '<u8'), ('pcopy', '<u8'),
                      ('n', '<i8'), ('wd', '<f4'), ('lr_scale', '<f4')])
# struct MTTranspose { const bf16* src; bf16* dst; int rows; int cols; int tile0; int pad; }  (32 bytes)
MT_TRANSPOSE = np.dtype([('src', '<u8'), ('dst', '<u8'), ('rows', '<i4'), ('cols', '<i4'), ('tile0', '<i4'),
                         ('pad', '<i4')])
# struct MTChunk { int t; int pad; long start; long len; }  (24 bytes)
MT_CHUNK = np.dtype([('t', '<i4'), ('pad', '<i4'), ('start', '<i8'), ('len', '<i8')])
CHUNK = 65536


def chunk_list(sizes, chunk=CHUNK):
    rows = []
    for t, n in enumerate(sizes):
        for s in range(0, int(n), chunk):
            rows.append((t, 0, s, min(chunk, int(n) - s)))
    return np.array(rows, dtype=MT_CHUNK) if rows else np.zeros(0, dtype=MT_CHUNK)


def to_device_bytes(arr: np.ndarray, device) -> torch.Tensor:
    """Asynchronous upload of a small metadata table (pinned host staging; no stream synchronisation)."""
    host = torch.from_numpy(arr.view(np.uint8).copy()).pin_memory()
    return host.to(device, non_blocking=True)


class PackedWeights:
    def __init__(self, device, dtype):
        self.device = torch.device(device)
        self.dtype = dtype
        self._spec = []          # (name, params, kind)
        self.buffers = {}        # name -> 2-D compute tensor
        self.slots = {}          # param -> (bf16_ptr or 0, fp32_copy_ptr or 0)
        self._versions = None
        self._table = None
        self._gen = 0            # shadow generation: bumped whenever the bf16 shadows are rewritten
        self._t_gen = -1         # generation the transposed copies were built from
        self._t_table = None     # (device descriptor table, ndesc, ntiles)

    def add_weight(self, name, params, transpose=False):
        self._spec.append((name, list(params), 'wt' if transpose else 'w'))

    def add_bias(self, name, params):
        self._spec.append((name, list(params), 'b'))

    def build(self):
        for name, params, kind in self._spec:
            rows = sum(p.shape[0] for p in params)
            cols = int(np.prod(params[0].shape[1:])) if params[0].dim() > 1 else 1
            if kind == 'b':
                buf = torch.empty(rows, dtype=torch.float32, device=self.device)
            elif self.dtype == torch.float32 and len(params) == 1:
                buf = None                     # fp32 mode: use the master parameter itself
            else:
                buf = torch.empty(rows, cols, dtype=self.dtype, device=self.device)
            off = 0
            for p in params:
                if buf is not None:
                    base = buf.data_ptr() + off * buf.element_size()
                    if kind == 'b' or self.dtype == torch.float32:
                        self.slots[p] = (0, base)
                    else:
                        self.slots[p] = (base, 0)
                off += p.numel()
            self.buffers[name] = buf
            if kind == 'wt' and self.dtype == torch.bfloat16 and rows % 8 == 0 and cols % 8 == 0:
                self.buffers[name + '^T'] = torch.empty(cols, rows, dtype=self.dtype, device=self.device)
        self._refresh_table_params = [p for _, ps, _ in self._spec for p in ps if p in self.slots]
        self._versions = None
        descs, tile0 = [], 0
        for name, _, kind in self._spec:
            t = self.buffers.get(name + '^T')
            if t is None:
                continue
            src = self.buffers[name]
            rows, cols = src.shape
            descs.append((src.data_ptr(), t.data_ptr(), rows, cols, tile0, 0))
            tile0 += -(-rows // 64) * -(-cols // 64)
        if descs:
            tab = np.array(descs, dtype=MT_TRANSPOSE)
            self._t_table = (to_device_bytes(tab, self.device), len(descs), tile0)

    def transposed(self, name):
        """Wᵀ [K, N] of weight pack `name` (None when the pack keeps no transposed copy), rebuilt if stale."""
        t = self.buffers.get(name + '^T')
        if t is None:
            return None
        if self._t_gen != self._gen:
            dt, n, ntiles = self._t_table
            L.call('cmhar_mt_transpose_bf16', dt.data_ptr(), n, ntiles, L.stream(self.device))
            self._t_gen = self._gen
        return t

    def __getitem__(self, name):
        buf = self.buffers[name]
        if buf is None:
            p = [ps for n, ps, _ in self._spec if n == name][0][0]
            return p.detach().reshape(p.shape[0], -1)
        return buf

    def get(self, name, default=None):
        return self[name] if name in self.buffers else default

    def mark_fresh(self):
        self._versions = [p._version for p in self._refresh_table_params]
        self._gen += 1

    def refresh(self, force=False):
        params = self._refresh_table_params
        vers = [p._version for p in params]
        if not force and self._versions == vers:
            return
        stale = [p for p, v, o in zip(params, vers, self._versions or [None] * len(params)) if force or v != o]
        if stale:
            tab = np.zeros(len(stale), dtype=MT_TENSOR)
            for i, p in enumerate(stale):
                bf, cp = self.slots[p]
                tab[i]['p'] = p.data_ptr()
                tab[i]['pbf'] = bf
                tab[i]['pcopy'] = cp
                tab[i]['n'] = p.numel()
            if self.dtype == torch.float16:
                # fp16 inference packs (refreshed only when the weights change): one cast launch per parameter
                for p in stale:
                    h, cp = self.slots[p]
                    rows = p.shape[0]
                    cols = p.numel() // rows
                    L.call('cmhar_copy2d', L.F32, L.F16 if h else L.F32, rows, cols, p.data_ptr(), cols, h or cp,
                           cols, 1.0, 0.0, 0.0, 0, L.stream(self.device))
            else:
                ch = chunk_list([p.numel() for p in stale])
                dt = to_device_bytes(tab, self.device)
                dc = to_device_bytes(ch, self.device)
                L.call('cmhar_mt_cast_bf16', dt.data_ptr(), dc.data_ptr(), len(ch), L.stream(self.device))
            self._gen += 1
        self._versions = vers
