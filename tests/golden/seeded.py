"""Deterministic weights/inputs shared by the golden generator and the parity tests.

Weights are NOT stored in the fixtures: every state_dict entry is regenerated from (seed, key) with a CPU
torch.Generator, so the reference model (in `make_golden.py`) and the build's modules (in `tests/`) load
bit-identical parameters from nothing but the key list and shapes recorded in each fixture.
"""
from __future__ import annotations

import zlib
from typing import Dict, Tuple

import torch


def _gen(seed: int, key: str) -> torch.Generator:
    g = torch.Generator()
    g.manual_seed((seed * 1000003 + zlib.crc32(key.encode())) & 0x7FFFFFFF)
    return g


def seeded_tensor(seed: int, key: str, shape: Tuple[int, ...], dtype=torch.float32) -> torch.Tensor:
    g = _gen(seed, key)
    name = key.rsplit('.', 1)[-1]
    if dtype in (torch.int64, torch.long):
        return torch.zeros(shape, dtype=dtype)
    if name == 'running_var':
        return 0.5 + torch.rand(shape, generator=g)
    if name == 'running_mean':
        return 0.1 * torch.randn(shape, generator=g)
    x = torch.randn(shape, generator=g)
    is_norm = ('norm' in key or 'layernorm' in key or '.net.1.' in key or
               (key.startswith('classifier.') or '.classifier.' in key) and len(shape) == 1 and 'weight' in name)
    if len(shape) == 1:
        if name == 'weight' and is_norm:
            return 1.0 + 0.05 * x
        return 0.02 * x
    if len(shape) == 0:
        return x
    if name in ('cls_token', 'pos_encoding'):
        return x                                            # reference init is randn (models.py:78,82)
    fan_in = 1
    for s in shape[1:]:
        fan_in *= s
    return x / fan_in ** 0.5


def seeded_state_dict(template: Dict[str, torch.Tensor], seed: int) -> Dict[str, torch.Tensor]:
    return {k: seeded_tensor(seed, k, tuple(v.shape), v.dtype) for k, v in template.items()}


def seeded_input(seed: int, shape, scale: float = 1.0) -> torch.Tensor:
    g = torch.Generator()
    g.manual_seed(seed)
    return scale * torch.randn(shape, generator=g)
