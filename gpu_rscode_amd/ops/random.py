"""Device synthetic-data generator: counter-based (splitmix64) random bytes, 16 B per lane store.

Benchmark input is generated in HBM so host links never bound a device-resident measurement
(SURVEY §7.0).
"""
from __future__ import annotations

import torch

from .._native import hip


def fill_random_(t: torch.Tensor, seed: int = 0, stream=None) -> torch.Tensor:
    """Fill a contiguous uint8 CUDA tensor in place with deterministic random bytes."""
    if t.dtype != torch.uint8 or t.device.type != "cuda" or not t.is_contiguous():
        raise TypeError("fill_random_ expects a contiguous uint8 CUDA tensor")
    if t.data_ptr() % 16:
        raise ValueError("fill_random_ needs a 16-byte aligned tensor")
    st = stream or torch.cuda.current_stream(t.device)
    hip().fill_random(t.data_ptr(), t.numel(), int(seed) & ((1 << 64) - 1), st.cuda_stream)
    return t
