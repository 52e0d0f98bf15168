"""Host-resident streaming: the reference's ``-s`` stream pipeline and single-process multi-GPU
column sharding (``src/encode.cu:109-238,357-432``), run by the native runtime
(``csrc/runtime/pipeline.cpp``): pinned host rows -> H2D -> v_perm GEMM -> D2H on S HIP streams per
device, one host thread per device, no host synchronisation inside the loop.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from .._native import hip


@dataclass
class PipelineResult:
    wall_ms: float
    devices: list

    @property
    def h2d_bytes(self) -> int:
        return sum(d["bytes_h2d"] for d in self.devices)


def _host_rows(x: torch.Tensor) -> list[int]:
    if x.device.type != "cpu" or x.dtype != torch.uint8 or x.dim() != 2 or x.stride(1) != 1:
        raise ValueError("expected a 2-D uint8 host tensor with contiguous rows")
    return [x[i].data_ptr() for i in range(x.shape[0])]


def gemm_host(coeff: np.ndarray, inputs: torch.Tensor, outputs: torch.Tensor, devices=None, streams: int = 2,
              slice_bytes: int = 16 << 20, max_blocks: int = 0) -> PipelineResult:
    """outputs = coeff . inputs for host tensors, streamed through ``devices`` (default: all).

    Pin ``inputs``/``outputs`` (``tensor.pin_memory()``) for asynchronous DMA; pageable memory works
    but serialises the copies.
    """
    coeff = np.ascontiguousarray(coeff, dtype=np.uint8)
    m, k = coeff.shape
    if inputs.shape[0] != k or outputs.shape[0] != m:
        raise ValueError("row counts do not match the coefficient matrix")
    ncols = min(inputs.shape[1], outputs.shape[1])
    if devices is None:
        devices = list(range(torch.cuda.device_count()))
    res = hip().gemm_host(list(devices), _host_rows(inputs), _host_rows(outputs), coeff.tobytes(), ncols, streams,
                          slice_bytes, max_blocks, False)
    return PipelineResult(res["wall_ms"], list(res["devices"]))


def encode_host(rs, data: torch.Tensor, parity: torch.Tensor | None = None, **kw):
    """Encode host-resident [k, C] data with codec ``rs`` through the streaming pipeline."""
    if parity is None:
        parity = torch.empty((rs.p, data.shape[1]), dtype=torch.uint8, pin_memory=data.is_pinned())
    return parity, gemm_host(rs.E, data, parity, **kw)
