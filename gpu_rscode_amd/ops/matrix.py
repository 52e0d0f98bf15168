"""Coding-matrix construction (host and device).

* ``encoding_matrix`` — host (C++), bit-compatible with the reference Vandermonde
  ``E[i][j] = (j+1)^i`` (``src/matrix.cu:752-759``) plus MDS Cauchy / systematic Vandermonde.
* ``gen_matrix_device`` — the reference's K3 ``gen_encoding_matrix`` as a bounds-checked device
  kernel; used when a rank generates E on its GPU before an RCCL broadcast.
* ``generator`` — G = [I_k; E] (``src/cpu-rs.c:459-463``).
"""
from __future__ import annotations

import numpy as np
import torch

from .. import gf
from .._native import cpu, hip

KINDS = ("vandermonde", "cauchy", "sys_vandermonde")


def encoding_matrix(kind: str, k: int, p: int) -> np.ndarray:
    if p == 0:
        return np.zeros((0, k), dtype=np.uint8)
    raw = cpu().encoding_matrix(kind, k, p)
    return np.frombuffer(raw, dtype=np.uint8).reshape(p, k).copy()


def generator(e: np.ndarray) -> np.ndarray:
    return gf.GF256.generator(np.asarray(e, dtype=np.uint8))


def gen_matrix_device(kind: str, k: int, p: int, device=None, stream=None) -> torch.Tensor:
    code = {"vandermonde": 0, "cauchy": 1}.get(kind)
    if code is None:
        raise ValueError(f"device generation supports {['vandermonde', 'cauchy']}, got {kind!r}")
    dev = torch.device(device or "cuda")
    out = torch.empty((p, k), dtype=torch.uint8, device=dev)
    st = stream or torch.cuda.current_stream(dev)
    hip().gen_matrix(out.data_ptr(), k, p, code, st.cuda_stream)
    return out


def decode_matrix(g: np.ndarray, rows) -> np.ndarray:
    """inv(G[rows]) on the host (C++). Raises SingularMatrixError for unrecoverable patterns."""
    g = np.asarray(g, dtype=np.uint8)
    k = g.shape[1]
    raw = cpu().decode_matrix(g.tobytes(), k, [int(r) for r in rows])
    if raw is None:
        raise gf.SingularMatrixError(f"erasure pattern with survivors {list(rows)} is unrecoverable")
    return np.frombuffer(raw, dtype=np.uint8).reshape(k, k).copy()
