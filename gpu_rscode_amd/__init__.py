"""gpu_rscode_amd — a gfx950 (MI355X) native Reed-Solomon erasure-coding framework.

Capabilities of zvonkok/GPU-RSCode (the reference), re-designed for CDNA4:
  * GF(2^8) (poly 0x11D) systematic RS codes, reference Vandermonde or MDS matrices (``models``),
  * hand-written HIP kernels: v_perm GF-GEMM, LDS Gauss-Jordan inverse, matrix generation,
    synthetic data (``ops``; sources in ``csrc/kernels``),
  * pinned multi-stream host pipeline and multi-GPU column sharding (native, ``csrc/runtime``),
  * torch.distributed (RCCL over xGMI) stripe sharding, matrix broadcast, parity gather (``parallel``),
  * the reference's file formats and CLI (``utils``, ``bin/RS``, ``bin/CPU-RS``).
"""
from __future__ import annotations

import os

# dmabuf IPC, needed by RCCL peers on this driver: the HIP runtime reads this once when it
# initialises, so it is set here, before this package imports torch (parallel.dist.ensure_ipc_env
# refuses to build an RCCL group if HIP started without it).
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

import torch  # noqa: E402,F401  — load torch's HIP runtime before the native extension

from . import gf  # noqa: E402
from .gf import GF, SingularMatrixError
from .models import ReedSolomon, UnrecoverableError, alloc_rows, flat_rows

__version__ = "0.2.0"

__all__ = ["gf", "GF", "SingularMatrixError", "ReedSolomon", "UnrecoverableError", "alloc_rows", "flat_rows", "__version__"]
