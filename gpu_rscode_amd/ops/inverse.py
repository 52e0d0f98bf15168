"""Device Gauss-Jordan inverse over GF(2^8) (``csrc/kernels/gf_invert.hip``).

Replaces the reference's GPU inversion (``GPU_invert_matrix``, ``src/matrix.cu:666-744``) and its
host fallback ``CPU_invert_matrix`` (``src/cpu-decode.c:251-298``, what the reference decoder
actually uses, ``src/decode.cu:333``): one launch per batch of matrices, row pivoting, singular
detection via a per-matrix status word, optional direct emission of decode-GEMM tables.
"""
from __future__ import annotations

import numpy as np
import torch

from ..gf import SingularMatrixError
from .._native import hip
from .gemm import GemmPlan


def gf_invert(a: torch.Tensor, *, check: bool = True, stream: torch.cuda.Stream | None = None):
    """Invert one (n, n) or a batch (b, n, n) of uint8 GF(2^8) matrices on the GPU.

    Returns ``(inverse, status)``; ``status[b] == 1`` marks a singular matrix (its inverse is
    zeroed). With ``check=True`` the call synchronises and raises :class:`SingularMatrixError`.
    """
    if a.dtype != torch.uint8 or a.device.type != "cuda":
        raise TypeError("gf_invert expects a uint8 CUDA tensor")
    squeeze = a.dim() == 2
    a3 = a.unsqueeze(0) if squeeze else a
    if a3.dim() != 3 or a3.shape[1] != a3.shape[2] or a3.shape[1] > 256:
        raise ValueError("expected (n, n) or (b, n, n) with n <= 256")
    a3 = a3.contiguous()
    b, n, _ = a3.shape
    out = torch.empty_like(a3)
    status = torch.empty(b, dtype=torch.int32, device=a.device)
    st = stream or torch.cuda.current_stream(a.device)
    hip().invert(a3.data_ptr(), out.data_ptr(), n, b, status.data_ptr(), 0, 0, 0, 0, st.cuda_stream)
    if check and bool(status.any().item()):
        bad = torch.nonzero(status).flatten().tolist()
        raise SingularMatrixError(f"singular GF(2^8) matrix at batch index {bad}")
    return (out[0] if squeeze else out), (status[0] if squeeze else status)


def invert_into_plan(a: torch.Tensor, plan: GemmPlan, sel_rows, *, status: torch.Tensor | None = None,
                     stream: torch.cuda.Stream | None = None) -> torch.Tensor:
    """Invert ``a`` (k x k, device) and write the v_perm tables of inverse rows ``sel_rows`` into
    ``plan`` — a decode with zero host round-trips. ``plan`` must have k inputs and len(sel_rows)
    outputs. ``sel_rows`` may be a device int32 tensor (no host->device copy: graph-capturable).
    For an ``engine="mfma"`` plan the inverse is also written to a device buffer and the matrix-core
    bit-matrix is rebuilt from its selected rows on the same stream.
    Returns the device status word (0 ok, 1 singular: tables left untouched)."""
    n = a.shape[0]
    if plan.k != n or plan.m != len(sel_rows):
        raise ValueError("plan shape does not match (k inputs, len(sel_rows) outputs)")
    if isinstance(sel_rows, torch.Tensor) and sel_rows.device == a.device and sel_rows.dtype == torch.int32:
        sel = sel_rows
    else:
        sel = torch.as_tensor(np.asarray(sel_rows, dtype=np.int32)).to(a.device, non_blocking=True)
    if status is None:
        status = torch.zeros(1, dtype=torch.int32, device=a.device)
    st = stream or torch.cuda.current_stream(a.device)
    a = a.contiguous()
    inv = 0
    if plan.engine == "mfma":  # the matrix-core operand is rebuilt from the device inverse too
        if getattr(plan, "_inv_buf", None) is None or plan._inv_buf.shape[0] != n:
            plan._inv_buf = torch.empty((n, n), dtype=torch.uint8, device=a.device)
        inv = plan._inv_buf.data_ptr()
    hip().invert(a.data_ptr(), inv, n, 1, status.data_ptr(), plan.desc.data_ptr(), sel.data_ptr(), plan.m,
                 plan.m_pad, st.cuda_stream)
    if plan.engine == "mfma":
        plan.set_device_coeff(plan._inv_buf, sel, stream=st)
    if not torch.cuda.is_current_stream_capturing():
        sel.record_stream(st)
    return status


def decode_system_into_plan(g: torch.Tensor, rows: torch.Tensor, erased: torch.Tensor, plan: GemmPlan, *,
                            status: torch.Tensor | None = None,
                            stream: torch.cuda.Stream | None = None) -> torch.Tensor:
    """Systematic decode with no k x k inverse: solve [G[P, erased] | B'] (e x (e+k)) on device and
    write the decode tables (and, on the matrix-core engine, the bit-matrix) into ``plan``.

    ``g``: the (n, k) generator [I; E] on device; ``rows``: the k survivor ids (device int32, the
    plan's input order); ``erased``: the e erased native ids (device int32, the plan's output
    order, e = plan.m). Graph-capturable (no host copies). Returns the device status word.
    (csrc/kernels/gf_invert.hip::gf_decode_system_kernel.)
    """
    k = g.shape[1]
    if plan.k != k or plan.m != erased.numel() or rows.numel() != k:
        raise ValueError("plan shape does not match (k survivors in, e erased natives out)")
    for t in (rows, erased):
        if t.dtype != torch.int32 or t.device != g.device:
            raise ValueError("rows / erased must be int32 tensors on the generator's device")
    if status is None:
        status = torch.zeros(1, dtype=torch.int32, device=g.device)
    st = stream or torch.cuda.current_stream(g.device)
    g = g.contiguous()
    dm = 0
    if plan.engine == "mfma":
        if getattr(plan, "_dm_buf", None) is None or plan._dm_buf.shape != (plan.m, k):
            plan._dm_buf = torch.empty((plan.m, k), dtype=torch.uint8, device=g.device)
        dm = plan._dm_buf.data_ptr()
    hip().decode_system(g.data_ptr(), k, rows.data_ptr(), erased.data_ptr(), plan.m, dm, status.data_ptr(),
                        plan.desc.data_ptr(), plan.m_pad, st.cuda_stream)
    if plan.engine == "mfma":
        plan.set_device_coeff(plan._dm_buf, stream=st)
    return status
