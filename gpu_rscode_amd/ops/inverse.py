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
from .gemm import Gemm16Plan, GemmPlan


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
                            status: torch.Tensor | None = None, stream: torch.cuda.Stream | None = None,
                            ptrs: torch.Tensor | None = None) -> torch.Tensor:
    """Systematic decode with no k x k inverse: solve [G[P, erased] | B'] (e x (e+k)) on device and
    write the decode tables (and, on the matrix-core engine, the bit-matrix) into ``plan``.

    ``g``: the (n, k) generator [I; E] on device; ``rows``: the k survivor ids (device int32, the
    plan's input order); ``erased``: the e erased native ids (device int32, the plan's output
    order, e = plan.m). Graph-capturable (no host copies). Returns the device status word.
    With ``ptrs`` (device int64 [n + k]: every chunk row's address, then every output row's) the plan
    is built on the device from ``rows`` alone: ``erased`` is derived and written by the kernel, and
    so are the descriptor's row pointers (see :class:`PatternDecoder`); status 2 = invalid pattern.
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
    n_chunks = 0
    if ptrs is not None:
        n_chunks = g.shape[0]
        if ptrs.dtype != torch.int64 or ptrs.device != g.device or ptrs.numel() != n_chunks + k:
            raise ValueError("ptrs must be a device int64 tensor of n chunk + k output row addresses")
    hip().decode_system(g.data_ptr(), k, rows.data_ptr(), erased.data_ptr(), plan.m, dm, status.data_ptr(),
                        plan.desc.data_ptr(), plan.m_pad, st.cuda_stream, 0 if ptrs is None else ptrs.data_ptr(),
                        n_chunks)
    if plan.engine == "mfma":
        plan.set_device_coeff(plan._dm_buf, stream=st)
    return status


def _is_w16(g: torch.Tensor) -> bool:
    return g.dtype in (torch.int16, torch.uint16)


def decode16_device_supported(n: int, k: int, e: int) -> bool:
    """Whether the device builds GF(2^16) decode plans for (n, k, e): one workgroup's LDS, else the
    blocked multi-workgroup solve (any e up to ~19 K)."""
    return hip().decode_system16_supported(n, k, e) or hip().decode_system16_workspace(n, k, e) >= 0


def decode_system16_into_plan(g: torch.Tensor, rows: torch.Tensor, erased: torch.Tensor, plan: Gemm16Plan, *,
                              status: torch.Tensor | None = None, stream: torch.cuda.Stream | None = None,
                              ptrs: torch.Tensor | None = None, dm: torch.Tensor | None = None,
                              force_blocked: bool = False) -> torch.Tensor:
    """GF(2^16) form of :func:`decode_system_into_plan` (``csrc/kernels/gf_decode16.hip``): ``g`` is
    the (n, k) generator as a 16-bit device tensor; ``erased`` (device int32 [e]) is always written
    by the kernel (derived from ``rows``); ``dm`` (optional, int16 [e, k]) receives the decode rows.
    Writes the plan's four-record tables (and with ``ptrs`` its row pointers). Graph-capturable.
    Systems past one workgroup's LDS (e.g. k = 2000, e = 100; any e > 256) take the blocked
    multi-workgroup solve with a device workspace cached on the plan (``force_blocked``: for any
    size, tests). Returns the device status word (0 ok, 1 singular, 2 invalid survivor list)."""
    n, k = g.shape
    e = erased.numel()
    if plan.k != k or plan.m != e or rows.numel() != k:
        raise ValueError("plan shape does not match (k survivors in, e erased natives out)")
    for t in (rows, erased):
        if t.dtype != torch.int32 or t.device != g.device:
            raise ValueError("rows / erased must be int32 tensors on the generator's device")
    blocked = force_blocked or not hip().decode_system16_supported(n, k, e)
    ws_bytes = hip().decode_system16_workspace(n, k, e) if blocked else 0
    if ws_bytes < 0:
        raise ValueError(f"GF(2^16) device decode system (n={n}, k={k}, e={e}) is too large for the device solve")
    ws = None
    if blocked:
        ws = getattr(plan, "_solve_ws", None)
        if ws is None or ws.numel() < ws_bytes or ws.device != g.device:
            ws = plan._solve_ws = torch.empty(ws_bytes, dtype=torch.uint8, device=g.device)
    if status is None:
        status = torch.zeros(1, dtype=torch.int32, device=g.device)
    if ptrs is not None and (ptrs.dtype != torch.int64 or ptrs.device != g.device or ptrs.numel() != n + k):
        raise ValueError("ptrs must be a device int64 tensor of n chunk + k output row addresses")
    if dm is not None and (dm.device != g.device or dm.numel() != e * k or not dm.is_contiguous()):
        raise ValueError("dm must be a contiguous [e, k] 16-bit device tensor")
    st = stream or torch.cuda.current_stream(g.device)
    g = g.contiguous()
    if dm is None and plan.engine == "mfma":  # the bit-matrix is rebuilt from the device-solved rows
        if getattr(plan, "_dm_buf", None) is None or plan._dm_buf.shape != (e, k):
            plan._dm_buf = torch.empty((e, k), dtype=torch.int16, device=g.device)
        dm = plan._dm_buf
    hip().decode_system16(g.data_ptr(), n, k, rows.data_ptr(), erased.data_ptr(), e,
                          0 if dm is None else dm.data_ptr(), status.data_ptr(), plan.desc.data_ptr(), plan.m_pad,
                          st.cuda_stream, 0 if ptrs is None else ptrs.data_ptr(), 0 if ws is None else ws.data_ptr(),
                          force_blocked)
    if ws is not None and not torch.cuda.is_current_stream_capturing():
        ws.record_stream(st)
    if plan.engine == "mfma":
        plan.set_device_coeff(dm, stream=st)
    return status


class PatternDecoder:
    """A decode whose erasure pattern lives in DEVICE memory: one plan serves every pattern with
    ``e`` erased natives, and nothing about the pattern passes through the host.

    ``rows`` (device int32 [k]) holds the survivor chunk ids; it may be written by a kernel, a
    device copy, or an RCCL broadcast from a coordinator rank (bench.py: rank 0 picks the step's
    failed chunks — a lost node takes the same chunk index from every stripe, so one pattern per
    step). :meth:`solve` checks the pattern, solves the systematic decode system and writes the
    descriptor (row pointers and tables) on the device; :meth:`run` rebuilds the erased natives
    into ``out`` and copies the surviving natives in the same pass. Both are graph-capturable.

    GF(2^16) codes (``g`` a 16-bit tensor: int16 / uint16 holding the field's symbols) run the same
    way on :class:`~gpu_rscode_amd.ops.gemm.Gemm16Plan` with the w = 16 solve (gf_decode16.hip).

    Args:
        g: (n, k) generator [I; E] on the device.
        chunks: the stripe's n rows (k natives then the parity rows), 16-byte aligned.
        out: k output rows, 16-byte aligned.
        e: erased natives per pattern (1..min(k, n-k)).
        engine: GEMM engine ("auto": FP4 matrix cores for wide stripes).
    """

    def __init__(self, g: torch.Tensor, chunks, out, e: int, engine: str = "auto"):
        chunks, out = list(chunks), list(out)
        n, k = g.shape
        if len(chunks) != n or len(out) != k:
            raise ValueError(f"need the stripe's {n} chunk rows and {k} output rows")
        if not 1 <= e <= min(k, n - k):
            raise ValueError(f"e must be in [1, {min(k, n - k)}]")
        rows_all = chunks + out
        if any(r.dtype != torch.uint8 or r.dim() != 1 or r.device != g.device or r.data_ptr() % 16 for r in rows_all):
            raise ValueError("chunk / output rows must be 16-byte aligned uint8 rows on the generator's device")
        self.g, self.k, self.n, self.e = g, k, n, e
        self.wide = _is_w16(g)
        # placeholders until the first solve: inputs = the natives, outputs = the first e output rows
        if self.wide:
            if not decode16_device_supported(n, k, e):
                raise ValueError(f"GF(2^16) device decode system (n={n}, k={k}, e={e}) is too large for the device solve")
            self.plan = Gemm16Plan(chunks[:k], out[:e], copies=out, device_tables=True,
                                   engine="auto" if engine == "auto" else ("mfma" if engine == "mfma" else "valu16"))
        else:
            self.plan = GemmPlan(chunks[:k], out[:e], copies=out, device_tables=True, engine=engine)
        ncols = min(r.numel() for r in rows_all)
        self.plan.ncols = ncols - (ncols % 2 if self.wide else 0)
        if self.plan.engine == "mfma":
            self.plan.in_stride = 0  # survivors are not equally spaced: DMA row pointers come from the descriptor
        dev = g.device
        self.ptrs = torch.tensor([int(r.data_ptr()) for r in rows_all], dtype=torch.int64, device=dev)
        self.rows = torch.zeros(k, dtype=torch.int32, device=dev)
        self.erased = torch.zeros(e, dtype=torch.int32, device=dev)
        self.status = torch.zeros(1, dtype=torch.int32, device=dev)
        self._keep = rows_all  # the rows the pointer table names stay alive with the decoder

    @property
    def engine(self) -> str:
        return self.plan.engine

    def solve(self, stream: torch.cuda.Stream | None = None, rows: torch.Tensor | None = None) -> torch.Tensor:
        """Build the plan for the pattern now in :attr:`rows` — or in ``rows`` (any device int32 [k]
        tensor, e.g. a row of a device-resident pattern pool: no copy) — as device work on ``stream``."""
        rows = self.rows if rows is None else rows
        if rows.dtype != torch.int32 or rows.device != self.g.device or rows.numel() != self.k or not rows.is_contiguous():
            raise ValueError("rows must be a contiguous int32 [k] tensor on the decoder's device")
        if self.wide:
            return decode_system16_into_plan(self.g, rows, self.erased, self.plan, status=self.status, stream=stream,
                                             ptrs=self.ptrs)
        return decode_system_into_plan(self.g, rows, self.erased, self.plan, status=self.status, stream=stream,
                                       ptrs=self.ptrs)

    def run(self, stream: torch.cuda.Stream | None = None, **kw) -> None:
        if self.wide:  # (the v_perm variant knobs are GF(2^8) ablations)
            kw = {key: v for key, v in kw.items() if key in ("col0", "ncols", "max_blocks")}
        self.plan.run(stream, **kw)
