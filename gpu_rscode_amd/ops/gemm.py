"""GF-GEMM tensor op on gfx950: ``out[i] = XOR_j L_ij(in[j])`` over byte rows.

``L_ij`` is any GF(2)-linear byte map — multiplication by a GF(2^8) coefficient (the reference's
only case, ``src/matrix.cu:232-407``), or the nibble-wise GF(2^4) "GF(16) method" of
``doc/design.tex:190-209``. The kernel (``csrc/kernels/gf_gemm.hip``) reads a device descriptor of
row pointers + per-map v_perm tables; :class:`GemmPlan` builds and caches that descriptor so a
repeated encode/decode is one kernel launch.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Sequence

import numpy as np
import torch

from .. import gf
from .._native import hip
from ..utils.tune import tune_int, tune_str

MAX_TILE = 16


def tile_for(m: int) -> int:
    t = 1
    while t < m and t < MAX_TILE:
        t <<= 1
    return t


def pad_m(m: int) -> int:
    t = tile_for(m)
    return (m + t - 1) // t * t


@dataclass(frozen=True)
class DescLayout:
    in_off: int
    copy_off: int
    out_off: int
    tab_off: int
    bytes: int


def desc_layout(k: int, m_pad: int, batch: int = 1) -> DescLayout:
    """Mirror of ``gfrs::desc_layout`` (``csrc/include/gfrs/desc.h``); a test pins the two equal."""
    in_off = 16
    copy_off = in_off + 8 * k * batch
    out_off = copy_off + 8 * k * batch
    tab_off = (out_off + 8 * m_pad * batch + 31) // 32 * 32
    return DescLayout(in_off, copy_off, out_off, tab_off, tab_off + 32 * k * m_pad)


def perm_tables_from_coeff(coeff: np.ndarray) -> np.ndarray:
    """(m, k) GF(2^8) coefficients -> (m, k, 8) uint32 v_perm records."""
    coeff = np.asarray(coeff, dtype=np.uint8)
    cache: dict[int, np.ndarray] = {}
    m, k = coeff.shape
    out = np.zeros((m, k, 8), dtype=np.uint32)
    for i in range(m):
        for j in range(k):
            c = int(coeff[i, j])
            if c not in cache:
                cache[c] = gf.perm_record(gf.byte_map_gf256(c))
            out[i, j] = cache[c]
    return out


def perm_tables_from_maps(maps: np.ndarray) -> np.ndarray:
    """(m, k, 256) linear byte maps -> (m, k, 8) uint32 v_perm records."""
    maps = np.asarray(maps, dtype=np.uint8)
    m, k, _ = maps.shape
    out = np.zeros((m, k, 8), dtype=np.uint32)
    for i in range(m):
        for j in range(k):
            out[i, j] = gf.perm_record(maps[i, j])
    return out


def build_desc(in_ptrs: Sequence[int], out_ptrs: Sequence[int], copy_ptrs: Sequence[int] | None,
               tables: np.ndarray | None, batch: int = 1) -> np.ndarray:
    """Descriptor bytes for ``batch`` stripes of k inputs and m outputs each (pointer lists are
    stripe-major: ``batch * k`` / ``batch * m``); ``tables`` is (m, k, 8) uint32 or None (zeros)."""
    if len(in_ptrs) % batch or len(out_ptrs) % batch:
        raise ValueError("pointer lists must hold batch * k / batch * m entries")
    k, m = len(in_ptrs) // batch, len(out_ptrs) // batch
    if not (1 <= k <= 256 and 1 <= m <= 256):
        raise ValueError("GF-GEMM supports 1 <= k, m <= 256")
    mp = pad_m(m)
    lay = desc_layout(k, mp, batch)
    d = np.zeros(lay.bytes, dtype=np.uint8)
    d[0:16] = np.frombuffer(np.array([k, m, mp, batch], dtype="<i4").tobytes(), dtype=np.uint8)
    d[lay.in_off : lay.in_off + 8 * k * batch] = np.frombuffer(np.array(in_ptrs, dtype="<u8").tobytes(),
                                                               dtype=np.uint8)
    if copy_ptrs is not None:
        if len(copy_ptrs) != k * batch:
            raise ValueError("copy_ptrs must have batch * k entries")
        d[lay.copy_off : lay.copy_off + 8 * k * batch] = np.frombuffer(
            np.array([p or 0 for p in copy_ptrs], dtype="<u8").tobytes(), dtype=np.uint8)
    outs = []
    for b in range(batch):
        outs += list(out_ptrs[b * m : (b + 1) * m]) + [0] * (mp - m)
    d[lay.out_off : lay.out_off + 8 * mp * batch] = np.frombuffer(np.array(outs, dtype="<u8").tobytes(),
                                                                  dtype=np.uint8)
    if tables is not None:
        t = np.zeros((k, mp, 8), dtype="<u4")
        t[:, :m, :] = np.transpose(np.asarray(tables, dtype=np.uint32), (1, 0, 2))
        d[lay.tab_off :] = np.frombuffer(t.tobytes(), dtype=np.uint8)
    return d


def _batched_rows(x) -> list[list[torch.Tensor]] | None:
    """[B, rows, C] tensor or list of per-stripe row lists -> list of stripes; None if not batched."""
    if isinstance(x, torch.Tensor):
        return [_rows(x[b]) for b in range(x.shape[0])] if x.dim() == 3 else None
    if isinstance(x, (list, tuple)) and x and isinstance(x[0], (list, tuple)):
        return [list(s) for s in x]
    return None


def _rows(x) -> list[torch.Tensor]:
    if isinstance(x, torch.Tensor):
        if x.dim() == 1:
            return [x]
        if x.dim() != 2:
            raise ValueError("expected a 2-D [rows, bytes] tensor or a list of 1-D tensors")
        return [x[i] for i in range(x.shape[0])]
    return list(x)


def _check_rows(rows: list[torch.Tensor], what: str, device: torch.device | None) -> torch.device:
    for r in rows:
        if r.dtype != torch.uint8:
            raise TypeError(f"{what} rows must be uint8, got {r.dtype}")
        if r.dim() != 1 or (r.numel() > 1 and r.stride(0) != 1):
            raise ValueError(f"{what} rows must be contiguous 1-D byte rows")
        if device is None:
            device = r.device
        elif r.device != device:
            raise ValueError(f"all rows must live on one device ({device} vs {r.device})")
    return device


class GemmPlan:
    """A reusable device GF-GEMM.

    Args:
        inputs: k input byte rows (2-D uint8 tensor or list of 1-D tensors) on one GPU.
        outputs: m output byte rows on the same GPU.
        coeff: (m, k) GF(2^8) coefficients; or
        maps: (m, k, 256) GF(2)-linear byte maps (e.g. :func:`gf.byte_map_gf16_nibbles`); or neither
            with ``device_tables=True`` (tables are written later on device, e.g. by
            :func:`gpu_rscode_amd.ops.inverse.invert_into_plan`).
        copies: optional k destination rows (or None entries): input j is copied there in the same
            pass (the fused survivor copy of decode).
        hold_buffers: keep references to the row tensors (default). A plan only stores raw
            pointers in its descriptor, so a cache that hands a plan out only for the exact pointers
            of live tensors (``ReedSolomon``'s plan cache) passes False: otherwise every cached plan
            pins its caller's buffers and a loop over fresh buffers keeps all of them alive.
    """

    def __init__(self, inputs, outputs, coeff=None, *, maps=None, copies=None, device_tables: bool = False,
                 engine: str = "auto", mfma_mg: int = 8, hold_buffers: bool = True):
        bi, bo = _batched_rows(inputs), _batched_rows(outputs)
        if (bi is None) != (bo is None):
            raise ValueError("inputs and outputs must both be batched ([B, rows, C]) or both not")
        self.batch = 1
        if bi is not None:
            # batched: B stripes of identical shape, one launch (grid.y = stripe)
            if len(bi) != len(bo) or len(bi) < 1 or len(bi) > 65535:
                raise ValueError("batched plan needs 1..65535 stripes in inputs and outputs")
            if engine not in ("valu", "auto", "mfma"):
                raise ValueError("batched plans run on the v_perm kernel or, for wide codes, the FP4 matrix cores")
            self.batch = len(bi)
            self._stripes_in, self._stripes_out = bi, bo
            inputs, outputs = bi[0], bo[0]
            if copies is not None:  # per stripe: k destination rows (or None entries)
                if len(copies) != self.batch or any(len(c) != len(bi[0]) for c in copies):
                    raise ValueError("batched copies need one list of k destinations per stripe")
                self._stripes_copy = [list(c) for c in copies]
                copies = copies[0]
        self.inputs = _rows(inputs)
        self.outputs = _rows(outputs)
        self.copies = None if copies is None else [c for c in copies]
        dev = _check_rows(self.inputs, "input", None)
        dev = _check_rows(self.outputs, "output", dev)
        if self.copies is not None:
            if len(self.copies) != len(self.inputs):
                raise ValueError("copies must have one entry per input row")
            dev = _check_rows([c for c in self.copies if c is not None], "copy", dev)
        if dev.type != "cuda":
            raise ValueError("GemmPlan runs on a GPU; use the CPU codec for host tensors")
        self.device = dev
        self.k, self.m = len(self.inputs), len(self.outputs)
        self.m_pad = pad_m(self.m)
        all_in = [r for st in self._stripes_in for r in st] if self.batch > 1 else self.inputs
        all_out = [r for st in self._stripes_out for r in st] if self.batch > 1 else self.outputs
        if self.batch > 1:
            _check_rows(all_in, "input", dev)
            _check_rows(all_out, "output", dev)
            if any(len(st) != self.k for st in self._stripes_in) or any(len(st) != self.m for st in self._stripes_out):
                raise ValueError("every stripe needs the same number of input / output rows")
        all_copy = ([c for st in self._stripes_copy for c in st] if self.batch > 1 and self.copies is not None
                    else (self.copies or []))
        if self.batch > 1 and self.copies is not None:
            _check_rows([c for c in all_copy if c is not None], "copy", dev)
        lens = [r.numel() for r in all_in + all_out + [c for c in all_copy if c is not None]]
        self.ncols = min(lens) if lens else 0
        if coeff is not None:
            tables = perm_tables_from_coeff(np.asarray(coeff).reshape(self.m, self.k))
        elif maps is not None:
            tables = perm_tables_from_maps(maps)
        elif device_tables:
            tables = None
        else:
            raise ValueError("need coeff, maps or device_tables=True")
        ptr = lambda t: int(t.data_ptr())  # noqa: E731
        self.bytewise = any(ptr(r) % 16 for r in all_in + all_out) or any(
            c is not None and ptr(c) % 16 for c in all_copy)
        host = build_desc([ptr(r) for r in all_in], [ptr(r) for r in all_out],
                          None if self.copies is None else [ptr(c) if c is not None else 0 for c in all_copy],
                          tables, self.batch)
        self.desc = torch.from_numpy(host).to(self.device)
        self.layout = desc_layout(self.k, self.m_pad, self.batch)
        # batched matrix-core launches address stripe b's rows as stripe 0's plus b fixed strides
        self.in_bstride = self.out_bstride = None
        if self.batch > 1:
            strides = _batch_strides(self._stripes_in, self._stripes_out,
                                     self._stripes_copy if self.copies is not None else None)
            if strides is not None:
                self.in_bstride, self.out_bstride = strides
        if engine == "auto":
            engine = _auto_engine(self.k, self.m, maps is None, self.bytewise, self.batch, self.ncols,
                                  batch_fp4=self.batch > 1 and self.in_bstride is not None
                                  and hip().fp4_batched_supported(self.k, self.m, mfma_mg))
        self.engine = engine
        self.bitmat = None
        self.fp4_form = None
        if engine == "mfma" and self.batch > 1 and (
                self.in_bstride is None or not hip().fp4_batched_supported(self.k, self.m, mfma_mg)):
            raise ValueError("batched engine='mfma' needs k in (112, 128], m <= 32 and stripes at fixed strides")
        if engine in ("mfma", "mfma_i8"):
            # matrix-core GF(2) bit-matrix paths: "mfma" = FP4 block-scaled MFMA
            # (csrc/kernels/gf_mfma_fp4.hip), "mfma_i8" = int8 MFMA (csrc/kernels/gf_mfma.hip).
            # GF(2^8) coefficients (host coeff=, or device_tables=True and set_device_coeff /
            # invert_into_plan later), aligned rows; fused copies on "mfma" only. The column
            # remainder of a chunk runs on the v_perm tables that the descriptor also carries.
            if maps is not None or self.bytewise or (self.batch > 1 and engine != "mfma"):
                raise ValueError(f"engine={engine!r} needs GF(2^8) coefficients, aligned rows, one stripe")
            if engine == "mfma_i8" and (coeff is None or self.copies is not None):
                raise ValueError("engine='mfma_i8' needs coeff= and no copies")
            if not 1 <= mfma_mg <= 8:
                raise ValueError("mfma_mg must be 1..8")
            self.mfma_mg = mfma_mg
            # equally spaced input rows (one allocation): the FP4 kernel computes DMA addresses
            ptrs = [ptr(r) for r in self.inputs]
            stride = ptrs[1] - ptrs[0] if self.k > 1 else 1
            uniform = stride != 0 and all(p - ptrs[0] == j * stride for j, p in enumerate(ptrs))
            self.in_stride = stride if uniform else 0
            # the FP4 kernel form the native router runs for this shape (v1 / ar / tm:
            # fp4_route in csrc/kernels/gf_mfma_fp4.hip; one bit-matrix layout serves all three)
            self.fp4_form = (hip().fp4_route(self.k, self.m, self.copies is not None, mfma_mg)
                             if engine == "mfma" and self.batch == 1 else None)
            if coeff is not None:
                self._build_bitmat(coeff)
            else:  # filled on device later (set_device_coeff / invert_into_plan)
                self.bitmat = torch.zeros(self._bitmat_bytes(), dtype=torch.uint8, device=self.device)
        elif engine == "lut":  # LDS nibble-table ablation (csrc/kernels/gf_gemm_lut.hip)
            if self.bytewise or self.batch > 1:
                raise ValueError("engine='lut' needs 16-byte aligned rows and one stripe")
        elif engine != "valu":
            raise ValueError(f"unknown engine {engine!r}")
        self.has_copies = self.copies is not None
        if not hold_buffers:
            self.inputs = self.outputs = self.copies = None
            self._stripes_in = self._stripes_out = self._stripes_copy = None
        self._mark_ready()

    def _bitmat_bytes(self) -> int:
        if self.engine == "mfma":
            return hip().fp4_bitmat_bytes(self.k, self.m, self.mfma_mg)
        return hip().mfma_bitmat_bytes(self.k, self.m)

    def _build_bitmat(self, coeff) -> None:
        """Bit-matrix operand of the matrix-core engines, built on device from the m x k coefficients."""
        c = torch.from_numpy(np.ascontiguousarray(np.asarray(coeff, dtype=np.uint8).reshape(self.m, self.k)))
        c = c.to(self.device)
        h = hip()
        st = torch.cuda.current_stream(self.device).cuda_stream
        if self.engine == "mfma":
            if self.bitmat is None:
                self.bitmat = torch.empty(h.fp4_bitmat_bytes(self.k, self.m, self.mfma_mg), dtype=torch.uint8,
                                          device=self.device)
            h.fp4_bitmat(c.data_ptr(), self.m, self.k, self.bitmat.data_ptr(), self.mfma_mg, st)
        else:
            if self.bitmat is None:
                self.bitmat = torch.empty(h.mfma_bitmat_bytes(self.k, self.m), dtype=torch.uint8, device=self.device)
            h.mfma_bitmat(c.data_ptr(), self.m, self.k, self.bitmat.data_ptr(), st)
        self._coeff_dev = c

    def set_device_coeff(self, coeff: torch.Tensor, rows=None, stream: torch.cuda.Stream | None = None) -> None:
        """Rebuild the matrix-core operand from a DEVICE matrix: coefficient row i = coeff[rows[i]]
        (``rows`` a device int32 tensor, or None for coeff itself, m x k). No host round trip — the
        decode path feeds it the device-computed inverse. (v_perm tables: see invert_into_plan.)"""
        if self.engine != "mfma":
            raise ValueError("set_device_coeff applies to engine='mfma' plans")
        if coeff.dtype != torch.uint8 or coeff.device != self.device or coeff.dim() != 2 or coeff.shape[1] < self.k:
            raise ValueError("coeff must be a 2-D uint8 tensor on the plan's device with >= k columns")
        coeff = coeff.contiguous()
        st = stream or torch.cuda.current_stream(self.device)
        sel = 0
        if rows is not None:
            if rows.dtype != torch.int32 or rows.numel() != self.m:
                raise ValueError("rows must be an int32 tensor of m row indices")
            sel = rows.data_ptr()
        elif coeff.shape[0] < self.m:
            raise ValueError("coeff needs m rows")
        hip().fp4_bitmat_sel(coeff.data_ptr(), coeff.stride(0), sel, self.m, self.k, self.bitmat.data_ptr(),
                             self.mfma_mg, st.cuda_stream)
        if not torch.cuda.is_current_stream_capturing():
            coeff.record_stream(st)

    def _mark_ready(self) -> None:
        # descriptor writes are ordered on the current stream; launches on other streams wait on this
        self._ready = torch.cuda.Event()
        self._ready.record(torch.cuda.current_stream(self.device))

    def set_coeff(self, coeff, stream: torch.cuda.Stream | None = None) -> None:
        """Replace the coefficient tables (host-built, async H2D on ``stream``)."""
        tables = perm_tables_from_coeff(np.asarray(coeff).reshape(self.m, self.k))
        t = np.zeros((self.k, self.m_pad, 8), dtype="<u4")
        t[:, : self.m, :] = np.transpose(tables, (1, 0, 2))
        src = torch.from_numpy(np.frombuffer(t.tobytes(), dtype=np.uint8).copy())
        with torch.cuda.stream(stream) if stream is not None else _null():
            self.desc[self.layout.tab_off :].copy_(src, non_blocking=False)
            if self.bitmat is not None:
                self._build_bitmat(coeff)
            self._mark_ready()

    def table_view(self) -> torch.Tensor:
        """Device view of the table block (k, m_pad, 8) int32 words."""
        return self.desc[self.layout.tab_off :].view(torch.int32).view(self.k, self.m_pad, 8)

    def run(self, stream: torch.cuda.Stream | None = None, col0: int = 0, ncols: int | None = None,
            max_blocks: int = 0, vec: int | None = None, pf: int = 2, nt: bool = False) -> None:
        """Launch asynchronously on ``stream`` (default: the current stream).

        ``vec``/``pf``/``nt`` select an explicit v_perm kernel variant (ablation; ``vec=0`` = byte
        kernel; this bypasses a matrix-core engine); by default the plan's engine runs with the tuned
        configuration for the output tile.
        """
        ncols = self.ncols - col0 if ncols is None else ncols
        if col0 < 0 or ncols < 0 or col0 + ncols > self.ncols:
            raise ValueError(f"column range [{col0}, {col0 + ncols}) outside rows of {self.ncols} bytes")
        if stream is None:
            if self._ready is not None:
                torch.cuda.current_stream(self.device).wait_event(self._ready)
                self._ready = None
            # the raw handle: no Stream object per launch (small-object serving is launch-bound)
            s = torch._C._cuda_getCurrentRawStream(self.device.index)
        else:
            if self._ready is not None:
                stream.wait_event(self._ready)
                self._ready = None
            self.desc.record_stream(stream)
            s = stream.cuda_stream
        h = hip()
        if self.batch > 1 and self.engine == "mfma" and vec is None and col0 % 2 == 0:
            h.gemm_fp4_batched(int(self.bitmat.data_ptr()), int(self.desc.data_ptr()), self.k, self.m, self.batch, col0,
                               ncols, self.mfma_mg, self.in_stride, self.in_bstride, self.out_bstride, self.has_copies, s)
        elif self.batch > 1:
            if vec is not None:
                raise ValueError("kernel variants are not selectable on batched plans")
            h.gemm_batched(int(self.desc.data_ptr()), self.k, self.m_pad, self.batch, col0, ncols, self.bytewise, s,
                           self.has_copies)
        elif self.engine == "mfma" and vec is None and col0 % 2 == 0:
            h.gemm_fp4(int(self.bitmat.data_ptr()), int(self.desc.data_ptr()), self.k, self.m, col0, ncols,
                       self.mfma_mg, self.in_stride, self.has_copies, s)
        elif self.engine == "lut" and vec is None and col0 % 16 == 0:
            h.gemm_lut(int(self.desc.data_ptr()), self.k, self.m_pad, col0, ncols, s)
        elif self.engine == "mfma_i8" and vec is None and col0 % 2 == 0:
            h.gemm_mfma(int(self.bitmat.data_ptr()), int(self.desc.data_ptr()), self.k, self.m, col0, ncols, s)
        elif self.bytewise:
            h.gemm(int(self.desc.data_ptr()), self.k, self.m_pad, col0, ncols, True, max_blocks, s)
        elif vec is None:
            h.gemm(int(self.desc.data_ptr()), self.k, self.m_pad, col0, ncols, False, max_blocks, s, self.has_copies)
        else:
            h.gemm_variant(int(self.desc.data_ptr()), self.k, self.m_pad, col0, ncols, vec, pf, nt, max_blocks, s)


# wide stripes go to the FP4 matrix-core kernel: measured on MI355X (profiles/archive/r01_kbench5) it wins
# from k*m ~ 2k coefficients (k=128, p=32: 1.10 ms vs 1.45 ms per GiB); narrow codes stay on the
# v_perm kernel, which is at the HBM roofline there (k=10, p=4: 0.27 ms vs 0.87 ms).
_MFMA_MIN_K, _MFMA_MIN_M = 64, 16
# Short rows move the crossover down: the v_perm kernel parallelises over columns (and output
# tiles) only, so a few-KiB stripe leaves most of the chip idle while each lane walks all k rows,
# whereas the FP4 kernel reduces over k in the matrix cores. scripts/engine_cross.py on MI355X
# (profiles/sweeps/r07_engine_cross): up to 512 KiB per row the FP4 kernel wins from k = 16, m = 4
# (k=16 m=4: 7.4 vs 8.8 us; k=32 m=8: 7.5 vs 25.5; k=128 m=32: 17.6 vs 261), up to 4 MiB from
# k = 32, m = 8 (k=32 m=8: 49 vs 62 us); past that only the wide codes above.
_SHORT_ROW, _MID_ROW = 512 << 10, 4 << 20


# Batched wide codes (serving) take the batched FP4 launch from this many columns per stripe (two
# 128-column chunks of the A-resident kernel; below it the k-split v_perm kernel's shorter prologue
# wins) and 16 outputs, or 8..15 outputs up to _FP4_BATCH_MID_COLS columns over the whole batch.
# Measured on MI355X (profiles/serving/r08_fp4batch, RS(128,160)): encode 256 x 64 KiB 68.9 -> 30.8
# us, 256 x 1 MiB 419 -> 221 us; decode rebuilding 26 natives (+ 102 fused copies) 256 x 1 MiB
# 451 -> 256 us; rebuilding 8: 16 x 1 MiB 32.3 -> 28.1 but 256 x 1 MiB 150 -> 166 (v_perm kept);
# rebuilding 4 (memory-bound beside 124 copies) stays on the v_perm kernels. (scripts/serve_bench.py --code 128:160;
# GFRS_TUNE=fp4_batch_min_cols=N overrides, e.g. a huge value keeps every batch on the v_perm kernels.)
_FP4_BATCH_MIN_COLS = 256
_FP4_BATCH_MID_COLS = 1 << 20


def _auto_engine(k: int, m: int, gf256: bool, bytewise: bool, batch: int, ncols: int | None = None,
                 batch_fp4: bool = False) -> str:
    if not gf256 or bytewise:
        return "valu"
    if batch != 1:  # (a narrow decode — few rebuilt rows beside many fused copies — is memory-bound)
        if not batch_fp4 or ncols is None or ncols < tune_int("fp4_batch_min_cols", _FP4_BATCH_MIN_COLS):
            return "valu"
        return "mfma" if (m >= 16 or (m >= 8 and ncols * batch <= _FP4_BATCH_MID_COLS)) else "valu"
    if k >= _MFMA_MIN_K and m >= _MFMA_MIN_M:
        return "mfma"
    if ncols is not None and ((ncols <= _SHORT_ROW and k >= 16 and m >= 4) or
                              (ncols <= _MID_ROW and k >= 32 and m >= 8)):
        return "mfma"
    return "valu"


def _batch_strides(stripes_in, stripes_out, stripes_copy=None) -> tuple[int, int] | None:
    """(input, output) byte strides between consecutive stripes when every stripe's rows are stripe
    0's shifted by b strides (copy rows at the output stride, the same rows absent in every stripe);
    None otherwise."""
    def stride(stripes):
        base = [int(r.data_ptr()) for r in stripes[0]]
        d = int(stripes[1][0].data_ptr()) - base[0]
        for b, st in enumerate(stripes):
            if any(int(r.data_ptr()) != base[j] + b * d for j, r in enumerate(st)):
                return None
        return d
    d_in, d_out = stride(stripes_in), stride(stripes_out)
    if d_in is None or d_out is None:
        return None
    if stripes_copy is not None:
        base = [int(c.data_ptr()) if c is not None else 0 for c in stripes_copy[0]]
        for b, st in enumerate(stripes_copy):
            for j, c in enumerate(st):
                if (c is None) != (base[j] == 0) or (c is not None and int(c.data_ptr()) != base[j] + b * d_out):
                    return None
    return d_in, d_out


# GF(2^16) codes on the FP4 matrix-core engine (csrc/kernels/gf_mfma16.hip) against the v_perm
# w = 16 kernel, 1 GiB stripes (profiles/gf65536/r08_mfma16): encodes win from k = 16 at any m
# (k=16, m=4: 0.30 vs 0.40 ms; k=300, m=40: 1.98 vs 4.49), k = 10 loses (0.55 vs 0.48). Decodes,
# which also copy the survivors, lose at m = 4 (k=16: 0.51 vs 0.43) and win from m = 8 on wider
# codes (k=64, m=8: 0.62 vs 0.73; k=300, m=40: 2.43 vs 4.52). (GFRS_TUNE=gf16_mfma=0 / 1: never /
# always where supported.)
_GF16_MFMA_MIN_K = 16
_GF16_MFMA_COPY_MIN_M, _GF16_MFMA_COPY_MIN_KM = 8, 256


def _auto_engine16(k: int, m: int, symwise: bool, copies: bool = False) -> bool:
    forced = tune_str("gf16_mfma")
    if symwise or k > 65535:
        return False
    if forced is not None:
        return forced == "1"
    if k < _GF16_MFMA_MIN_K or m < 4:
        return False
    return not copies or (m >= _GF16_MFMA_COPY_MIN_M and k * m >= _GF16_MFMA_COPY_MIN_KM)


def _pack16(coeff) -> bytes:
    """GF(2^16) coefficients as the native pipeline's packed form: little-endian byte pairs
    (``gfrs::pack16``, ``csrc/include/gfrs/host_desc.h``)."""
    return np.ascontiguousarray(np.asarray(coeff, dtype=np.int64).astype("<u2")).tobytes()


def desc_layout16(k: int, m_pad: int, batch: int = 1) -> DescLayout:
    """Mirror of ``gfrs::desc_layout16``: four 32-byte records per coefficient."""
    lay = desc_layout(k, m_pad, batch)
    return DescLayout(lay.in_off, lay.copy_off, lay.out_off, lay.tab_off, lay.tab_off + 4 * 32 * k * m_pad)


class Gemm16Plan:
    """A reusable device GF(2^16) GEMM (``csrc/kernels/gf_gemm16.hip``): ``out[i] = XOR_j c[i][j] * in[j]``
    over little-endian 16-bit symbols in uint8 byte rows.

    The reference's field family names w = 16 (``src/galoisfield.cu:22-32``, poly 0x1100B) but only
    GF(2^8) was ever built; here it runs on the same v_perm engine as four byte maps per coefficient.

    Args:
        inputs: k byte rows (2-D uint8 tensor or list of 1-D tensors) on one GPU, 2-byte aligned;
            or B stripes ([B, k, C] tensor or list of row lists) for one batched launch.
        outputs: m byte rows on the same GPU (batched: [B, m, C] or B row lists).
        coeff: (m, k) GF(2^16) coefficients (uint16-valued); or None with ``device_tables=True``
            (the tables are written later on the device, :func:`~gpu_rscode_amd.ops.inverse.PatternDecoder`).
        copies: optional k destination rows (or None entries): fused survivor copy of decode
            (batched: one such list per stripe).
        hold_buffers: as :class:`GemmPlan`.
    Batched stripes whose rows sit at fixed strides from stripe 0's run the matrix-core engine in one
    persistent launch; otherwise (and with ``engine="valu16"``) the v_perm kernels take grid.y =
    stripe.
    Rows shorter than the others bound the column range, which must be a whole number of symbols.
    """

    def __init__(self, inputs, outputs, coeff=None, *, copies=None, device_tables: bool = False,
                 engine: str = "auto", mfma_mg: int = 2, hold_buffers: bool = True):
        if coeff is None and not device_tables:
            raise ValueError("need coeff or device_tables=True")
        bi, bo = _batched_rows(inputs), _batched_rows(outputs)
        if (bi is None) != (bo is None):
            raise ValueError("inputs and outputs must both be batched ([B, rows, C]) or both not")
        self.batch = 1
        stripes_copy = None
        if bi is not None:
            if len(bi) != len(bo) or not 1 <= len(bi) <= 65535:
                raise ValueError("batched plan needs 1..65535 stripes in inputs and outputs")
            if any(len(st) != len(bi[0]) for st in bi) or any(len(st) != len(bo[0]) for st in bo):
                raise ValueError("every stripe needs the same number of input / output rows")
            self.batch = len(bi)
            if copies is not None:
                if len(copies) != self.batch or any(len(c) != len(bi[0]) for c in copies):
                    raise ValueError("batched copies need one list of k destinations per stripe")
                stripes_copy = [list(c) for c in copies]
                copies = stripes_copy[0]
            inputs, outputs = bi[0], bo[0]
        else:
            bi, bo = [_rows(inputs)], [_rows(outputs)]
            if copies is not None:
                stripes_copy = [list(copies)]
        self.inputs, self.outputs = _rows(inputs), _rows(outputs)
        self.copies = None if copies is None else list(copies)
        if self.copies is not None and len(self.copies) != len(self.inputs):
            raise ValueError("copies must have one entry per input row")
        all_in = [r for st in bi for r in st]
        all_out = [r for st in bo for r in st]
        all_copy = [c for st in (stripes_copy or []) for c in st if c is not None]
        dev = _check_rows(all_in, "input", None)
        dev = _check_rows(all_out, "output", dev)
        if all_copy:
            dev = _check_rows(all_copy, "copy", dev)
        if dev.type != "cuda":
            raise ValueError("Gemm16Plan runs on a GPU; use the CPU codec for host tensors")
        self.device = dev
        self.k, self.m = len(self.inputs), len(self.outputs)
        if not (1 <= self.k <= 65535 and 1 <= self.m <= 65535):
            raise ValueError("GF(2^16) GEMM supports 1 <= k, m <= 65535")
        self.m_pad = pad_m(self.m)
        rows = all_in + all_out + all_copy
        self.ncols = min(r.numel() for r in rows)
        if self.ncols % 2:
            raise ValueError("GF(2^16) rows hold 16-bit symbols: the column range must be an even byte count")
        ptr = lambda t: int(t.data_ptr())  # noqa: E731
        if any(ptr(r) % 2 for r in rows):
            raise ValueError("GF(2^16) rows must be 2-byte aligned")
        self.symwise = any(ptr(r) % 16 for r in rows)
        if coeff is not None:
            coeff = np.asarray(coeff, dtype=np.int64).reshape(self.m, self.k)
            if coeff.min() < 0 or coeff.max() > 65535:
                raise ValueError("GF(2^16) coefficients must be in [0, 65535]")
        self.layout = desc_layout16(self.k, self.m_pad, self.batch)
        lay = self.layout
        host = np.zeros(lay.bytes, dtype=np.uint8)
        host[0:16] = np.frombuffer(np.array([self.k, self.m, self.m_pad, self.batch], dtype="<i4").tobytes(),
                                   dtype=np.uint8)

        def put(off, vals):
            b = np.frombuffer(np.array(vals, dtype="<u8").tobytes(), dtype=np.uint8)
            host[off: off + b.size] = b
        put(lay.in_off, [ptr(r) for r in all_in])
        if stripes_copy is not None:
            put(lay.copy_off, [ptr(c) if c is not None else 0 for st in stripes_copy for c in st])
        put(lay.out_off, [v for st in bo for v in [ptr(r) for r in st] + [0] * (self.m_pad - self.m)])
        # batched matrix-core launches address stripe b's rows as stripe 0's plus b fixed strides
        self.in_bstride = self.out_bstride = None
        if self.batch > 1:
            strides = _batch_strides(bi, bo, stripes_copy)
            if strides is not None:
                self.in_bstride, self.out_bstride = strides
        if coeff is not None:  # else written on the device (decode_system16_into_plan)
            t = np.zeros((self.k, self.m_pad, 4, 8), dtype="<u4")
            t[:, : self.m] = np.transpose(gf.perm_quads16(coeff), (1, 0, 2, 3))
            host[self.layout.tab_off:] = np.frombuffer(t.tobytes(), dtype=np.uint8)
        self.desc = torch.from_numpy(host).to(self.device)
        if engine == "auto":
            engine = "mfma" if _auto_engine16(self.k, self.m, self.symwise, self.copies is not None) else "valu16"
            if self.batch > 1 and self.in_bstride is None:
                engine = "valu16"  # scattered stripes: the batched v_perm kernel (per-stripe pointers)
        if engine == "valu":
            engine = "valu16"
        if engine not in ("valu16", "mfma"):
            raise ValueError(f"unknown GF(2^16) engine {engine!r}")
        if engine == "mfma" and self.batch > 1 and self.in_bstride is None:
            raise ValueError("batched engine='mfma' needs stripes at fixed strides (one [B, rows, C] allocation)")
        self.engine = engine
        self.bitmat = None
        self.has_copies = self.copies is not None
        if engine == "mfma":
            # the FP4 matrix-core engine (csrc/kernels/gf_mfma16.hip), ragged tail included; the
            # descriptor's v_perm records serve starts off a 4-byte boundary
            if self.symwise:
                raise ValueError("engine='mfma' needs 16-byte aligned rows")
            self.mfma_mg = mfma_mg
            ptrs = [ptr(r) for r in self.inputs]
            stride = ptrs[1] - ptrs[0] if self.k > 1 else 1
            self.in_stride = stride if stride != 0 and all(q - ptrs[0] == j * stride for j, q in enumerate(ptrs)) else 0
            self.bitmat = torch.zeros(hip().fp16_bitmat_bytes(self.k, self.m, mfma_mg), dtype=torch.uint8,
                                      device=self.device)
            if coeff is not None:
                self.set_device_coeff(torch.from_numpy(np.ascontiguousarray(coeff.astype("<u2")).view(np.int16))
                                      .to(self.device))
        self._stripes = (bi, bo, stripes_copy) if hold_buffers else None
        if not hold_buffers:
            self.inputs = self.outputs = self.copies = None
        self._ready = torch.cuda.Event()
        self._ready.record(torch.cuda.current_stream(self.device))

    def set_device_coeff(self, coeff: torch.Tensor, rows=None, stream: torch.cuda.Stream | None = None) -> None:
        """Rebuild the matrix-core bit-matrix from a DEVICE 16-bit matrix (int16 / uint16, >= k
        columns): coefficient row i = coeff[rows[i]] (device int32) or coeff[i]. No host round trip
        (the w = 16 decode feeds it the device-solved decode rows)."""
        if self.engine != "mfma":
            raise ValueError("set_device_coeff applies to engine='mfma' plans")
        if coeff.dtype not in (torch.int16, torch.uint16) or coeff.device != self.device or coeff.dim() != 2 \
                or coeff.shape[1] < self.k:
            raise ValueError("coeff must be a 2-D 16-bit tensor on the plan's device with >= k columns")
        coeff = coeff.contiguous()
        st = stream or torch.cuda.current_stream(self.device)
        sel = 0
        if rows is not None:
            if rows.dtype != torch.int32 or rows.numel() != self.m:
                raise ValueError("rows must be an int32 tensor of m row indices")
            sel = rows.data_ptr()
        elif coeff.shape[0] < self.m:
            raise ValueError("coeff needs m rows")
        hip().fp16_bitmat(coeff.data_ptr(), coeff.stride(0), sel, self.m, self.k, self.bitmat.data_ptr(),
                          self.mfma_mg, st.cuda_stream)
        if not torch.cuda.is_current_stream_capturing():
            coeff.record_stream(st)

    def run(self, stream: torch.cuda.Stream | None = None, col0: int = 0, ncols: int | None = None,
            max_blocks: int = 0) -> None:
        """Launch asynchronously on ``stream`` (default: the current stream); byte columns
        ``[col0, col0 + ncols)``, both even."""
        ncols = self.ncols - col0 if ncols is None else ncols
        if col0 < 0 or ncols < 0 or col0 + ncols > self.ncols or (col0 | ncols) & 1:
            raise ValueError(f"column range [{col0}, {col0 + ncols}) must be whole symbols inside {self.ncols} bytes")
        st = stream or torch.cuda.current_stream(self.device)
        if self._ready is not None:
            st.wait_event(self._ready)
            self._ready = None
        if stream is not None:
            self.desc.record_stream(stream)
        if self.batch > 1:
            if self.engine == "mfma":
                hip().gemm16_fp4_batched(int(self.bitmat.data_ptr()), int(self.desc.data_ptr()), self.k, self.m,
                                         self.batch, col0, ncols, self.mfma_mg, self.in_stride, self.in_bstride,
                                         self.out_bstride, self.has_copies, st.cuda_stream)
            else:
                hip().gemm16_batched(int(self.desc.data_ptr()), self.k, self.m_pad, self.batch, col0, ncols,
                                     self.symwise, st.cuda_stream)
            return
        if self.engine == "mfma" and max_blocks == 0 and col0 % 4 == 0:
            hip().gemm16_fp4(int(self.bitmat.data_ptr()), int(self.desc.data_ptr()), self.k, self.m, col0, ncols,
                             self.mfma_mg, self.in_stride, self.has_copies, st.cuda_stream)
            return
        hip().gemm16(int(self.desc.data_ptr()), self.k, self.m_pad, col0, ncols, self.symwise, max_blocks,
                     st.cuda_stream)


class _null:
    def __enter__(self):
        return None

    def __exit__(self, *a):
        return False


def gf_gemm(coeff, inputs, outputs=None, *, maps=None, copies=None, stream=None) -> torch.Tensor:
    """One-shot GF-GEMM. Returns the output tensor (allocated as [m, C] when ``outputs`` is None)."""
    ins = _rows(inputs)
    m = (np.asarray(coeff).shape[0] if coeff is not None else np.asarray(maps).shape[0])
    if outputs is None:
        c = min(r.numel() for r in ins)
        outputs = torch.empty((m, c), dtype=torch.uint8, device=ins[0].device)
    GemmPlan(ins, outputs, coeff, maps=maps, copies=copies).run(stream)
    return outputs
