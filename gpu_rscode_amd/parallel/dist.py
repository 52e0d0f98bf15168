"""Stripe-sharded data parallelism over torch.distributed (RCCL over xGMI on MI355X, gloo on CPU).

The reference's only multi-GPU strategy is column-sharded data parallelism inside one process:
``minChunkSizePerDevice = C / GPU_num`` with the remainder on the last device
(``src/encode.cu:368-381``), host-staged H2H copies in (``:389-398``) and out (``:410-429``), E
recomputed per device (``:141``) and the decode inverse shared by host pointer
(``src/decode.cu:375``). Here every GPU is its own rank and the four hand-offs become collectives
(SURVEY §5.8):

  =====================================  ====================================================
  reference site                         here
  =====================================  ====================================================
  E generated on every device (:141)     :func:`broadcast_matrix` from rank 0
  A^-1 shared by host pointer            :func:`broadcast_matrix` (or identical device inverse)
  stripe scatter via H2H (:389-398)      :func:`scatter_columns` (point-to-point isend/irecv)
  parity gather via H2H (:410-429)       :func:`gather_columns` / :func:`gather_pieces`
                                         (point-to-point, received in place on rank 0)
  =====================================  ====================================================

xGMI is point-to-point (7 links per GPU), so scatter/gather use one send per peer — each peer
drives its own link into rank 0 — instead of a ring collective whose per-hop forwarding would be
link-bound. Shards are 4 KiB-aligned column ranges so every rank's rows stay 16-byte aligned.
"""
from __future__ import annotations

import datetime
import os
import socket
from dataclasses import dataclass

import numpy as np
import torch
import torch.distributed as dist

from ..models.rs import ReedSolomon, alloc_rows

SHARD_ALIGN = 4096
IPC_ENV = "HSA_ENABLE_IPC_MODE_LEGACY"


def default_pg_timeout() -> float:
    """Process-group timeout (s) of every entry point that does not pass its own: GFRS_PG_TIMEOUT_S,
    else 300 (``bench.py`` passes a longer one that covers its budgets)."""
    return float(os.environ.get("GFRS_PG_TIMEOUT_S", 300))


def ensure_ipc_env(backend: str) -> None:
    """RCCL peers on this driver need dmabuf IPC (``HSA_ENABLE_IPC_MODE_LEGACY=0``; without it
    ``hipIpcGetMemHandle`` fails when the first peer buffer is shared). The HIP runtime reads the
    variable once, when it initialises: set it here if HIP has not started yet, and refuse to build
    an RCCL group if it has started without it (the package's ``__init__`` sets it before importing
    torch, so every entry point through the package gets it in time)."""
    if backend != "nccl" or os.environ.get(IPC_ENV) == "0":
        return
    if torch.cuda.is_initialized():
        raise RuntimeError(f"{IPC_ENV}=0 must be set before HIP initialises (RCCL peers use dmabuf IPC on this "
                           "driver); export it before the process starts")
    os.environ[IPC_ENV] = "0"


@dataclass
class DistContext:
    rank: int
    world: int
    local_rank: int
    device: torch.device
    backend: str

    @property
    def is_root(self) -> bool:
        return self.rank == 0


def init_distributed(backend: str | None = None, force_pg: bool | None = None,
                     timeout_s: float | None = None) -> DistContext:
    """Initialise from torchrun's environment (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_*).

    The process group gets a bounded timeout (``timeout_s``, default :func:`default_pg_timeout`):
    a collective whose peer is gone raises (gloo) or is aborted by the RCCL watchdog after at most
    that long, instead of hanging the job.

    Backend defaults to ``nccl`` (RCCL) when a GPU is visible, else ``gloo``. Safe to call when a
    process group already exists. At world 1 no process group is created unless ``force_pg`` (or
    ``GFRS_FORCE_PG=1``): then a one-rank group runs every collective against rank 0 itself, which
    is how the RCCL code paths execute on a single MI355X (tests, ``bench.py --force-pg``).
    """
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if (world > 1 or force_pg) and backend in (None, "nccl"):
        ensure_ipc_env("nccl")  # (before torch.cuda.set_device initialises HIP below)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if force_pg is None:
        force_pg = os.environ.get("GFRS_FORCE_PG") == "1"
    use_gpu = torch.cuda.is_available() and torch.cuda.device_count() > 0 and backend != "gloo"
    if use_gpu:
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    backend = backend or ("nccl" if use_gpu else "gloo")
    if world > 1 or force_pg:
        ensure_ipc_env(backend)
    if (world > 1 or force_pg) and not dist.is_initialized():
        kw = {"device_id": device} if device.type == "cuda" else {}
        if world == 1 and "MASTER_PORT" not in os.environ:
            kw.update(init_method=f"tcp://127.0.0.1:{free_port()}", rank=0, world_size=1)
        if timeout_s is None:
            timeout_s = default_pg_timeout()
        dist.init_process_group(backend, timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return DistContext(rank, world, local, device, backend)


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _world() -> int:
    return dist.get_world_size() if dist.is_initialized() else 1


def _self_p2p() -> bool:
    """A one-rank process group: a rank's own piece moves through RCCL send/recv to itself, so the
    grouped point-to-point path of N > 1 runs unchanged at world 1 (--force-pg)."""
    return dist.is_initialized() and dist.get_world_size() == 1 and dist.get_backend() == "nccl"


def _rank() -> int:
    return dist.get_rank() if dist.is_initialized() else 0


def shard_range(ncols: int, world: int, rank: int, align: int = SHARD_ALIGN) -> tuple[int, int]:
    """Contiguous column shard of rank ``rank``: aligned equal shares, remainder on the last rank
    (the reference's split, ``src/encode.cu:368-381``)."""
    per = (ncols // world) // align * align
    a = rank * per
    b = ncols if rank == world - 1 else a + per
    return a, b


_BCAST_DTYPES = {np.dtype(np.uint8): torch.uint8, np.dtype(np.int32): torch.int32}


def broadcast_matrix(mat: np.ndarray | None, device: torch.device, src: int = 0, dtype=np.uint8) -> np.ndarray:
    """Broadcast a small matrix from ``src`` to every rank: E or a decode inverse (``dtype`` uint8:
    GF(2^8) symbols), GF(2^16) symbols or chunk ids (``int32``: values up to 65535 survive, which a
    byte broadcast would truncate past 255). Returns ``dtype``."""
    dt = np.dtype(dtype)
    if dt not in _BCAST_DTYPES:
        raise ValueError(f"broadcast_matrix: dtype {dt} (uint8 or int32)")
    if not dist.is_initialized():
        return np.asarray(mat).astype(dt)
    shape = torch.zeros(2, dtype=torch.int64, device=device)
    if _rank() == src:
        m = np.asarray(mat)
        if m.size and (m.min() < np.iinfo(dt).min or m.max() > np.iinfo(dt).max):
            raise ValueError(f"broadcast_matrix: values outside {dt}")
        m = np.ascontiguousarray(m.astype(dt))
        shape[0], shape[1] = m.shape
    dist.broadcast(shape, src)
    rows, cols = int(shape[0]), int(shape[1])
    buf = torch.empty((rows, cols), dtype=_BCAST_DTYPES[dt], device=device)
    if _rank() == src:
        buf.copy_(torch.from_numpy(m))
    dist.broadcast(buf, src)
    return buf.cpu().numpy()


def _aligned_rows(t: torch.Tensor) -> bool:
    return t.stride(1) == 1 and t.data_ptr() % 16 == 0 and (t.shape[0] <= 1 or t.stride(0) % 16 == 0)


def scatter_columns(full: torch.Tensor | None, rows: int, ncols: int, device: torch.device, src: int = 0,
                    align: int = SHARD_ALIGN) -> torch.Tensor:
    """Rank ``src`` holds ``full`` [rows, ncols] (unit column stride); every rank gets its column
    shard [rows, b - a] on ``device``.

    Point-to-point, one message per (peer, row): every row piece travels straight from its place in
    ``full`` into the receiver's pitched shard (256-byte row pitch, 16-byte aligned rows for the GEMM
    kernels) — no staging copies on either side. Rank ``src`` returns a view of its own shard inside
    ``full`` when that is already on ``device`` with 16-byte aligned rows (nothing moves); otherwise
    its shard is copied into pitched rows on ``device`` (through RCCL send/recv to itself on a
    one-rank group), so no rank falls back to the bytewise kernel for an odd C."""
    world, rank = _world(), _rank()
    a, b = shard_range(ncols, world, rank, align)
    own_p2p = False
    if rank == src:
        if full is None or full.dim() != 2 or full.stride(1) != 1 or full.shape[0] != rows or full.shape[1] < ncols:
            raise ValueError("scatter_columns: rank src needs full [rows, >= ncols] with unit column stride")
        view = full[:, a:b]
        if full.device == device and _aligned_rows(view):
            local = view
        else:
            local = alloc_rows(rows, b - a, device)
            own_p2p = _self_p2p() and full.device == device and device.type == "cuda"
            if not own_p2p:
                local.copy_(view)
    else:
        local = alloc_rows(rows, b - a, device)
    if not dist.is_initialized():
        return local
    ops = []
    if rank == src:
        for r in range(world):
            ra, rb = shard_range(ncols, world, r, align)
            if r != src and rb > ra:
                ops += [dist.P2POp(dist.isend, full[i, ra:rb], r) for i in range(rows)]
        if own_p2p and b > a:
            for i in range(rows):
                ops += [dist.P2POp(dist.isend, full[i, a:b], src), dist.P2POp(dist.irecv, local[i], src)]
    elif b > a:
        ops += [dist.P2POp(dist.irecv, local[i], src) for i in range(rows)]
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    return local


def gather_pieces(local: torch.Tensor, widths: list[int], dst: int = 0,
                  out: torch.Tensor | None = None) -> torch.Tensor | None:
    """Rank r contributes ``local`` [rows, widths[r]] (rows 1-D contiguous); rank ``dst`` returns the
    pieces side by side in rank order as one [rows, sum(widths)] tensor (``out`` if given, else a new
    pitched one), others None.

    One point-to-point message per (peer, row), received in place into the destination's column
    slice — each peer drives its own xGMI link into ``dst``. dst's own piece is not moved when
    ``local`` already is that slice of ``out``; otherwise it is copied (RCCL send/recv to itself on a
    one-rank group)."""
    world, rank = _world(), _rank()
    rows = local.shape[0]
    if len(widths) != world or local.shape[1] != widths[rank]:
        raise ValueError("gather_pieces: widths must list every rank's piece width (this rank's = local.shape[1])")
    if out is None and not dist.is_initialized():
        return local  # one process, no group: the piece is the whole
    ops = []
    full = None
    if rank == dst:
        offs = [0]
        for w in widths:
            offs.append(offs[-1] + w)
        if out is None:
            full = alloc_rows(rows, offs[-1], local.device)
        else:
            if out.dim() != 2 or out.shape[0] != rows or out.shape[1] < offs[-1] or out.stride(1) != 1:
                raise ValueError("gather_pieces: out must be [rows, >= sum(widths)] with unit column stride")
            full = out
        mine = full[:, offs[dst]:offs[dst + 1]]
        if widths[dst] and mine.data_ptr() != local.data_ptr():
            if _self_p2p() and local.device.type == "cuda":
                for i in range(rows):
                    ops += [dist.P2POp(dist.isend, local[i], dst), dist.P2POp(dist.irecv, mine[i], dst)]
            else:
                mine.copy_(local)
        for r in range(world):
            if r != dst and widths[r]:
                ops += [dist.P2POp(dist.irecv, full[i, offs[r]:offs[r + 1]], r) for i in range(rows)]
    elif widths[rank]:
        ops += [dist.P2POp(dist.isend, local[i], dst) for i in range(rows)]
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    return full


def gather_columns(local: torch.Tensor, ncols: int, dst: int = 0, align: int = SHARD_ALIGN) -> torch.Tensor | None:
    """Inverse of :func:`scatter_columns`: rank ``dst`` returns [rows, ncols], others None."""
    world = _world()
    widths = [b - a for a, b in (shard_range(ncols, world, r, align) for r in range(world))]
    return gather_pieces(local, widths, dst)


class DistributedRS:
    """A (k, n) codec whose stripes are column-sharded over all ranks.

    Rank 0 owns the coding matrix and broadcasts it, so every rank encodes with bit-identical
    tables even if ranks were configured differently (the reference regenerates E per device).
    ``field`` as :class:`~gpu_rscode_amd.models.ReedSolomon`: ``"gf256"`` (the reference's bytes),
    ``"gf65536"`` (16-bit symbols, n <= 65535, ``src/galoisfield.cu:22-32``; shards then hold whole
    symbols — the 4 KiB shard alignment is even) or ``"gf16"``. Matrices and survivor ids travel as
    int32 for every field wider than a byte.
    """

    def __init__(self, k: int, n: int, ctx: DistContext, matrix: str = "vandermonde", field: str = "gf256"):
        self.ctx = ctx
        self.rs = ReedSolomon(k, n, matrix=matrix, field=field)
        self.field = field
        dt = self.rs.E.dtype
        wire = np.int32 if dt.itemsize > 1 else np.uint8
        self.rs.E = broadcast_matrix(self.rs.E if ctx.is_root else None, ctx.device, dtype=wire).astype(dt)
        self.rs.G = np.vstack([np.eye(k, dtype=dt), self.rs.E])
        self.k, self.n, self.p = k, n, n - k

    def encode_local(self, data_shard, parity_shard=None):
        """Encode this rank's column shard (no communication)."""
        return self.rs.encode(data_shard, parity_shard)

    def decode_local(self, survivors_shard, rows, out=None, device_invert: bool = False):
        return self.rs.decode(survivors_shard, rows, out=out, device_invert=device_invert)

    def encode_global(self, data: torch.Tensor | None, ncols: int) -> torch.Tensor | None:
        """Rank 0's [k, C] stripe -> scatter -> per-rank encode -> parity gathered on rank 0."""
        shard = scatter_columns(data, self.k, ncols, self.ctx.device)
        parity = self.encode_local(shard)
        if self.ctx.device.type == "cuda":
            torch.cuda.synchronize(self.ctx.device)
        return gather_columns(parity, ncols)

    def decode_global(self, survivors: torch.Tensor | None, rows, ncols: int) -> torch.Tensor | None:
        """Rank 0's k survivor rows (chunk ids ``rows``) -> natives [k, C] on rank 0."""
        rows = [int(r) for r in broadcast_matrix(np.asarray([rows]) if self.ctx.is_root else None,
                                                 self.ctx.device, dtype=np.int32)[0]]
        shard = scatter_columns(survivors, self.k, ncols, self.ctx.device)
        out = self.decode_local(shard, rows)
        if self.ctx.device.type == "cuda":
            torch.cuda.synchronize(self.ctx.device)
        return gather_columns(out, ncols)
