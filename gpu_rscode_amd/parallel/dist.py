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
  parity gather via H2H (:410-429)       :func:`gather_columns`  (point-to-point into rank 0)
  =====================================  ====================================================

xGMI is point-to-point (7 links per GPU), so scatter/gather use one send per peer — each peer
drives its own link into rank 0 — instead of a ring collective whose per-hop forwarding would be
link-bound. Shards are 4 KiB-aligned column ranges so every rank's rows stay 16-byte aligned.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np
import torch
import torch.distributed as dist

from ..models.rs import ReedSolomon, alloc_rows

SHARD_ALIGN = 4096


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


def init_distributed(backend: str | None = None) -> DistContext:
    """Initialise from torchrun's environment (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_*).

    Backend defaults to ``nccl`` (RCCL) when a GPU is visible, else ``gloo``. Safe to call when a
    process group already exists.
    """
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_gpu = torch.cuda.is_available() and torch.cuda.device_count() > 0 and backend != "gloo"
    if use_gpu:
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    backend = backend or ("nccl" if use_gpu else "gloo")
    if world > 1 and not dist.is_initialized():
        kw = {"device_id": device} if device.type == "cuda" else {}
        dist.init_process_group(backend, **kw)
    return DistContext(rank, world, local, device, backend)


def _world() -> int:
    return dist.get_world_size() if dist.is_initialized() else 1


def _rank() -> int:
    return dist.get_rank() if dist.is_initialized() else 0


def shard_range(ncols: int, world: int, rank: int, align: int = SHARD_ALIGN) -> tuple[int, int]:
    """Contiguous column shard of rank ``rank``: aligned equal shares, remainder on the last rank
    (the reference's split, ``src/encode.cu:368-381``)."""
    per = (ncols // world) // align * align
    a = rank * per
    b = ncols if rank == world - 1 else a + per
    return a, b


def broadcast_matrix(mat: np.ndarray | None, device: torch.device, src: int = 0) -> np.ndarray:
    """Broadcast a small uint8 matrix (E, or a decode inverse) from ``src`` to every rank."""
    if _world() == 1:
        return np.asarray(mat, dtype=np.uint8)
    shape = torch.zeros(2, dtype=torch.int64, device=device)
    if _rank() == src:
        m = np.ascontiguousarray(mat, dtype=np.uint8)
        shape[0], shape[1] = m.shape
    dist.broadcast(shape, src)
    rows, cols = int(shape[0]), int(shape[1])
    buf = torch.empty((rows, cols), dtype=torch.uint8, device=device)
    if _rank() == src:
        buf.copy_(torch.from_numpy(m))
    dist.broadcast(buf, src)
    return buf.cpu().numpy()


def scatter_columns(full: torch.Tensor | None, rows: int, ncols: int, device: torch.device, src: int = 0,
                    align: int = SHARD_ALIGN) -> torch.Tensor:
    """Rank ``src`` holds ``full`` [rows, ncols]; every rank receives its column shard
    [rows, b - a] (256-byte pitched rows). Point-to-point, one send per peer."""
    world, rank = _world(), _rank()
    a, b = shard_range(ncols, world, rank, align)
    local = alloc_rows(rows, b - a, device)
    if world == 1:
        local.copy_(full[:, a:b])
        return local
    recv = torch.empty((rows, b - a), dtype=torch.uint8, device=device)
    ops = []
    keep = []
    if rank == src:
        for r in range(world):
            ra, rb = shard_range(ncols, world, r, align)
            if r == src:
                recv.copy_(full[:, ra:rb])
                continue
            piece = full[:, ra:rb].contiguous()
            keep.append(piece)
            ops.append(dist.P2POp(dist.isend, piece, r))
    else:
        ops.append(dist.P2POp(dist.irecv, recv, src))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    local.copy_(recv)
    return local


def gather_columns(local: torch.Tensor, ncols: int, dst: int = 0, align: int = SHARD_ALIGN) -> torch.Tensor | None:
    """Inverse of :func:`scatter_columns`: rank ``dst`` returns [rows, ncols], others None."""
    world, rank = _world(), _rank()
    if world == 1:
        return local.clone()
    rows = local.shape[0]
    ops, bufs = [], {}
    if rank == dst:
        full = torch.empty((rows, ncols), dtype=torch.uint8, device=local.device)
        for r in range(world):
            ra, rb = shard_range(ncols, world, r, align)
            if r == dst:
                full[:, ra:rb].copy_(local)
                continue
            bufs[r] = torch.empty((rows, rb - ra), dtype=torch.uint8, device=local.device)
            ops.append(dist.P2POp(dist.irecv, bufs[r], r))
    else:
        send = local.contiguous()
        ops.append(dist.P2POp(dist.isend, send, dst))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    if rank != dst:
        return None
    for r, buf in bufs.items():
        ra, rb = shard_range(ncols, world, r, align)
        full[:, ra:rb].copy_(buf)
    return full


class DistributedRS:
    """A (k, n) codec whose stripes are column-sharded over all ranks.

    Rank 0 owns the coding matrix and broadcasts it, so every rank encodes with bit-identical
    tables even if ranks were configured differently (the reference regenerates E per device).
    """

    def __init__(self, k: int, n: int, ctx: DistContext, matrix: str = "vandermonde"):
        self.ctx = ctx
        self.rs = ReedSolomon(k, n, matrix=matrix)
        self.rs.E = broadcast_matrix(self.rs.E if ctx.is_root else None, ctx.device)
        self.rs.G = np.vstack([np.eye(k, dtype=np.uint8), self.rs.E])
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
        rows = [int(r) for r in broadcast_matrix(np.asarray([rows], dtype=np.uint8) if self.ctx.is_root else None,
                                                 self.ctx.device)[0]]
        shard = scatter_columns(survivors, self.k, ncols, self.ctx.device)
        out = self.decode_local(shard, rows)
        if self.ctx.device.type == "cuda":
            torch.cuda.synchronize(self.ctx.device)
        return gather_columns(out, ncols)
