"""Per-step parity placement over torch.distributed (RCCL over xGMI on MI355X, gloo on CPU).

After every rank has encoded its own stripe, its parity has to leave the GPU for where it is
stored. The reference gathers every device's parity slices into one host buffer after the worker
threads join (``src/encode.cu:410-429``; decode: ``src/decode.cu:380-405``). On an MI355X node the
GPUs are a fully connected xGMI mesh — 7 point-to-point links per GPU — so *where* the parity goes
decides which links carry it:

``root``   every peer sends its whole parity block to rank 0 (the reference's pattern, as grouped
           point-to-point send/recv: each peer drives its own link into rank 0). Rank 0's inbound
           links carry (N-1) blocks per step; the other 6·N links of the mesh idle.
``owners`` parity is placed chunk-contiguously: the concatenation of every rank's parity bytes is
           cut into N equal contiguous pieces and rank o owns piece o (it receives 1/N of every
           rank's block). That is one ``all_to_all_single`` in which every link of the mesh carries
           1/N of a block instead of a whole one — the xGMI-native placement: N× less traffic on the
           busiest link than ``root``, spread over all N-1 links of every GPU.
``none``   no traffic (compute-only reference point).

Exchanges run asynchronously on the process group's own stream (RCCL's internal stream on GPU) so
the next step's encode/decode overlaps them; :meth:`ParityExchange.wait` orders a later overwrite
of a source buffer after the exchange that reads it (double-buffered sources).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

MODES = ("owners", "root", "none")


def even_splits(nbytes: int, world: int) -> list[int]:
    """``nbytes`` cut into ``world`` contiguous pieces, sizes differing by at most one byte."""
    base, rem = divmod(nbytes, world)
    return [base + (1 if r < rem else 0) for r in range(world)]


def _checksum(x: torch.Tensor) -> torch.Tensor:
    """Two int64 digests of a flat uint8 tensor: byte sum and a position-weighted sum of a prefix."""
    n = min(x.numel(), 1 << 16)
    w = torch.arange(1, n + 1, dtype=torch.int64, device=x.device)
    return torch.stack([x.sum(dtype=torch.int64), (x[:n].to(torch.int64) * w).sum()])


class ParityExchange:
    """Moves a rank's flat parity block (one of ``len(sources)`` alternating buffers) per step.

    Args:
        sources: flat contiguous uint8 tensors of equal size (the parity storage, padding included),
            one per pipeline slot. Every rank must pass the same sizes.
        mode: ``"owners"``, ``"root"`` or ``"none"`` (see module docstring).
        root: destination rank of ``"root"``.
    """

    def __init__(self, sources: list[torch.Tensor], mode: str = "owners", root: int = 0):
        if mode not in MODES:
            raise ValueError(f"mode must be one of {MODES}")
        if not sources or any(s.dtype != torch.uint8 or s.dim() != 1 or not s.is_contiguous() for s in sources):
            raise ValueError("sources must be flat contiguous uint8 tensors")
        if len({s.numel() for s in sources}) != 1:
            raise ValueError("every source buffer must have the same size")
        self.sources = sources
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.mode = mode if self.world > 1 else "none"
        self.root = root
        self.nbytes = sources[0].numel()
        dev = sources[0].device
        self.recv: torch.Tensor | None = None
        self.recv_list: list[torch.Tensor | None] = []
        if self.mode == "owners":
            self.in_splits = even_splits(self.nbytes, self.world)
            mine = self.in_splits[self.rank]
            self.out_splits = [mine] * self.world  # every source sends me its piece `rank`
            self.recv = torch.empty(mine * self.world, dtype=torch.uint8, device=dev)
        elif self.mode == "root" and self.rank == root:
            self.recv_list = [torch.empty(self.nbytes, dtype=torch.uint8, device=dev) if r != root else None
                              for r in range(self.world)]
        self.pending: list[list | None] = [None] * len(sources)

    # ---- traffic accounting (per step) ---------------------------------------------------------
    @property
    def bytes_sent(self) -> int:
        """Bytes this rank sends to other ranks per step."""
        if self.mode == "owners":
            return self.nbytes - self.in_splits[self.rank]
        if self.mode == "root":
            return 0 if self.rank == self.root else self.nbytes
        return 0

    @property
    def bytes_received(self) -> int:
        if self.mode == "owners":
            return self.in_splits[self.rank] * (self.world - 1)
        if self.mode == "root":
            return self.nbytes * (self.world - 1) if self.rank == self.root else 0
        return 0

    @property
    def bytes_per_link(self) -> int:
        """Bytes the busiest point-to-point link carries per step (one direction): owners — one
        rank's piece (every ordered pair of ranks exchanges one piece over its direct xGMI link);
        root — a whole block into the root."""
        if self.mode == "owners":
            return max(self.in_splits)
        if self.mode == "root":
            return self.nbytes
        return 0

    # ---- per-step ------------------------------------------------------------------------------
    def start(self, slot: int) -> None:
        """Launch the exchange of ``sources[slot]`` asynchronously (ordered after the work queued so
        far on the current stream)."""
        if self.mode == "none":
            return
        self.wait(slot)
        src = self.sources[slot]
        if self.mode == "owners":
            w = dist.all_to_all_single(self.recv, src, self.out_splits, self.in_splits, async_op=True)
            self.pending[slot] = [w]
            return
        ops = []
        if self.rank == self.root:
            for r in range(self.world):
                if r != self.root:
                    ops.append(dist.P2POp(dist.irecv, self.recv_list[r], r))
        else:
            ops.append(dist.P2POp(dist.isend, src, self.root))
        self.pending[slot] = dist.batch_isend_irecv(ops) if ops else None

    def wait(self, slot: int) -> None:
        """Order later work on the current stream after the exchange reading ``sources[slot]``."""
        works = self.pending[slot]
        if works:
            for w in works:
                w.wait()
        self.pending[slot] = None

    def drain(self) -> None:
        for s in range(len(self.sources)):
            self.wait(s)

    # ---- verification (outside timed regions) ---------------------------------------------------
    def verify(self, slot: int) -> bool:
        """True when what the last exchange delivered equals the senders' ``sources[slot]`` pieces
        (checksums exchanged with the same pattern). Collective: every rank must call it."""
        if self.mode == "none":
            return True
        self.drain()
        src = self.sources[slot]
        dev = src.device
        if self.mode == "owners":
            offs = [0]
            for s in self.in_splits:
                offs.append(offs[-1] + s)
            send = torch.stack([_checksum(src[offs[o]:offs[o + 1]]) for o in range(self.world)])  # [world, 2]
            expect = torch.empty_like(send)
            dist.all_to_all_single(expect, send)
            mine = self.in_splits[self.rank]
            got = torch.stack([_checksum(self.recv[r * mine:(r + 1) * mine]) for r in range(self.world)])
            # my own piece never travels: it is compared against itself (recv holds a copy of it)
            ok = torch.equal(got, expect)
        else:
            mine = _checksum(src)
            allsum = [torch.empty_like(mine) for _ in range(self.world)] if self.rank == self.root else None
            dist.gather(mine, allsum, dst=self.root)
            ok = True
            if self.rank == self.root:
                ok = all(torch.equal(_checksum(self.recv_list[r]), allsum[r])
                         for r in range(self.world) if r != self.root)
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        return bool(flag.item())
