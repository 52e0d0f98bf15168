"""Per-step placement of coded bytes over torch.distributed (RCCL over xGMI on MI355X, gloo on CPU).

After every rank has encoded its own stripe, its parity has to leave the GPU for where it is
stored. The reference gathers every device's parity slices into one host buffer after the worker
threads join (``src/encode.cu:410-429``; decode: ``src/decode.cu:380-405``). On an MI355X node the
GPUs are a fully connected xGMI mesh — 7 point-to-point links per GPU — so *where* the parity goes
decides which links carry it:

``root``   every peer sends its whole parity block to rank 0 (the reference's pattern, as grouped
           point-to-point send/recv: each peer drives its own link into rank 0). Rank 0's inbound
           links carry (N-1) blocks per step; the other links of the mesh idle.
``owners`` parity is placed chunk-contiguously: the concatenation of every rank's parity bytes is
           cut into N equal contiguous pieces and rank o owns piece o (it receives 1/N of every
           rank's block). That is one ``all_to_all_single`` in which every link of the mesh carries
           1/N of a block instead of a whole one — N× less traffic on the busiest link than
           ``root``, spread over all N-1 links of every GPU.
``none``   no traffic (compute-only reference point).

:class:`StripeGather` is the strong-scaling form (one stripe column-sharded over all ranks, the
reference's multi-GPU semantics, ``src/encode.cu:368-381``): every rank's column piece of the
parity and decoded rows lands in place in rank 0's full rows.

Exchanges run asynchronously on the process group's own stream (RCCL's internal stream on GPU) so
the next step's encode/decode overlaps them. Every slot has its own receive storage, so exchanges
of consecutive slots never share a destination; :meth:`wait` orders a later overwrite of a source
buffer after the exchange that reads it (double-buffered sources).

With a one-rank RCCL process group (``bench.py --force-pg``, ``GFRS_FORCE_PG=1``) the same calls run
against rank 0 itself: ``owners`` is an ``all_to_all_single`` to self and ``root`` a grouped
send/recv to self, so every RCCL code path executes on a single MI355X.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

MODES = ("owners", "root", "none")


class InjectedFault(RuntimeError):
    """Raised by :func:`maybe_fault` (fault injection for the N > 1 bench's failure isolation)."""


def maybe_fault(mode: str) -> None:
    """Fault injection: ``GFRS_FAULT_MODE=<mode>`` makes the exchange of that mode
    (``owners``, ``root``, ``strong``) fail when it starts — on every rank, or only on rank
    ``GFRS_FAULT_RANK``. ``GFRS_FAULT_KIND=hang`` sleeps instead of raising (a peer that never joins
    its collectives), which is what a stuck xGMI transfer looks like to the other ranks."""
    if os.environ.get("GFRS_FAULT_MODE") != mode:
        return
    want = os.environ.get("GFRS_FAULT_RANK")
    if want not in (None, "") and dist.is_initialized() and int(want) != dist.get_rank():
        return
    if os.environ.get("GFRS_FAULT_KIND", "raise") == "hang":
        import time

        time.sleep(float(os.environ.get("GFRS_FAULT_HANG_S", "3600")))
    raise InjectedFault(f"injected fault in {mode} exchange (GFRS_FAULT_MODE)")


def _gather_small(t: torch.Tensor, dst: int) -> list[torch.Tensor] | None:
    """dist.gather of a small tensor (checksums); gloo gets host copies (it gathers host memory)."""
    if dist.get_backend() == "gloo" and t.is_cuda:
        t = t.cpu()
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())] if dist.get_rank() == dst else None
    dist.gather(t, out, dst=dst)
    return out


class _StagedRecv:
    """A gloo receive into host memory whose bytes are copied to the device tensor on wait()."""

    def __init__(self, work, host: torch.Tensor, dst: torch.Tensor):
        self.work, self.host, self.dst = work, host, dst

    def wait(self) -> None:
        self.work.wait()
        self.dst.copy_(self.host)


def batch_p2p(ops: list[tuple[str, torch.Tensor, int]]) -> list | None:
    """Grouped point-to-point: ``ops`` is a list of ``("send" | "recv", tensor, peer)``; returns the
    works to wait on (None when empty).

    RCCL (and gloo on host tensors) move the tensors in place. gloo cannot send device memory, so a
    gloo group over GPU tensors — the N-ranks-on-one-GPU rehearsal (``bench.py --pg-backend gloo``) —
    stages through host copies: a send copies its piece to the host first, a receive lands in host
    memory and is copied to its device destination by ``wait()``. That path exists only to run the
    rank-0 receive lists and piece bookkeeping of the N > 1 modes on one GPU; it is not timed as a
    link rate."""
    if not ops:
        return None
    staged = dist.get_backend() == "gloo" and any(t.is_cuda for _, t, _ in ops)
    if not staged:
        return dist.batch_isend_irecv([dist.P2POp(dist.isend if kind == "send" else dist.irecv, t, peer)
                                       for kind, t, peer in ops])
    works = []
    for kind, t, peer in ops:
        if kind == "send":
            works.append(dist.isend(t.to("cpu"), peer))
        else:
            host = torch.empty(t.shape, dtype=t.dtype)
            works.append(_StagedRecv(dist.irecv(host, peer), host, t))
    return works


def even_splits(nbytes: int, world: int) -> list[int]:
    """``nbytes`` cut into ``world`` contiguous pieces, sizes differing by at most one byte."""
    base, rem = divmod(nbytes, world)
    return [base + (1 if r < rem else 0) for r in range(world)]


def _checksum(x: torch.Tensor, chunk: int = 1 << 26) -> torch.Tensor:
    """Two int64 digests of a flat uint8 tensor: byte sum and a position-weighted sum of all bytes
    (weights cycle through 1..65536, so a moved or swapped byte changes it). Chunked, so a GiB-sized
    row needs only 2 x 512 MiB of int64 temporaries."""
    out = torch.zeros(2, dtype=torch.int64, device=x.device)
    for a in range(0, x.numel(), chunk):
        c = x[a:a + chunk].to(torch.int64)
        w = torch.arange(a, a + c.numel(), dtype=torch.int64, device=x.device).remainder_(1 << 16).add_(1)
        out[0] += c.sum()
        out[1] += (c * w).sum()
    return out


def _pg_world_rank() -> tuple[int, int, bool]:
    if dist.is_initialized():
        return dist.get_world_size(), dist.get_rank(), True
    return 1, 0, False


def _self_loop() -> bool:
    """A one-rank RCCL group: a rank's own block travels through send/recv to itself (gloo has no
    self point-to-point; there the own block simply stays put)."""
    return dist.is_initialized() and dist.get_world_size() == 1 and dist.get_backend() == "nccl"


class ParityExchange:
    """Moves a rank's flat parity block (one of ``len(sources)`` alternating buffers) per step.

    Args:
        sources: flat contiguous uint8 tensors of equal size (the parity storage, padding included),
            one per pipeline slot. Every rank must pass the same sizes.
        mode: ``"owners"``, ``"root"`` or ``"none"`` (see module docstring).
        root: destination rank of ``"root"``.

    Receive storage is per slot: ``recvs[slot]`` (owners: the pieces this rank owns, in source-rank
    order) and ``recv_lists[slot][r]`` (root, on the root: rank r's block).
    """

    def __init__(self, sources: list[torch.Tensor], mode: str = "owners", root: int = 0):
        if mode not in MODES:
            raise ValueError(f"mode must be one of {MODES}")
        if not sources or any(s.dtype != torch.uint8 or s.dim() != 1 or not s.is_contiguous() for s in sources):
            raise ValueError("sources must be flat contiguous uint8 tensors")
        if len({s.numel() for s in sources}) != 1:
            raise ValueError("every source buffer must have the same size")
        self.sources = sources
        self.world, self.rank, has_pg = _pg_world_rank()
        # a one-rank process group still runs the exchange (against itself): --force-pg
        self.mode = mode if has_pg else "none"
        self.self_loop = _self_loop()
        self.root = root
        self.nbytes = sources[0].numel()
        dev = sources[0].device
        slots = len(sources)
        self.recvs: list[torch.Tensor | None] = [None] * slots
        self.recv_lists: list[list[torch.Tensor | None]] = [[] for _ in range(slots)]
        if self.mode == "owners":
            self.in_splits = even_splits(self.nbytes, self.world)
            mine = self.in_splits[self.rank]
            self.out_splits = [mine] * self.world  # every source sends me its piece `rank`
            self.recvs = [torch.empty(mine * self.world, dtype=torch.uint8, device=dev) for _ in range(slots)]
        elif self.mode == "root" and self.rank == root:
            self.recv_lists = [[torch.empty(self.nbytes, dtype=torch.uint8, device=dev)
                                if (r != root or self.self_loop) else None for r in range(self.world)]
                               for _ in range(slots)]
        self.pending: list[list | None] = [None] * slots

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
        root — a whole block into the root. Zero at world 1 (nothing crosses a link)."""
        if self.world == 1:
            return 0
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
        maybe_fault(self.mode)
        self.wait(slot)
        src = self.sources[slot]
        if self.mode == "owners":
            w = dist.all_to_all_single(self.recvs[slot], src, self.out_splits, self.in_splits, async_op=True)
            self.pending[slot] = [w]
            return
        ops = []
        if self.rank == self.root:
            for r in range(self.world):
                if r != self.root or self.self_loop:
                    ops.append(("recv", self.recv_lists[slot][r], r))
        if self.rank != self.root or self.self_loop:
            ops.append(("send", src, self.root))
        self.pending[slot] = batch_p2p(ops)

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
        """True when what slot ``slot``'s last exchange delivered equals the senders' ``sources[slot]``
        pieces (checksums of every byte, exchanged with the same pattern). Collective: every rank
        must call it."""
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
            recv = self.recvs[slot]
            got = torch.stack([_checksum(recv[r * mine:(r + 1) * mine]) for r in range(self.world)])
            ok = torch.equal(got, expect)
        else:
            allsum = _gather_small(_checksum(src), self.root)
            ok = True
            if self.rank == self.root:
                ok = all(torch.equal(_checksum(self.recv_lists[slot][r]).cpu(), allsum[r].cpu())
                         for r in range(self.world) if r != self.root or self.self_loop)
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        return bool(flag.item())


class StripeGather:
    """Strong scaling's per-step gather: rank r's column piece ``[offs[r], offs[r+1])`` of every row
    lands in place in rank ``dst``'s full rows (the reference's H2H gather of parity and decoded
    slices after its device threads join, ``src/encode.cu:410-429``, ``src/decode.cu:380-405``, as
    grouped point-to-point — one message per (peer, row), each peer on its own xGMI link).

    Args:
        pieces: per slot, this rank's 1-D piece rows (same row count on every rank and slot).
        fulls: per slot, on ``dst`` only: the full rows (``sum(widths)`` bytes each). When dst's
            piece rows are views of the full rows at offset 0 (it computed in place) nothing moves
            for its own piece; otherwise it is copied (or, on a one-rank RCCL group, sent to self).
        widths: every rank's piece width in bytes.
    """

    def __init__(self, pieces: list[list[torch.Tensor]], fulls: list[list[torch.Tensor]] | None,
                 widths: list[int], dst: int = 0):
        self.world, self.rank, self.has_pg = _pg_world_rank()
        if len(widths) != self.world:
            raise ValueError("widths must list every rank's piece width")
        self.pieces, self.fulls, self.widths, self.dst = pieces, fulls, widths, dst
        self.offs = [0]
        for w in widths:
            self.offs.append(self.offs[-1] + w)
        if any(len(p) != len(pieces[0]) for p in pieces) or any(r.numel() < widths[self.rank] for p in pieces for r in p):
            raise ValueError("every slot needs the same number of piece rows, each widths[rank] bytes")
        if self.rank == dst:
            if fulls is None or len(fulls) != len(pieces) or any(len(f) != len(pieces[0]) for f in fulls):
                raise ValueError("rank dst needs full rows for every slot")
            if any(r.numel() < self.offs[-1] for f in fulls for r in f):
                raise ValueError("full rows must hold sum(widths) bytes")
        self.self_loop = _self_loop()
        self.pending: list[list | None] = [None] * len(pieces)

    def _in_place(self, slot: int) -> bool:
        """dst computed its own piece inside its full rows: every piece row starts at column
        offs[dst] of the matching full row."""
        if self.widths[self.dst] == 0:
            return True
        a = self.offs[self.dst]
        return all(p.data_ptr() == f[a:].data_ptr() for p, f in zip(self.pieces[slot], self.fulls[slot]))

    @property
    def bytes_per_link(self) -> int:
        """Bytes the busiest link into dst carries per step (one peer's piece of every row)."""
        rows = len(self.pieces[0])
        peers = [self.widths[r] for r in range(self.world) if r != self.dst]
        return rows * max(peers) if peers else 0

    @property
    def bytes_received(self) -> int:
        rows = len(self.pieces[0])
        return rows * (self.offs[-1] - self.widths[self.dst]) if self.rank == self.dst else 0

    def start(self, slot: int) -> None:
        maybe_fault("strong")
        self.wait(slot)
        w_mine = self.widths[self.rank]
        ops = []
        if self.rank == self.dst:
            full, mine = self.fulls[slot], self.pieces[slot]
            own_moves = w_mine and not self._in_place(slot)
            for r in range(self.world):
                if r == self.dst or not self.widths[r]:
                    continue
                a, b = self.offs[r], self.offs[r + 1]
                ops += [("recv", row[a:b], r) for row in full]
            if own_moves:
                a, b = self.offs[self.dst], self.offs[self.dst + 1]
                if self.self_loop:
                    for row, src in zip(full, mine):
                        ops += [("recv", row[a:b], self.dst), ("send", src[:w_mine], self.dst)]
                else:
                    for row, src in zip(full, mine):
                        row[a:b].copy_(src[:w_mine], non_blocking=True)
        elif w_mine:
            ops += [("send", row[:w_mine], self.dst) for row in self.pieces[slot]]
        self.pending[slot] = batch_p2p(ops)

    def wait(self, slot: int) -> None:
        works = self.pending[slot]
        if works:
            for w in works:
                w.wait()
        self.pending[slot] = None

    def drain(self) -> None:
        for s in range(len(self.pieces)):
            self.wait(s)

    def verify(self, slot: int) -> bool:
        """dst's full rows equal every rank's pieces (checksums of every byte). Collective."""
        self.drain()
        dev = self.pieces[slot][0].device
        w_mine = self.widths[self.rank]
        mine = torch.stack([_checksum(r[:w_mine]) for r in self.pieces[slot]])  # [rows, 2]
        if self.world == 1 and not self.has_pg:
            allsum = [mine]
        else:
            allsum = _gather_small(mine, self.dst)
        ok = True
        if self.rank == self.dst:
            for r in range(self.world):
                a, b = self.offs[r], self.offs[r + 1]
                got = torch.stack([_checksum(row[a:b]) for row in self.fulls[slot]])
                ok = ok and torch.equal(got.cpu(), allsum[r].cpu())
        if not self.has_pg:
            return bool(ok)
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        return bool(flag.item())
