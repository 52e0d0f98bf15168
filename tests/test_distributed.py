"""Multi-process stripe sharding over torch.distributed (gloo on CPU, world sizes 2 and 3).

The same code path runs over RCCL on MI355X (bench.py, N > 1); here it is exercised with the gloo
backend so the distributed logic is covered without a GPU.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gpu_rscode_amd.gf import GF256
from gpu_rscode_amd.parallel import dist as pdist


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, fn_name):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    ctx = pdist.init_distributed(backend="gloo")
    try:
        globals()[fn_name](ctx)
    finally:
        dist.destroy_process_group()


def _run(fn_name, world=2):
    mp.spawn(_worker, args=(world, _free_port(), fn_name), nprocs=world, join=True)


def test_shard_range_partitions_and_aligns():
    for ncols in (1, 4095, 4096 * 7 + 3, 107374183):
        for world in (1, 2, 3, 8):
            spans = [pdist.shard_range(ncols, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == ncols
            for (a, b), (c, _) in zip(spans, spans[1:]):
                assert b == c and a % 4096 == 0


def _case_broadcast(ctx):
    e = GF256.vandermonde_ref(10, 4) if ctx.rank == 0 else None
    got = pdist.broadcast_matrix(e, ctx.device)
    assert np.array_equal(got, GF256.vandermonde_ref(10, 4))


def _case_scatter_gather(ctx):
    C = 3 * 4096 + 123
    full = torch.arange(5 * C, dtype=torch.int64).remainder(251).to(torch.uint8).view(5, C)
    shard = pdist.scatter_columns(full if ctx.rank == 0 else None, 5, C, ctx.device)
    a, b = pdist.shard_range(C, ctx.world, ctx.rank)
    assert torch.equal(shard, full[:, a:b])
    back = pdist.gather_columns(shard, C)
    if ctx.rank == 0:
        assert torch.equal(back, full)
    else:
        assert back is None


def _case_distributed_codec(ctx):
    k, n, C = 10, 14, 5 * 4096 + 77
    drs = pdist.DistributedRS(k, n, ctx)
    data = torch.from_numpy(np.random.default_rng(0).integers(0, 256, size=(k, C), dtype=np.uint8))
    parity = drs.encode_global(data if ctx.rank == 0 else None, C)
    if ctx.rank == 0:
        assert np.array_equal(parity.numpy(), GF256.gemm(GF256.vandermonde_ref(k, n - k), data.numpy()))
        stripe = torch.cat([data, parity])
        rows = [0, 1, 3, 5, 6, 8, 10, 11, 12, 13]
        surv = stripe[rows]
    else:
        rows, surv = None, None
    out = drs.decode_global(surv, rows, C)
    if ctx.rank == 0:
        assert torch.equal(out, data)


def _case_distributed_codec16(ctx):
    """GF(2^16) over the process group: E broadcast as int32 (16-bit symbols), survivor ids > 255
    broadcast as int32 (a byte broadcast would wrap 256..269 to 0..13 and decode garbage), shards of
    whole symbols; bit-exact against the single-process codec."""
    from gpu_rscode_amd.models import ReedSolomon

    k, n, C = 250, 270, 3 * 4096 + 78  # C even: whole 16-bit symbols
    drs = pdist.DistributedRS(k, n, ctx, field="gf65536")
    ref = ReedSolomon(k, n, field="gf65536")
    assert drs.rs.E.dtype == np.uint16 and np.array_equal(drs.rs.E, ref.E)
    data = torch.from_numpy(np.random.default_rng(1).integers(0, 256, size=(k, C), dtype=np.uint8))
    parity = drs.encode_global(data if ctx.rank == 0 else None, C)
    if ctx.rank == 0:
        want = torch.zeros((n - k, C), dtype=torch.uint8)
        ref.encode(data, want)
        assert torch.equal(parity, want)
        stripe = torch.cat([data, parity])
        rows = list(range(20, k)) + list(range(k, n))  # natives 0..19 erased: parity ids 250..269 used
        assert max(rows) > 255
        surv = stripe[rows]
    else:
        rows, surv = None, None
    out = drs.decode_global(surv, rows, C)
    if ctx.rank == 0:
        assert torch.equal(out, data)


def _case_parity_exchange(ctx):
    """ParityExchange delivers exactly the senders' bytes: owners = piece `rank` of every rank's
    block, in source order; root = every peer's whole block on rank 0. Two alternating slots, each
    with its own receive storage."""
    from gpu_rscode_amd.parallel.placement import ParityExchange, even_splits

    nbytes = 3 * 4096 + 17  # not divisible by the world size: uneven pieces

    def block(r, slot):
        return torch.arange(nbytes, dtype=torch.int64).add(7 * r + 131 * slot).remainder(251).to(torch.uint8)

    def check(x, mode, slot):
        if mode == "owners":
            sp = even_splits(nbytes, ctx.world)
            off = sum(sp[: ctx.rank])
            mine = sp[ctx.rank]
            want = torch.cat([block(r, slot)[off:off + mine] for r in range(ctx.world)])
            assert torch.equal(x.recvs[slot], want), (mode, slot)
            assert x.bytes_sent == nbytes - mine and x.bytes_received == mine * (ctx.world - 1)
        elif mode == "root" and ctx.rank == 0:
            for r in range(1, ctx.world):
                assert torch.equal(x.recv_lists[slot][r], block(r, slot)), (mode, slot, r)

    srcs = [block(ctx.rank, s) for s in range(2)]
    for mode in ("owners", "root", "none"):
        x = ParityExchange(srcs, mode)
        for slot in (0, 1, 0):
            x.start(slot)
            x.wait(slot)
            check(x, mode, slot)
            assert x.verify(slot)
        # both slots in flight at once: start(0), start(1), wait(0), wait(1) — neither slot's
        # delivery may be torn by the other's
        x.start(0)
        x.start(1)
        x.wait(0)
        x.wait(1)
        for slot in (0, 1):
            check(x, mode, slot)
            assert x.verify(slot)
        x.drain()


def _case_stripe_gather(ctx):
    """StripeGather: every rank's column piece of each slot's rows lands in rank 0's full rows; rank
    0's own piece is computed in place (a view of its full rows) and never moves."""
    from gpu_rscode_amd.parallel.placement import StripeGather

    ncols, rows, slots = 3 * 4096 + 77, 3, 2
    widths = [b - a for a, b in (pdist.shard_range(ncols, ctx.world, r) for r in range(ctx.world))]
    a, b = pdist.shard_range(ncols, ctx.world, ctx.rank)

    def content(slot):
        return (torch.arange(rows * ncols, dtype=torch.int64).view(rows, ncols) * 3 + 17 * slot).remainder(251).to(
            torch.uint8)

    fulls = None
    if ctx.rank == 0:
        full_t = [torch.zeros((rows, ncols), dtype=torch.uint8) for _ in range(slots)]
        fulls = [[f[i] for i in range(rows)] for f in full_t]
        pieces_t = [f[:, : b - a] for f in full_t]
    else:
        pieces_t = [torch.zeros((rows, b - a), dtype=torch.uint8) for _ in range(slots)]
    for s in range(slots):
        pieces_t[s].copy_(content(s)[:, a:b])
    g = StripeGather([[p[i] for i in range(rows)] for p in pieces_t], fulls, widths)
    g.start(0)
    g.start(1)
    g.wait(0)
    g.wait(1)
    for s in range(slots):
        assert g.verify(s)
        if ctx.rank == 0:
            assert torch.equal(full_t[s], content(s))
    if ctx.rank == 0:
        assert g.bytes_received == rows * (ncols - widths[0])


def _case_scatter_odd_c_alignment(ctx):
    """An odd C in a plain contiguous [k, C] tensor: row i starts at i*C, so rank 0's shard cannot be
    a view — it gets a pitched, 16-byte aligned copy like every other rank."""
    C = 2 * 4096 + 4095
    full = torch.arange(4 * C, dtype=torch.int64).remainder(253).to(torch.uint8).view(4, C)
    shard = pdist.scatter_columns(full if ctx.rank == 0 else None, 4, C, ctx.device)
    a, b = pdist.shard_range(C, ctx.world, ctx.rank)
    assert torch.equal(shard, full[:, a:b])
    assert all(shard[i].data_ptr() % 16 == 0 for i in range(4))
    if ctx.rank == 0:
        assert shard.data_ptr() != full.data_ptr()


@pytest.mark.parametrize("case", ["_case_broadcast", "_case_scatter_gather", "_case_distributed_codec",
                                  "_case_parity_exchange", "_case_stripe_gather", "_case_scatter_odd_c_alignment"])
def test_distributed_world2(case):
    _run(case, 2)


def test_distributed_codec_world3():
    _run("_case_distributed_codec", 3)


def test_distributed_codec_gf65536_world3():
    _run("_case_distributed_codec16", 3)


def _case_broadcast_wide(ctx):
    ids = np.array([[0, 255, 256, 4095, 65534]]) if ctx.rank == 0 else None
    got = pdist.broadcast_matrix(ids, ctx.device, dtype=np.int32)
    assert got.dtype == np.int32 and got.tolist() == [[0, 255, 256, 4095, 65534]]


def test_broadcast_int32_world2():
    _run("_case_broadcast_wide", 2)


def test_parity_exchange_world3():
    _run("_case_parity_exchange", 3)


def test_stripe_gather_world3():
    _run("_case_stripe_gather", 3)


def _forced_worker(rank, fn_name):
    for v in ("MASTER_PORT", "WORLD_SIZE", "RANK", "LOCAL_RANK"):
        os.environ.pop(v, None)
    ctx = pdist.init_distributed(backend="gloo", force_pg=True)
    assert dist.is_initialized() and dist.get_world_size() == 1
    try:
        globals()[fn_name](ctx)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case", ["_case_broadcast", "_case_distributed_codec", "_case_parity_exchange",
                                  "_case_stripe_gather"])
def test_forced_one_rank_group(case):
    """--force-pg: a one-rank process group runs the same collectives against itself."""
    mp.spawn(_forced_worker, args=(case,), nprocs=1, join=True)
